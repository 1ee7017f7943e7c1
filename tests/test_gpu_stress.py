"""Numerical stress scenes for the conservative parts of the HIP path (gpu).

The kernels prune with fp32 node boxes and fp64 world boxes ("Exact
closest hit under a BVH"): they may skip only work whose outcome is already decided.
These scenes put that argument under pressure -- meshes far from the object-space
origin, tiny and huge scales, a camera far away, grazing rays along a mesh, dense
triangle soups with many near-coincident faces, mirrors and glass sending deep
secondary rays -- and require the image and ray counters to equal the CPU oracle's
(itself pinned bit for bit to the unmodified reference, test_oracle.py).  The scenes are
generated deterministically (seeded numpy) into a temporary directory.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIGHTS = """ltp   10 10 10 0.2 0.3 0.5
ltd   50 50 -20 0.1 0.2 0.5
ltp   -1 1 1 0.3 0.25 0.0
lta   1 1 1
"""
MAT_SHINY = "mat   0.0 0.025 0.05   0.6 0.6 0.6   0.8 0.8 0.8 1.0   0.4 0.4 0.4\n"
MAT_MIRROR = "mat   0 0 0   0.4 0.4 0.4   1.0 0.6 0.6 2.0  1 1 1\n"
MAT_GLASS = "mat   0 0 0   0.1 0.1 0.1   0.5 0.5 0.5 8.0  0.1 0.1 0.1  0.9 0.9 0.9 1.5\n"


def write_soup(path, n, center, extent, seed, thin=False):
    """A triangle soup of n faces around `center` (object-space coordinates), with vertex
    normals; `thin` makes slivers (near-degenerate faces)."""
    rng = np.random.default_rng(seed)
    lines = []
    for i in range(n):
        c = np.asarray(center, dtype=np.float64) + rng.uniform(-extent, extent, 3)
        e = extent * 0.3
        a = c + rng.uniform(-e, e, 3)
        b = c + rng.uniform(-e, e, 3)
        d = (a + b) / 2 + rng.uniform(-e, e, 3) * (1e-4 if thin else 1.0)
        for v in (a, b, d):
            lines.append("v %.17g %.17g %.17g" % tuple(v))
        nrm = rng.normal(size=3)
        lines.append("vn %.17g %.17g %.17g" % tuple(nrm / np.linalg.norm(nrm)))
    for i in range(n):
        k = 3 * i
        lines.append("f %d//%d %d//%d %d//%d" % (k + 1, i + 1, k + 2, i + 1, k + 3, i + 1))
    path.write_text("\n".join(lines) + "\n")


def scene(tmp_path, name, body):
    f = tmp_path / (name + ".rti")
    f.write_text(body)
    return str(f)


def check(gpu, oracle, path, w=40, h=30, bdepth=3, bits=False):
    want, cnt = oracle.render(path, w, h, bdepth=bdepth)
    s = gpu.load_scene(path)
    got = s.renderScene(options=gpu.Options(renderWidth_=w, renderHeight_=h, bounceDepth_=bdepth))
    st = s.last_stats
    s.close()
    if bits:  # binary64 bit patterns: NaN payloads and the sign of zero count too
        got, want = np.ascontiguousarray(got).view(np.uint64), np.ascontiguousarray(want).view(np.uint64)
    diff = int((got != want).any(axis=2).sum())
    assert diff == 0, f"{diff} pixels differ from the oracle"
    assert (st.trace_rays, st.shadow_rays) == (cnt["trace_rays"], cnt["shadow_rays"])
    return st


@pytest.mark.parametrize("offset", [0.0, 1e3, 1e5])
def test_mesh_far_from_object_origin(gpu, oracle, tmp_path, offset):
    """Vertices around (offset, offset, offset), brought back by the geometry's transform:
    the fp32 node test must stay conservative when |vertex| >> the mesh's extent."""
    write_soup(tmp_path / "soup.obj", 500, (offset, offset, offset), 1.0, seed=1)
    body = ("cam   0 0 6   -1.5 -1.1 2    1.5 -1.1 2   -1.5 1.1 2   1.5 1.1 2\n" + LIGHTS +
            f"xft   {-offset} {-offset} {-offset}\n" + MAT_SHINY + 'obj   "soup.obj"\nxfz\n' + MAT_MIRROR +
            "sph   1.6 0.2 -1.0 0.6\n")
    check(gpu, oracle, scene(tmp_path, "far", body))


# (1e-6 is too small: the reference parser drops faces whose cross product is within Eigen's
# isZero tolerance as degenerate, parsers.cpp:336)
@pytest.mark.parametrize("scale", [1e-3, 1e6])
def test_tiny_and_huge_scales(gpu, oracle, tmp_path, scale):
    write_soup(tmp_path / "soup.obj", 500, (0, 0, 0), scale, seed=2)
    body = ("cam   0 0 6   -1.5 -1.1 2    1.5 -1.1 2   -1.5 1.1 2   1.5 1.1 2\n" + LIGHTS +
            f"xfs   {1.0 / scale} {1.0 / scale} {1.0 / scale}\n" + MAT_SHINY + 'obj   "soup.obj"\n')
    check(gpu, oracle, scene(tmp_path, "scale", body))


def test_far_camera_and_slivers(gpu, oracle, tmp_path):
    """A camera 1e4 away with a narrow field of view on a soup of slivers (near-degenerate
    faces, determinants close to zero) plus a mirror sphere behind it."""
    write_soup(tmp_path / "soup.obj", 400, (0, 0, 0), 1.0, seed=3, thin=True)
    body = ("cam   0 0 10000   -0.0002 -0.00015 9999    0.0002 -0.00015 9999   -0.0002 0.00015 9999   "
            "0.0002 0.00015 9999\n" + LIGHTS + MAT_SHINY + 'obj   "soup.obj"\n' + MAT_MIRROR +
            "sph   0 0 -3 1.5\n")
    check(gpu, oracle, scene(tmp_path, "farcam", body))


def test_grazing_rays_and_glass(gpu, oracle, tmp_path):
    """The camera looks along a flat dense mesh (rays nearly parallel to its faces) through
    a glass sphere: grazing slabs, refraction and total internal reflection."""
    rng = np.random.default_rng(4)
    lines, faces = [], []
    n = 24
    for i in range(n + 1):
        for j in range(n + 1):
            lines.append("v %.17g %.17g %.17g" % (-2 + 4 * i / n, -0.5 + rng.uniform(-1e-3, 1e-3), -4 + 4 * j / n))
    for i in range(n):
        for j in range(n):
            a, b, c, d = i * (n + 1) + j + 1, (i + 1) * (n + 1) + j + 1, (i + 1) * (n + 1) + j + 2, i * (n + 1) + j + 2
            faces += ["f %d %d %d" % (a, b, c), "f %d %d %d" % (a, c, d)]
    (tmp_path / "grid.obj").write_text("\n".join(lines + faces) + "\n")
    body = ("cam   0 -0.45 3   -1 -0.52 2    1 -0.52 2   -1 0.2 2   1 0.2 2\n" + LIGHTS + MAT_MIRROR +
            'obj   "grid.obj"\n' + MAT_GLASS + "sph   0 0 0.5 0.5\n")
    check(gpu, oracle, scene(tmp_path, "grazing", body), bdepth=6)


KD, KS = "0.5 0.6 0.7", "0.8 0.7 0.6"


@pytest.mark.parametrize("kd,ks,ns", [(KD, KS, 0.0), (KD, KS, 0.5), (KD, KS, 1.0), (KD, KS, 3.0), ("0 0 0", KS, 2.0),
                                      (KD, "0 0 0", 1.0), (KD, "0 0 0", 0.0), ("0 0 0", "0 0 0", 5.0),
                                      (KD, "0 0 0", -1.0)])
def test_zero_phong_terms_lights_behind(gpu, oracle, tmp_path, kd, ks, ns):
    """Shadow rays whose diffuse and specular additions are certain exact zeros are not
    traced (k_shadow, DMaterial/DLight::zero_terms).  Exercised with ns = 0 (pow(0, 0) = 1:
    the specular term is not zero), fractional, integer and negative exponents, zero kd or
    ks, point lights with and without falloff and a directional light, placed so that many
    hits face away from them.  Compared bit for bit (NaN and -0 included)."""
    write_soup(tmp_path / "soup.obj", 300, (0, 0, 0), 1.0, seed=7)
    mat = f"mat   0.01 0.02 0.03   {kd}   {ks} {ns}   0.3 0.3 0.3\n"  # every geometry's
    body = ("cam   0 0 6   -1.5 -1.1 2    1.5 -1.1 2   -1.5 1.1 2   1.5 1.1 2\n"
            "ltp   0 0 -8 0.3 0.3 0.3\n"          # behind everything, no falloff
            "ltp   2 -3 -2 0.4 0.2 0.1 1.5\n"     # behind, with falloff
            "ltd   0.2 -0.3 -1 0.2 0.2 0.2\n"     # directional, pointing towards the camera
            "ltp   -3 3 4 0.2 0.3 0.4\n"          # in front
            "lta   0.1 0.1 0.1\n" + mat + 'obj   "soup.obj"\n' +
            "sph   1.6 0.2 -1.0 0.6\n" + "tri   -4 -1.2 4   4 -1.2 4   4 -1.2 -4\n")
    st = check(gpu, oracle, scene(tmp_path, "behind", body), w=48, h=36, bdepth=3, bits=True)
    assert (st.shadow_rays_zero_terms > 0) == (ns > 0)


def write_normal_soup(path, n, seed, mode):
    """Triangle soup with per-vertex normals for the facing pre-test (intersect.h
    face_facing_rejects): 'spread' three unrelated normals per face (wide cones), 'grazing'
    one normal nearly perpendicular to the view axis with 1e-7 per-vertex jitter (narrow
    cones whose facing sign flips across the image), 'scaled' normals of magnitudes 1e-9 to
    1e3 (faces whose pre-test is disabled) and 'flipped' vertex normals opposite to each
    other (interpolated normal through zero)."""
    rng = np.random.default_rng(seed)
    v, vn, f = [], [], []
    for i in range(n):
        c = rng.uniform(-1.2, 1.2, 3) * np.array([1.0, 0.8, 0.5])
        pts = [c + rng.uniform(-0.25, 0.25, 3) for _ in range(3)]
        if mode == "spread":
            ns = [rng.normal(size=3) for _ in range(3)]
        elif mode == "grazing":
            base = np.array([rng.normal(), rng.normal(), rng.uniform(-1e-3, 1e-3)])
            ns = [base + rng.normal(size=3) * 1e-7 for _ in range(3)]
        elif mode == "scaled":
            base = rng.normal(size=3)
            ns = [base * s for s in rng.choice([1e-9, 1e-3, 1.0, 1e3], 3)]
        else:  # flipped
            base = rng.normal(size=3)
            ns = [base, -base, base * rng.uniform(0.5, 2.0)]
        for p, q in zip(pts, ns):
            v.append("v %.17g %.17g %.17g" % tuple(p))
            vn.append("vn %.17g %.17g %.17g" % tuple(q))
        k = 3 * i
        f.append("f %d//%d %d//%d %d//%d" % (k + 1, k + 1, k + 2, k + 2, k + 3, k + 3))
    path.write_text("\n".join(v + vn + f) + "\n")


@pytest.mark.parametrize("mode", ["spread", "grazing", "scaled", "flipped"])
def test_facing_pretest_vertex_normals(gpu, oracle, tmp_path, mode):
    """Faces are skipped before their fp64 Cramer test when the facing test certainly fails
    (normal cones): bit-exact on meshes whose vertex normals differ, sit near
    the facing boundary, have wildly different magnitudes or cancel -- camera rays, shadow
    rays from both sides, mirror and glass secondary rays."""
    write_normal_soup(tmp_path / "nsoup.obj", 400, seed=7, mode=mode)
    body = ("cam   0 0 6   -1.5 -1.1 2    1.5 -1.1 2   -1.5 1.1 2   1.5 1.1 2\n" + LIGHTS +
            "ltp   0 0 -5 0.3 0.3 0.3\n" + MAT_SHINY + 'obj   "nsoup.obj"\n' + MAT_GLASS +
            "sph   0.3 -0.2 1.5 0.5\n" + MAT_MIRROR + "sph   -1.6 0.9 -1.5 0.7\n")
    check(gpu, oracle, scene(tmp_path, "nsoup_" + mode, body), w=64, h=48, bdepth=4, bits=True)


CAM6 = "cam 0 0 6  -2 -2 2  2 -2 2  -2 2 2  2 2 2"


@pytest.mark.parametrize("xf,cam", [
    ("xfs 3 0.2 1\nxfr 30 45 10", CAM6), ("xfr 0 0 37\nxfs 0.05 4 0.5", CAM6),
    ("xfr 80 0.1 0\nxfs 1 1 1e-3", CAM6), ("xfr 60 20 0\nxfs 1 1 0.02", CAM6),
    ("xft 1e4 -2e4 3e4\nxfs 2 2 2", "cam 1e4 -2e4 3.0008e4  9996 -20004 3.0004e4  10004 -20004 3.0004e4  9996 -19996 3.0004e4  "
                                    "10004 -19996 3.0004e4"),
    ("xfs 1e-3 1e-3 1e-3", "cam 0 0 0.006  -0.002 -0.002 0.002  0.002 -0.002 0.002  -0.002 0.002 0.002  0.002 0.002 0.002")])
def test_sphere_bounding_cull_silhouettes(gpu, oracle, tmp_path, xf, cam):
    """The bounding-sphere cull of sphere geometries (intersect.h sphere_cull, round 3) may
    skip a sphere only when the exact ray cannot reach it.  Ellipsoids under anisotropic
    scales and rotations (flattened to discs), far translations and tiny scales, framed so
    that many primary, mirror and shadow rays graze their silhouettes, must render bit for
    bit as the oracle (rows of mirror and glass spheres reflecting each other)."""
    rows = [f"sph {1.5 * i - 1.5:.3f} {1.5 * j - 1.5:.3f} 0 0.7" for i in range(3) for j in range(3)]
    body = cam + "\n" + LIGHTS + xf + "\n" + MAT_MIRROR + "\n".join(rows[:5]) + "\n" + MAT_GLASS + "\n".join(rows[5:]) + "\n"
    check(gpu, oracle, scene(tmp_path, "ellipsoids", body), w=96, h=72, bdepth=4, bits=True)
