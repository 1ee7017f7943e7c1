"""The flat scene descriptor (include/rtamd.h rt_scene_desc), host side (no GPU).

A caller that already holds the reference's Scene (scene.h:35-38) hands it over as
rt_scene_desc; rt_scene_create_desc must then upload exactly what parsing the same scene
from its files uploads.  rt_debug_builder_digest hashes the flattened upload (geometry,
LBVHs, materials, lights, camera) on the host, so the equality is checked here without a
GPU; the GPU tests render both routes (test_gpu_api.py).
"""
import ctypes
import os
import subprocess

import pytest

from cases import REPO, SCENES, scene_files


def _parsed(rt, scene):
    s = rt.Scene(diag=True)  # digest(): a hook of librtamd_diag.so
    try:
        rt.RTIParser(s).parseFile(os.path.join(SCENES, scene))
    except rt.RTError:
        s.close()
        return None
    return s


@pytest.mark.parametrize("scene", scene_files())
def test_descriptor_round_trip_uploads_the_same_scene(rt, scene):
    """rt_builder_get_desc -> rt_builder_set_desc: identical flattened upload."""
    s = _parsed(rt, scene)
    if s is None:
        pytest.skip("scene rejected by the reference")
    d = s.desc()
    s2 = rt.Scene(diag=True)
    s2.set_desc(d)
    assert s2.digest() == s.digest()
    assert s2.hasCamera() == s.hasCamera()
    s.close()
    s2.close()


@pytest.mark.parametrize("scene", ["excess_inputs/bunny.rti", "inputs/input-08.rti", "inputs/input-09.rti",
                                   "excess_inputs/minicooper_sub.rti"])
def test_descriptor_derived_inverse_matches_parser(rt, scene):
    """xf.derive = 1: the inverse and determinant computed from fwd alone are the bits the
    reference's Transformable::forwardTransform(xf) stores (rtbase.h:51-54)."""
    s = _parsed(rt, scene)
    d = s.desc()
    for k in range(d.n_geometries):
        g = d.geometries[k]
        g.xf.derive = 1
        for i in range(16):
            g.xf.inv[i] = float("nan")
        g.xf.det = float("nan")
    s2 = rt.Scene(diag=True)
    s2.set_desc(d)
    assert s2.digest() == s.digest()
    s.close()
    s2.close()


def test_descriptor_errors(rt):
    s = _parsed(rt, "inputs/input-02.rti")
    d = s.desc()
    mesh = next(k for k in range(d.n_geometries) if d.geometries[k].kind == rt.RT_GEOM_MESH)
    g = d.geometries[mesh]
    # a face point that is not a homogeneous point (Mesh::updateBoundingBox invariant)
    old = g.faces[0].points[1][3]
    g.faces[0].points[1][3] = 2.0
    with pytest.raises(rt.ArgumentError, match="w != 1"):
        rt.Scene().set_desc(d)
    g.faces[0].points[1][3] = old
    old_kind = g.kind
    g.kind = 7
    with pytest.raises(rt.ArgumentError, match="unknown kind"):
        rt.Scene().set_desc(d)
    g.kind = old_kind
    faces = ctypes.cast(g.faces, ctypes.c_void_p).value  # (a field read shares the struct's memory)
    g.faces = ctypes.POINTER(rt.rt_face_desc)()
    with pytest.raises(rt.ArgumentError, match="bad face array"):
        rt.Scene().set_desc(d)
    g.faces = ctypes.cast(faces, ctypes.POINTER(rt.rt_face_desc))
    d.lights[0].kind = 9
    with pytest.raises(rt.ArgumentError, match="unknown kind"):
        rt.Scene().set_desc(d)
    s.close()


def test_descriptor_without_camera_is_rejected_at_upload(rt):
    d = rt.rt_scene_desc()
    s = rt.Scene()
    s.set_desc(d)
    assert not s.hasCamera()
    with pytest.raises(rt.RTError, match="At least one camera"):
        rt.Scene.from_desc(d)
    s.close()


def test_native_descriptor_from_memory_matches_file_route(tmp_path):
    """tests/native/desc_check.cpp: a C++ caller fills rt_scene_desc from an in-memory scene
    (reference construction rules, no file) and gets the device scene of the equivalent
    .rti/.obj files."""
    exe = tmp_path / "desc_check"
    lib = os.path.join(REPO, "cs184-raytracer_amd", "rtamd")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(REPO, "tests", "native", "desc_check.cpp"), "-L" + lib, "-lrtamd_diag",
                    "-Wl,-rpath," + lib], check=True)
    p = subprocess.run([str(exe), str(tmp_path), "digest"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
