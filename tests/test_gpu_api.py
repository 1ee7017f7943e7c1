"""GPU tests of the C-ABI entry points added around the render path (round 2).

- rt_scene_create_desc: a scene handed over as rt_scene_desc (the caller's own Scene,
  scene.h:35-38) renders bit-exactly like the parsed files (reference goldens);
- rt_render_rgb8: RGB8 quantised on the device equals convertToRGBImage of the f64 image;
- progress: reported from the calling thread, monotone, ending at the total (scene.cpp:41-44);
- any number of lights (scene.cpp:77-108 has no limit);
- a render that fails midway leaves nothing behind: the next render is exact;
- --intersection-only with an RGB8-only output is normalised by the global maximum.
Every image is compared bit for bit with the reference's goldens or the pinned oracle.
"""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from cases import OPTION_SETS, REPO, SCENES, SCHEDULES, apply_schedule, option_kwargs, scene_files

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("scene", scene_files())
def test_descriptor_scene_matches_reference(gpu, golden, scene):
    """rt_builder_get_desc -> rt_scene_create_desc -> render == the reference's image."""
    name, w, h, flags = OPTION_SETS[0]
    ref = golden["cases"][f"{scene}|{name}"]
    if ref["rc"] != 0:
        pytest.skip("scene rejected by the reference")
    src = gpu.load_scene(os.path.join(SCENES, scene))
    s = gpu.Scene.from_desc(src.desc())
    kw = option_kwargs(flags)
    o = gpu.Options(renderWidth_=w, renderHeight_=h, bounceDepth_=kw["bdepth"], intersectionOnly_=kw["intersection_only"])
    img = s.renderScene(options=o)
    assert sha(img) == ref["f64_sha256"]
    s.close()
    src.close()


def test_native_descriptor_render(gpu, oracle, tmp_path):
    """tests/native/desc_check.cpp on the GPU: the in-memory descriptor and the equivalent
    files render identical f64 and RGB8 images, and both equal the oracle's render."""
    exe = tmp_path / "desc_check"
    lib = os.path.join(REPO, "cs184-raytracer_amd", "rtamd")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(REPO, "tests", "native", "desc_check.cpp"), "-L" + lib, "-lrtamd_diag",
                    "-Wl,-rpath," + lib], check=True)
    p = subprocess.run([str(exe), str(tmp_path), "render"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    got = np.fromfile(tmp_path / "desc.raw", dtype=np.float64).reshape(90, 160, 3)
    want, _ = oracle.render(str(tmp_path / "scene.rti"), 160, 90, bdepth=5)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


@pytest.mark.parametrize("scene,bdepth,io", [("excess_inputs/bunny.rti", 4, False), ("inputs/input-09.rti", 10, False),
                                             ("inputs/input-02.rti", 0, True)])
def test_render_rgb8_host(gpu, scene, bdepth, io):
    """rt_render_rgb8 == convertToRGBImage(rt_render) (writers.cpp:4-9), --intersection-only
    normalised by the global maximum first (scene.cpp:50-58)."""
    s = gpu.load_scene(os.path.join(SCENES, scene))
    o = gpu.Options(renderWidth_=83, renderHeight_=47, bounceDepth_=bdepth, intersectionOnly_=io)
    img = s.renderScene(options=o)
    rgb = s.render_rgb8(options=o)
    assert np.array_equal(rgb, gpu.to_rgb8(img))
    if not io:
        part = s.render_rgb8(options=o, rows=(1, 47, 3))
        assert np.array_equal(part, rgb[1::3])
    s.close()


def test_intersection_only_rgb8_device_output(gpu):
    """rt_render_device with --intersection-only and only an RGB8 output: normalised from a
    staging f64 image (it used to return without writing the bytes)."""
    torch = pytest.importorskip("torch")
    scene = "inputs/input-03.rti"
    s = gpu.load_scene(os.path.join(SCENES, scene))
    o = gpu.Options(renderWidth_=64, renderHeight_=40, intersectionOnly_=True)
    img = s.renderScene(options=o)
    out8 = torch.zeros((40, 64, 3), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    s.render_device(s.params(64, 40, 10, True), 0, out8.data_ptr())
    assert np.array_equal(out8.cpu().numpy(), gpu.to_rgb8(img))
    with pytest.raises(gpu.ArgumentError):
        s.render_device(s.params(64, 40, 10, True, 0, 40, 2), 0, out8.data_ptr())
    s.close()


def test_progress_is_incremental_and_complete(gpu):
    """Progress from the calling thread: starts at 0, never decreases, ends at the total."""
    scene = "excess_inputs/refraction3.rti"
    s = gpu.load_scene(os.path.join(SCENES, scene))
    calls = []
    o = gpu.Options(renderWidth_=512, renderHeight_=512, bounceDepth_=8)
    img = s.renderScene(options=o, phandler=lambda c, t: calls.append((c, t)), chunk_pixels=16384)
    total = 512 * 512
    assert calls[0] == (0, total) and calls[-1] == (total, total)
    assert all(t == total for _, t in calls)
    assert all(a[0] <= b[0] for a, b in zip(calls, calls[1:]))
    rgb = s.render_rgb8(options=o, phandler=lambda c, t: calls.append((c, t)))
    assert np.array_equal(rgb, gpu.to_rgb8(img))
    s.close()


def test_many_lights(gpu, oracle, tmp_path):
    """70 point lights (+ ambient): more than the fused shading's 64-bit verdict mask; the
    light-major layout and k_shade take them (scene.cpp:77-108 loops over any number)."""
    lines = ["cam 0 0 6  -1.6 -0.9 2  1.6 -0.9 2  -1.6 0.9 2  1.6 0.9 2"]
    rng = np.random.default_rng(5)
    for k in range(70):
        x, y, z = rng.uniform(-6, 6, 3)
        lines.append(f"ltp {x:.6f} {y:.6f} {z + 6:.6f}  {0.01 * (k % 7):.3f} 0.012 0.015")
    lines += ["lta 0.1 0.1 0.1", "mat 0.1 0.1 0.1 0.5 0.5 0.5 0.4 0.4 0.4 8 0.3 0.3 0.3",
              "sph 0 0 0 1", "sph 1.5 0.3 -1 0.6",
              "xft 0.17 -1.1 0", "xfs 10 10 10", f'obj "{os.path.join(SCENES, "excess_inputs", "bunny.obj")}"', "xfz",
              "tri -10 -1.2 10  10 -1.2 10  10 -1.2 -10"]
    f = tmp_path / "lights70.rti"
    f.write_text("\n".join(lines) + "\n")
    want, cnt = oracle.render(str(f), 64, 40, bdepth=3)
    s = gpu.load_scene(str(f))
    img = s.renderScene(options=gpu.Options(renderWidth_=64, renderHeight_=40, bounceDepth_=3))
    assert np.array_equal(img.view(np.uint64), want.view(np.uint64))
    assert (s.last_stats.trace_rays, s.last_stats.shadow_rays) == (cnt["trace_rays"], cnt["shadow_rays"])
    s.close()


@pytest.mark.parametrize("after,replay", [(0, True), (0, False), (1, False), (3, False)])
def test_render_after_a_failed_render_is_exact(gpu, oracle, after, replay):
    """A device failure in the middle of a render (injected after `after` closest-hit
    launches; a replayed plan counts as one) returns an error; the scene's next render is
    complete, bit-exact and counts exactly its own rays (no stale lane, counter or error word).
    replay: the failing render replays a launch plan; else it is the first of its shape
    (host-driven, level by level)."""
    scene = "excess_inputs/bunny.rti"
    w, h, bdepth = 80, 45, 4
    want, cnt = oracle.render(os.path.join(SCENES, scene), w, h, bdepth=bdepth)
    s = gpu.load_scene(os.path.join(SCENES, scene), diag=True)
    o = gpu.Options(renderWidth_=w, renderHeight_=h, bounceDepth_=bdepth)
    # lanes and level buffers exist; with replay, a plan of this shape too
    s.renderScene(options=o if replay else gpu.Options(renderWidth_=w + 8, renderHeight_=h, bounceDepth_=bdepth))
    s.debug_fail_after(after)
    with pytest.raises(gpu.DeviceError, match="injected"):
        s.renderScene(options=o)
    img = s.renderScene(options=o)
    assert np.array_equal(img.view(np.uint64), want.view(np.uint64))
    assert (s.last_stats.trace_rays, s.last_stats.shadow_rays) == (cnt["trace_rays"], cnt["shadow_rays"])
    s.close()


@pytest.mark.parametrize("replay", [True, False])
def test_corrupt_row_descriptor_is_reported_not_written(gpu, oracle, replay):
    """The kernels compute every row and output address from by-value descriptors and check
    them (trace.hip chunk_row): descriptors naming rows the frame does not have (injected,
    librtamd_diag.so) fail the render with the named device error, write no pixel, and the
    scene's next render is exact."""
    torch = pytest.importorskip("torch")
    scene = os.path.join(SCENES, "excess_inputs/bunny.rti")
    w, h, bdepth = 64, 40, 4
    want, _ = oracle.render(scene, w, h, bdepth=bdepth)
    s = gpu.load_scene(scene, diag=True)
    prm = s.params(w, h, bdepth, False)
    out = torch.full((h, w, 3), -7.0, dtype=torch.float64, device="cuda")
    if replay:  # a launch plan of this shape exists: the bad chunk replays it on the caller's stream
        s.render_device(prm, out.data_ptr())
        out.fill_(-7.0)
    s.debug_corrupt_rows()
    with pytest.raises(gpu.DeviceError, match="row descriptor names no selected row"):
        s.render_device(prm, out.data_ptr())
    # segment 0's rows moved past the image: nothing written
    assert bool((out == -7.0).all())
    s.render_device(prm, out.data_ptr())
    assert np.array_equal(out.cpu().numpy().view(np.uint64), want.view(np.uint64))
    s.close()


def test_right_sized_levels_then_replay_on_a_torch_stream(gpu, oracle):
    """a call traced host-driven grows the level buffers and cuts them back after it
    (right_size_levels, record copies on the lane's stream); the next call of that shape replays
    its plan on the caller's stream.  The record copies complete before the first call returns,
    so the replay on a torch stream reads the new records: exact, three times."""
    torch = pytest.importorskip("torch")
    scene = os.path.join(SCENES, "excess_inputs/bunny.rti")
    w, h, bdepth = 480, 270, 4
    want, _ = oracle.render(scene, w, h, bdepth=bdepth)
    s = gpu.load_scene(scene)
    prm = s.params(w, h, bdepth, False)
    st = torch.cuda.Stream()
    out = torch.empty((h, w, 3), dtype=torch.float64, device="cuda")
    s.renderScene(options=gpu.Options(renderWidth_=w, renderHeight_=h, bounceDepth_=bdepth))  # minimal lane
    for _ in range(3):
        with torch.cuda.stream(st):
            out.fill_(0.0)
            s.render_device(prm, out.data_ptr(), 0, st.cuda_stream)
        st.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint64), want.view(np.uint64))
    assert s.info().level_bytes <= s.info().level_bytes_peak
    s.close()


def test_chunks_of_many_row_segments(gpu, oracle, monkeypatch):
    """More jobs of a few rows than one chunk's by-value descriptors hold (kMaxRowSegments):
    the chunks are cut at 32 segments, and every job's rows land in its own buffer, exact."""
    torch = pytest.importorskip("torch")
    scene = os.path.join(SCENES, "inputs/input-06.rti")
    w, h, bdepth = 48, 80, 3
    want, _ = oracle.render(scene, w, h, bdepth=bdepth)
    s = gpu.load_scene(scene)
    ways = 10  # 10 ranks' 8-row blocks of 8 frames: 80 jobs of 8 rows
    jobs, rows = [], []
    for f in range(8):
        for k in range(ways):
            jobs.append(s.params(w, h, bdepth, False, ((k + f) % ways) * 8, h, ways, row_block=8))
            rows.append([r for r in range(h) if (r // 8) % ways == (k + f) % ways])
    outs = [torch.full((len(r), w, 3), -1.0, dtype=torch.float64, device="cuda") for r in rows]
    for _ in range(2):  # host-driven, then replayed plans
        s.render_batch_device(jobs, [o.data_ptr() for o in outs], [0] * len(jobs))
        for o, r in zip(outs, rows):
            assert np.array_equal(o.cpu().numpy().view(np.uint64), np.ascontiguousarray(want[r]).view(np.uint64))
    s.close()


@pytest.mark.parametrize("scene", ["excess_inputs/bunny.rti", "inputs/input-06.rti"])
def test_fused_multi_level_shadow_batches(gpu, oracle, scene, monkeypatch):
    """All-lights shadow layout for the deep levels too (SHADOW_ALL_LIGHTS 3), packets for
    every level (PACKET_MASK 63) and one direct level, so deep levels are shaded in
    multi-level batches with the fused Phong terms."""
    w, h, bdepth = 72, 40, 6
    want, cnt = oracle.render(os.path.join(SCENES, scene), w, h, bdepth=bdepth)
    for k, v in (("RTAMD_SHADOW_ALL_LIGHTS", "3"), ("RTAMD_PACKET_MASK", "63"), ("RTAMD_DIRECT_LEVELS", "1"),
                 ("RTAMD_LIGHT_MAJOR_BELOW", "0")):
        monkeypatch.setenv(k, v)
    s = gpu.load_scene(os.path.join(SCENES, scene))
    img = s.renderScene(options=gpu.Options(renderWidth_=w, renderHeight_=h, bounceDepth_=bdepth))
    assert np.array_equal(img.view(np.uint64), want.view(np.uint64))
    assert (s.last_stats.trace_rays, s.last_stats.shadow_rays) == (cnt["trace_rays"], cnt["shadow_rays"])
    s.close()


def test_camera_eye_direction_vector_raises(gpu):
    """A camera eye with w == 0 (only possible through the descriptor) throws the Ray
    origin check's MathException (rtbase.h:13-14)."""
    src = gpu.load_scene(os.path.join(SCENES, "inputs/input-01.rti"))
    d = src.desc()
    d.camera.eye[3] = 0.0
    s = gpu.Scene.from_desc(d)
    with pytest.raises(gpu.MathException, match="ray origin is a direction vector"):
        s.renderScene(options=gpu.Options(renderWidth_=8, renderHeight_=8))
    s.close()
    src.close()


@pytest.mark.parametrize("scene,bdepth,chunk", [("excess_inputs/bunny.rti", 4, 0), ("excess_inputs/refraction3.rti", 8, 0),
                                                ("excess_inputs/refraction3.rti", 8, 900), ("inputs/input-06.rti", 10, 0),
                                                ("inputs/input-09.rti", 10, 1500)])
@pytest.mark.parametrize("schedule", SCHEDULES)
def test_replayed_plans_are_exact(gpu, oracle, scene, bdepth, chunk, schedule, monkeypatch):
    """Launch plans (the launch sequence of a traced chunk shape issued at once, device-read
    level sizes): the 2nd and 3rd renders of the same shape replay the plan, in level buffers
    cut back to the plan's ray counts; every render is bit-exact with the oracle and counts
    the reference's rays."""
    apply_schedule(monkeypatch, schedule)
    w, h = 90, 50
    want, cnt = oracle.render(os.path.join(SCENES, scene), w, h, bdepth=bdepth)
    s = gpu.load_scene(os.path.join(SCENES, scene))
    o = gpu.Options(renderWidth_=w, renderHeight_=h, bounceDepth_=bdepth)
    for _ in range(3):
        img = s.renderScene(options=o, chunk_pixels=chunk)
        assert np.array_equal(img.view(np.uint64), want.view(np.uint64))
        assert (s.last_stats.trace_rays, s.last_stats.shadow_rays) == (cnt["trace_rays"], cnt["shadow_rays"])
        assert (s.last_stats.reflect_rays, s.last_stats.refract_rays) == (cnt["reflect_rays"], cnt["refract_rays"])
    s.close()


def test_replayed_plan_batch_and_rgb8(gpu):
    """A batch of frames over three lanes (each lane builds, then replays, its plan) with
    f64 and RGB8 outputs."""
    torch = pytest.importorskip("torch")
    scene = "excess_inputs/bunny.rti"
    s = gpu.load_scene(os.path.join(SCENES, scene))
    w, h = 96, 54
    ref = s.renderScene(options=gpu.Options(renderWidth_=w, renderHeight_=h, bounceDepth_=4))
    prm = s.params(w, h, 4, False)
    for _ in range(3):
        outs = [torch.full((h, w, 3), -1.0, dtype=torch.float64, device="cuda") for _ in range(7)]
        out8 = [torch.zeros((h, w, 3), dtype=torch.uint8, device="cuda") for _ in range(7)]
        torch.cuda.synchronize()
        s.render_batch_device([prm] * 7, [o.data_ptr() for o in outs], [o.data_ptr() for o in out8])
        for k in range(7):
            assert np.array_equal(outs[k].cpu().numpy(), ref), k
            assert np.array_equal(out8[k].cpu().numpy(), gpu.to_rgb8(ref)), k
    s.close()


@pytest.mark.parametrize("schedule", SCHEDULES)
@pytest.mark.parametrize("scene,bdepth,io", [("excess_inputs/refraction3.rti", 8, False), ("inputs/input-05.rti", 10, False),
                                             ("inputs/input-02.rti", 10, True)])
def test_plan_miss_is_redone_exactly(gpu, oracle, scene, bdepth, io, schedule, monkeypatch):
    """A plan one level short (RTAMD_PLAN_TRUNCATE test hook): its replay raises DERR_PLAN
    on the device instead of writing the unplanned children, and the render is redone
    host-driven: still bit-exact, counters exact."""
    monkeypatch.setenv("RTAMD_PLAN_TRUNCATE", "1")
    apply_schedule(monkeypatch, schedule)
    w, h = 64, 40
    want, cnt = oracle.render(os.path.join(SCENES, scene), w, h, bdepth=bdepth, intersection_only=io)
    s = gpu.load_scene(os.path.join(SCENES, scene))
    o = gpu.Options(renderWidth_=w, renderHeight_=h, bounceDepth_=bdepth, intersectionOnly_=io)
    for _ in range(3):
        img = s.renderScene(options=o)
        assert np.array_equal(img.view(np.uint64), want.view(np.uint64))
        assert (s.last_stats.trace_rays, s.last_stats.shadow_rays) == (cnt["trace_rays"], cnt["shadow_rays"])
    s.close()


@pytest.mark.parametrize("pack", ["4194304", "20000", "1"])
def test_multi_frame_chunks(gpu, oracle, pack, monkeypatch):
    """Chunks packed from rows of several frames (consecutive batch entries with equal width,
    height and depth: one GPU's shares of row-partitioned frames, whole frames, chunked
    frames) trace as one wavefront; every entry equals its own render, bit for bit, and the
    summed counters equal the single renders' (RTAMD_BATCH_CHUNK bounds the packing)."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("RTAMD_BATCH_CHUNK", pack)
    scene = "excess_inputs/refraction3.rti"
    w, h, bd = 70, 44, 7
    want, cnt = oracle.render(os.path.join(SCENES, scene), w, h, bdepth=bd)
    s = gpu.load_scene(os.path.join(SCENES, scene))
    jobs = [s.params(w, h, bd, False, r, h, 4) for r in range(4)] + [s.params(w, h, bd, False)] + \
        [s.params(w, h, bd, False, 1, h, 2), s.params(w, h, bd, False, chunk_pixels=600)] + \
        [s.params(w, h, 3, False, 0, h, 2), s.params(w, h, bd, False, 0, h, 3)]
    rows = lambda p: len(range(p.row_begin, p.row_end, p.row_step))
    for _ in range(3):  # host-driven, then planned chunks
        outs = [torch.full((rows(p), w, 3), -1.0, dtype=torch.float64, device="cuda") for p in jobs]
        out8 = [torch.zeros((rows(p), w, 3), dtype=torch.uint8, device="cuda") for p in jobs]
        torch.cuda.synchronize()
        st = s.render_batch_device(jobs, [o.data_ptr() for o in outs], [o.data_ptr() for o in out8])
        for k, p in enumerate(jobs):
            if p.bounce_depth != bd:
                continue
            ref = want[p.row_begin:p.row_end:p.row_step]
            assert np.array_equal(outs[k].cpu().numpy().view(np.uint64), ref.view(np.uint64)), k
            assert np.array_equal(out8[k].cpu().numpy(), gpu.to_rgb8(ref)), k
    # counters: 3 whole frames at depth bd (4 quarter shares + 2 halves... = 1 + 1 + 1 + 1 frame
    # of rows 0::3) and one half frame at depth 3 checked against single renders
    single = [0, 0]
    for p in jobs:
        o = torch.empty((rows(p), w, 3), dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        one = s.render_device(p, o.data_ptr(), 0)
        single[0] += one.trace_rays
        single[1] += one.shadow_rays
    assert [st.trace_rays, st.shadow_rays] == single
    s.close()


def test_work_counters_are_optional(gpu, monkeypatch):
    """rt_render_params.work_stats selects the counting instantiation of the traversal
    kernels: the same bits either way, the traversal counters nonzero only when asked for
    (RTAMD_WORK_STATS=1 asks for every call); plans keyed on it."""
    torch = pytest.importorskip("torch")
    w, h = 96, 64
    s = gpu.load_scene(os.path.join(SCENES, "excess_inputs/bunny.rti"))
    outs = {}
    for rep in range(2):  # the second round replays the plans of the first
        for count in (False, True):
            out = torch.zeros((h, w, 3), dtype=torch.float64, device="cuda")
            st = s.render_device(s.params(w, h, 4, False, work_stats=count), out.data_ptr(), 0)
            torch.cuda.synchronize()
            outs[(rep, count)] = out.cpu().numpy()
            counters = (st.node_visits, st.tri_tests, st.candidates, st.sphere_tests) + tuple(st.stage_node_visits) + \
                tuple(st.stage_bvh_traversals)
            assert st.trace_rays > 0 and st.shadow_rays > 0
            if count:
                assert st.node_visits > 0 and st.tri_tests > 0 and st.sphere_tests > 0
            else:
                assert not any(counters), counters
    ref = outs[(0, False)]
    assert all(np.array_equal(ref.view(np.uint64), o.view(np.uint64)) for o in outs.values())
    s.close()
    monkeypatch.setenv("RTAMD_WORK_STATS", "1")
    s = gpu.load_scene(os.path.join(SCENES, "excess_inputs/bunny.rti"))
    out = torch.zeros((h, w, 3), dtype=torch.float64, device="cuda")
    st = s.render_device(s.params(w, h, 4, False), out.data_ptr(), 0)
    torch.cuda.synchronize()
    assert st.node_visits > 0 and np.array_equal(out.cpu().numpy().view(np.uint64), ref.view(np.uint64))
    s.close()
