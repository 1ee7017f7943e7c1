#!/usr/bin/env python
"""Benchmark of the ray-trace hot path on MI355X: Mrays/s at 1920x1080 (BASELINE.json).

Workload (BASELINE.json configs[2], the metric's 1920x1080 single-GPU config):
excess_inputs/bunny.rti (4,968-triangle bunny + reflective floor +
mirror spheres), 1920x1080, --bdepth 4.  A step renders a fixed batch of frames
(--frames-per-step, default 48: 24 two-frame chunks, 8 on each of the library's 3 batch
lanes, so that no lane traces a last chunk alone) of that scene through the C-ABI (librtamd.so); rays =
traceRay calls (primary + reflection + refraction) + shadow rays, counted by the kernels
and equal to the reference's counts.  Inputs (the scene) are resident in HBM before the
timed region; every frame is written as the reference's f64 RasterImage and as RGB8.

Multi-GPU (torchrun, one rank per GPU, RCCL over xGMI), --mode partition (default): every
frame is row-partitioned over the N ranks (8-row blocks interleaved: row r -> rank (r // 8)
mod N, the reference's image-space decomposition of scene.cpp:13-48 spread over GPUs; a
GPU's rows of all the step's frames are traced as shared wavefronts), each rank renders its rows
of all frames of the step (pipelined, rt_render_batch_device) and every frame's RGB8 rows
are gathered to rank 0 over RCCL.  The total work per step is fixed: "scaling": "strong".
--mode replica: frame-parallel instead (each rank renders whole frames, gathered to rank 0;
weak scaling).

In the same run (rank 0 prints ONE JSON line):
  - strong_scaling: ONE frame of each --sweep config (default C5 refraction3 4096^2 depth 8
    and C4 airboat 1920x1080, the 8-GPU configs) row-partitioned over n = 1, 2, 4, 8 <= N
    ranks (sub-communicators), gathered over RCCL: ms, speed-up, per-rank render ms and the
    imbalance (max / mean);
  - roofline of the dominant kernel on a non-overlapping time base: a solo pass
    (RTAMD_SERIAL=1: every kernel alone on one stream, HIP events around each launch)
    against the L2 (algorithmic bytes), HBM (PMC-measured bytes, profiles/) and FP64 roofs;
  - cpu_baseline: the unmodified reference (oracle/_ref) on this host's cores.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3_bunny_1920x1080_bd4]
"""
import argparse
import glob
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E peak (MI355X_MICROARCH.md, memory hierarchy)
# L2-served gather rate of the whole chip: rows every workgroup shares, served from each XCD's
# L2, measured 16.8-18.8 TB/s (MI355X_MICROARCH.md "Indexed rows: gather into LDS", the table's
# first row); the upper figure is the roof (the scene's nodes and faces are such shared rows)
L2_PEAK_GBS = 18800.0
# the hardware's aggregate L2 bandwidth (8 XCDs x 4 MiB L2, the round-1..3 roof): reported
# beside the measured gather ceiling as `l2_aggregate`, so that earlier rounds' L2 fractions
# (taken against this figure) stay comparable
L2_AGGREGATE_GBS = 34500.0
FP64_PEAK_TFLOPS = 78.6     # MI355X vector FP64
NODE_BYTES, TRI_BYTES, NRM_BYTES = 64, 72, 72   # SURVEY.md §8d algorithmic bytes (64-B fp32-box node)
RAY_IO_BYTES, PIXEL_BYTES = 64 + 64, 24
# algorithmic fp64 flops: node visit = two 28-flop slab tests; a triangle
# test 38 flops to the a-reject, +67 for one that reaches the normal + facing test; a
# sphere test 30 + two 28-flop transforms + 12 for the re-normalisation
NODE_FLOPS, TRI_FLOPS, CAND_FLOPS, SPHERE_FLOPS = 56, 38, 67, 98
STAGES = ["k_closest", "k_shadow", "k_shade"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend (nccl = RCCL; gloo only to rehearse N ranks on fewer GPUs)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3_bunny_1920x1080_bd4")
    ap.add_argument("--mode", default="partition", choices=["partition", "replica"])
    ap.add_argument("--emulate-ranks", type=int, default=1,
                    help="development: on ONE GPU, render only rank 0's rows of an N-way partition (the per-GPU "
                         "work of an N-GPU run, to tune it without N GPUs); the line then reports that share")
    ap.add_argument("--row-block", type=int, default=8,
                    help="partition granularity: blocks of this many rows interleaved over the ranks (8 = the "
                         "8x8 ray tiles stay whole)")
    ap.add_argument("--batch-block", type=int, default=0,
                    help="partition of a multi-frame step: blocks of this many rows, rotated per frame (0 = one "
                         "contiguous band of whole 8-row tiles per rank, rtamd.dist.band_rows)")
    ap.add_argument("--frames-per-step", type=int, default=48,
                    help="frames per step (partition: in total, every frame split over the ranks; "
                         "replica: per rank)")
    ap.add_argument("--sweep", default="C5_refraction3_4096_bd8,C4_airboat_sub_1920x1080",
                    help="configs whose single frame is row-partitioned over 1, 2, 4, 8 ranks ('' = none)")
    ap.add_argument("--sweep-reps", type=int, default=3)
    ap.add_argument("--step-order", action="store_true",
                    help="partition mode: hand each rank's frames to the batch call in step order "
                         "instead of rtamd.dist.batch_order (the A/B control)")
    ap.add_argument("--solo-frames", type=int, default=4,
                    help="frames rendered (one batch call) with every kernel alone (RTAMD_SERIAL=1) for the roofline "
                         "time base")
    ap.add_argument("--solo-only", action="store_true",
                    help="run only the solo pass (the command rocprofv3 profiles for the roofline)")
    ap.add_argument("--latency-frames", type=int, default=21,
                    help="single-frame renders timed after the run (wall-clock latency of one frame; median)")
    ap.add_argument("--latency-warmup", type=int, default=2,
                    help="single-frame renders before those, not timed: the first render of the frame's shape "
                         "is traced host-driven and builds its launch plan (api.cpp)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", default=None,
                    help="PMC-measured HBM bytes per launch (rocprofv3 FETCH_SIZE/WRITE_SIZE); default: the "
                         "latest profiles/round*/traffic.json")
    return ap.parse_args()


class stdout_to_stderr:
    """fd 1 -> fd 2 for the block: communication libraries print connection notices on
    stdout (gloo: "[Gloo] Rank 0 is connected to ..."), and rank 0's stdout must hold only
    the one JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def latest_valu():
    cands = sorted(glob.glob(os.path.join(REPO, "profiles", "round*", "valu.json")))
    return cands[-1] if cands else None


def latest_traffic():
    cands = sorted(glob.glob(os.path.join(REPO, "profiles", "round*", "traffic.json")))
    if cands:
        return cands[-1]
    old = os.path.join(REPO, "profiles", "traffic_round1.json")
    return old if os.path.exists(old) else None


def level_buffers(s):
    inf = s.info()
    return {"level_bytes": inf.level_bytes, "level_gib": round(inf.level_bytes / 2**30, 3),
            "level_bytes_peak": inf.level_bytes_peak, "level_peak_gib": round(inf.level_bytes_peak / 2**30, 3),
            "budget": inf.level_budget}


def core_info():
    """The host cores the CPU baseline may use, with the evidence: every
    CPU of this process's affinity set, capped by the cgroup CPU quota when one is set (the
    container's real share of a machine whose nproc counts every CPU) and by OMP_NUM_THREADS
    when the environment sets it (the GPU box sets it to its CPU share)."""
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    omp = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    cores, rule = affinity, "affinity set"
    if quota is not None and int(quota) < cores:
        cores, rule = max(1, int(quota)), "cgroup cpu.max quota"
    if omp is not None and omp < cores:
        cores, rule = omp, "OMP_NUM_THREADS (the box's CPU share)"
    return {"nproc": nproc, "affinity": affinity, "cgroup_quota_cpus": quota, "omp_num_threads": omp,
            "cores": cores, "rule": "cores = min(affinity, cgroup quota, OMP_NUM_THREADS): " + rule}


def _cores():
    return core_info()["cores"]


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def reference_overhead(harness, scene, w, h, bdepth, cores):
    """Wall time of the reference harness rendering no rows (scene parse, worker start, image
    write): subtracted from the sampled runs so that the CPU rate is rendering time only."""
    import subprocess
    env = dict(os.environ, RT_REF_ROWS="0:0:1")
    ts = []
    for _ in range(2):
        t0 = time.perf_counter()
        subprocess.run([harness, scene, "-o", "/dev/null", "-w", str(w), "-h", str(h), "--bdepth", str(bdepth),
                        "-t", str(cores)], env=env, check=True, capture_output=True)
        ts.append(time.perf_counter() - t0)
    return min(ts)


def reference_single_thread(s, scene, w, h, bdepth, target_s):
    """The unmodified reference on ONE core (one worker process, SURVEY.md §8d asks for the
    single-thread time beside the many-core one): evenly spaced rows of the same frame until
    about target_s of CPU work; rays are the kernels' counts for the same rows."""
    import subprocess
    import rtamd
    harness = os.path.join(REPO, "oracle", "_ref", "refharness")
    if not os.access(harness, os.X_OK):
        return None
    overhead = reference_overhead(harness, scene, w, h, bdepth, 1)
    step = 270
    while True:
        rows = (step // 2, h, step)
        env = dict(os.environ, RT_REF_ROWS="%d:%d:%d" % rows)
        t0 = time.perf_counter()
        subprocess.run([harness, scene, "-o", "/dev/null", "-w", str(w), "-h", str(h), "--bdepth", str(bdepth),
                        "-t", "1"], env=env, check=True, capture_output=True)
        dt = time.perf_counter() - t0
        if dt * 2.5 > target_s or step <= 1:
            s.renderScene(options=rtamd.Options(renderWidth_=w, renderHeight_=h, bounceDepth_=bdepth), rows=rows)
            rays = s.last_stats.rays
            n = len(range(*rows))
            render = max(dt - overhead, 1e-6)
            return {"value": rays / render / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "reference",
                    "sample": f"unmodified reference (oracle/_ref/refharness -t 1), {n} rows (every {step}th) of "
                              f"the same {w}x{h} frame: {rays} rays in {render:.2f} s of rendering ({dt:.2f} s wall "
                              f"less {overhead:.2f} s of parse, start and image write)",
                    "frame_s_projected": round(render * h / n, 1)}
        step = max(1, int(step / max(2.0, min(8.0, target_s / max(dt, 1e-3) / 1.5))))


def cpu_baseline(s, scene, w, h, bdepth, target_s):
    """CPU leg on this host's cores over a bounded, evenly spaced row sample of the same frame.

    Prefers the UNMODIFIED reference (oracle/_ref/refharness, built from /root/reference/src
    by `make -C oracle ref`; its fork-parallel pixel loop = one reference process per core);
    falls back to the bit-exact CPU restatement oracle/ ("port").  Rays in the sample are
    the kernels' counts for the same rows (equal to the reference's, see tests)."""
    import subprocess
    import rtamd
    cores = _cores()
    harness = os.path.join(REPO, "oracle", "_ref", "refharness")
    kind = "reference" if os.access(harness, os.X_OK) else "port"
    overhead = reference_overhead(harness, scene, w, h, bdepth, cores) if kind == "reference" else 0.0
    step = 90
    while True:
        rows = (step // 2, h, step)
        if kind == "reference":
            env = dict(os.environ, RT_REF_ROWS="%d:%d:%d" % rows)
            t0 = time.perf_counter()
            subprocess.run([harness, scene, "-o", "/dev/null", "-w", str(w), "-h", str(h), "--bdepth", str(bdepth),
                            "-t", str(cores)], env=env, check=True, capture_output=True)
            dt = time.perf_counter() - t0
        else:
            sys.path.insert(0, os.path.join(REPO, "oracle"))
            import pyoracle
            t0 = time.perf_counter()
            pyoracle.render(scene, w, h, bdepth=bdepth, threads=cores, rows=rows)
            dt = time.perf_counter() - t0
        s.renderScene(options=rtamd.Options(renderWidth_=w, renderHeight_=h, bounceDepth_=bdepth), rows=rows)
        rays = s.last_stats.rays
        n = len(range(*rows))
        if dt * 2.5 > target_s or step <= 1:
            what = ("unmodified reference (oracle/_ref/refharness, %d worker processes)" % cores if kind == "reference"
                    else "oracle/ CPU restatement (%d threads)" % cores)
            render = max(dt - overhead, 1e-6)
            return {"value": rays / render / 1e6, "unit": "Mrays/s", "cores": cores, "kind": kind,
                    "sample": f"{what}, brute-force face loop, on {n} rows (every {step}th) of the same {w}x{h} "
                              f"frame: {rays} rays in {render:.1f} s of rendering ({dt:.1f} s wall less "
                              f"{overhead:.2f} s of scene parse, process start and image write, timed with no rows)",
                    "value_incl_overhead": rays / dt / 1e6}
        step = max(1, int(step / max(2.0, min(8.0, target_s / max(dt, 1e-3) / 1.5))))


def same_algorithm_baseline(scene, w, h, bdepth, target_s):
    """The HIP path's own algorithm (LBVH, any-hit shadows, zero-term decisions) on this host's
    cores: oracle/cpu_bvh_cli (bit-exact with the oracle, tests/test_cpu_bvh.py), whole frames
    until target_s of render time (scene parse and LBVH build excluded) — SURVEY.md H6."""
    import subprocess
    cli = os.path.join(REPO, "oracle", "cpu_bvh_cli")
    if not os.access(cli, os.X_OK):
        return None
    cores = _cores()
    rays, secs, runs = 0, 0.0, 0
    while secs < target_s and runs < 50:
        p = subprocess.run([cli, scene, str(w), str(h), str(bdepth), str(cores), "0", str(h), "1", "/dev/null"],
                           check=True, capture_output=True, text=True)
        st = json.loads(p.stdout)
        rays += st["trace_rays"] + st["shadow_rays"]
        secs += st["render_s"]
        runs += 1
    return {"value": rays / secs / 1e6, "unit": "Mrays/s", "cores": cores, "kind": "port",
            "sample": f"same-algorithm CPU port (oracle/cpu_bvh_cli, {cores} threads: LBVH, any-hit shadows, "
                      f"zero-term decisions), {runs} whole {w}x{h} frames: {rays} rays in {secs:.1f} s of render time"}


def frame_parity(cfg, frame8, frame64):
    """The headline's images against the unmodified reference (tests/golden/ref_hashes.json,
    generated by tests/golden/make_golden.py from oracle/_ref): sha256 of one RGB8 frame of
    the last timed step (and of its f64 image when this rank rendered whole frames).
    Reference output contract: scene.cpp:25-31 (RasterImage), writers.cpp:4-9 (RGB8)."""
    import hashlib
    try:
        ref = json.load(open(os.path.join(REPO, "tests", "golden", "ref_hashes.json")))["configs"][cfg]
    except (OSError, ValueError, KeyError):
        return {"parity": None, "note": "no golden hashes for " + cfg}
    out = {"golden": "tests/golden/ref_hashes.json configs." + cfg}
    ok = True
    if frame8 is not None:
        got = hashlib.sha256(frame8.contiguous().cpu().numpy().tobytes()).hexdigest()
        out["rgb8_sha256_match"] = got == ref["rgb8_sha256"]
        ok = ok and out["rgb8_sha256_match"]
    if frame64 is not None:
        got = hashlib.sha256(frame64.contiguous().cpu().numpy().tobytes()).hexdigest()
        out["f64_sha256_match"] = got == ref["f64_sha256"]
        ok = ok and out["f64_sha256_match"]
    out["parity"] = bool(ok) if (frame8 is not None or frame64 is not None) else None
    return out


def stage_work(st):
    """SURVEY.md §8d algorithmic bytes and flops per kernel family of one render's counters."""
    nbytes, flops = [0, 0, 0], [0, 0, 0]
    for k, nrays in ((0, st.trace_rays), (1, st.shadow_rays)):
        nbytes[k] = (nrays * RAY_IO_BYTES + st.stage_node_visits[k] * NODE_BYTES + st.stage_tri_tests[k] * TRI_BYTES +
                     st.stage_candidates[k] * NRM_BYTES)
        flops[k] = (st.stage_node_visits[k] * NODE_FLOPS + st.stage_tri_tests[k] * TRI_FLOPS +
                    st.stage_candidates[k] * CAND_FLOPS + st.stage_sphere_tests[k] * SPHERE_FLOPS)
    nbytes[2] = st.pixels * PIXEL_BYTES
    return nbytes, flops


def solo_pass(scene_path, W, H, kw, frames, device):
    """Every kernel alone, in the bench's own (batch) schedule: `frames` frames in ONE
    rt_render_batch_device call on a scene created with RTAMD_SERIAL=1 (the shading kernels
    on the closest-hit chain's stream) and RTAMD_BATCH_LANES=1 (one pipeline), so the HIP
    events around each launch bracket that kernel and nothing else, while the batch-mode
    schedule (frames packed into shared chunks, direct/deferred shading split) is the one the
    timed steps run concurrently."""
    import rtamd
    import torch
    keep = {k: os.environ.get(k) for k in ("RTAMD_SERIAL", "RTAMD_BATCH_LANES")}
    os.environ.update({"RTAMD_SERIAL": "1", "RTAMD_BATCH_LANES": "1"})
    try:
        s = rtamd.load_scene(scene_path, device=device)
        s.upload()
    finally:
        for k, v in keep.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    outs = [torch.empty((H, W, 3), dtype=torch.float64, device="cuda") for _ in range(frames)]
    out8s = [torch.empty((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(frames)]
    prm = [s.params(W, H, kw["bdepth"], kw["intersection_only"], 0, H, 1)] * frames
    stream = torch.cuda.current_stream().cuda_stream
    ptrs = ([o.data_ptr() for o in outs], [o.data_ptr() for o in out8s])
    s.render_batch_device(prm, *ptrs, stream)  # allocations
    acc = {"ms": [0.0] * 3, "launches": [0] * 3, "bytes": [0] * 3, "flops": [0] * 3, "wall": 0.0}
    # the work counts: the same call with the counting kernels (rt_render_params.work_stats;
    # counting costs ~6% of the traversal kernels' time, so the timed call runs without it)
    counted = s.render_batch_device([s.params(W, H, kw["bdepth"], kw["intersection_only"], 0, H, 1, work_stats=True)]
                                    * frames, *ptrs, stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = s.render_batch_device(prm, *ptrs, stream)
    acc["wall"] += time.perf_counter() - t0
    nb, fl = stage_work(counted)
    for k in range(3):
        acc["ms"][k] += st.stage_ms[k]
        acc["launches"][k] += st.stage_launches[k]
        acc["bytes"][k] += nb[k]
        acc["flops"][k] += fl[k]
    per = lambda xs: [x // frames for x in xs]
    acc["work_per_frame"] = {"node_visits": per(counted.stage_node_visits), "tri_tests": per(counted.stage_tri_tests),
                             "candidates": per(counted.stage_candidates),
                             "sphere_tests": per(counted.stage_sphere_tests),
                             "bvh_traversals": per(counted.stage_bvh_traversals),
                             "max_node_visits_per_ray": list(counted.stage_max_node_visits)}
    s.close()
    return acc


def roofline(solo, frames, traffic_path, concurrent, valu_path=None):
    """Dominant kernel (largest solo time per frame) against three roofs; `bound` = the roof
    it is closest to.  achieved / peak / frac are that roof's; every fraction is listed."""
    dom = max(range(3), key=lambda k: solo["ms"][k])
    name = STAGES[dom]
    launches = solo["launches"][dom]
    t_launch_s = solo["ms"][dom] / launches * 1e-3
    alg_bytes = solo["bytes"][dom] / launches
    flops = solo["flops"][dom] / launches
    traffic, traffic_note = None, None
    if traffic_path and os.path.exists(traffic_path):
        try:
            tj = json.load(open(traffic_path))
            traffic = tj.get("hbm_bytes_per_launch", {}).get(name)
            traffic_note = os.path.relpath(traffic_path, REPO) + ": " + tj.get("method", "")
        except (OSError, ValueError):
            traffic = None
    roofs = {
        "l2": {"achieved": alg_bytes / t_launch_s / 1e9, "peak": L2_PEAK_GBS, "unit": "GB/s",
               "what": "SURVEY.md §8d algorithmic bytes (ray I/O + LBVH nodes + triangles + normals; the scene "
                       "is L2/MALL-resident) / solo launch time vs the chip's measured L2-served gather rate "
                       "(18.8 TB/s, MI355X_MICROARCH.md 'Indexed rows: gather into LDS')"},
        "l2_aggregate": {"achieved": alg_bytes / t_launch_s / 1e9, "peak": L2_AGGREGATE_GBS, "unit": "GB/s",
                         "what": "the same bytes vs the aggregate L2 bandwidth (34.5 TB/s) that rounds 1-3 used as "
                                 "the L2 roof (for comparison with them; the gather ceiling above is the roof)"},
        "fp64": {"achieved": flops / t_launch_s / 1e12, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                 "what": "SURVEY.md §8d algorithmic FP64 flops / solo launch time vs vector FP64 peak"},
    }
    if valu_path and os.path.exists(valu_path):
        try:
            vj = json.load(open(valu_path))
            vpl = vj.get("valu_per_launch", {}).get(name)
            if vpl and vj.get("peak_wave_instr_per_s"):
                roofs["valu"] = {"achieved": vpl / t_launch_s / 1e9, "peak": vj["peak_wave_instr_per_s"] / 1e9,
                                 "unit": "G wave-instr/s",
                                 "what": "PMC SQ_INSTS_VALU per launch (wave64 vector instructions, " +
                                         os.path.relpath(valu_path, REPO) + ") / solo launch time vs " +
                                         vj.get("peak_what", "the calibrated VALU issue rate"),
                                 "counters": {k: vj[k].get(name) for k in ("valu_busy", "wait_any", "wait_inst_any")
                                              if isinstance(vj.get(k), dict)}}
        except (OSError, ValueError):
            pass
    if traffic:
        roofs["hbm"] = {"achieved": traffic / t_launch_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "what": "PMC HBM bytes per launch (FETCH_SIZE, WRITE_SIZE; profiles/) / solo launch time"}
    for r in roofs.values():
        r["frac"] = r["achieved"] / r["peak"]
        r["achieved"] = round(r["achieved"], 3)
        r["frac"] = round(r["frac"], 4)
    bound = max((k for k in roofs if k != "l2_aggregate"), key=lambda k: roofs[k]["frac"])
    b = roofs[bound]
    return {
        "bound": bound, "achieved": b["achieved"], "peak": b["peak"], "unit": b["unit"], "frac": b["frac"],
        "traffic": traffic, "kernel": name,
        "time_base": f"solo: {frames} frames in one batch call (the bench's schedule) with RTAMD_SERIAL=1 and "
                     "RTAMD_BATCH_LANES=1 (every kernel alone on one stream), HIP events around each launch on that "
                     "stream; rocprofv3 of `bench.py --solo-only` gives the same durations (profiles/)",
        "avg_launch_ms": round(t_launch_s * 1e3, 4), "launches_per_frame": launches / frames,
        "algorithmic_bytes_per_launch": round(alg_bytes), "fp64_flops_per_launch": round(flops),
        "roofs": roofs, "traffic_source": traffic_note,
        "solo_ms_per_frame": {STAGES[k]: round(solo["ms"][k] / frames, 4) for k in range(3)},
        "solo_frame_wall_ms": round(solo["wall"] / frames * 1e3, 3),
        "concurrent": concurrent,
    }


XGMI_LINK_GBS = 64.0    # assumed per-link, per-direction rate of the RGB8 gather (prompt: 7 links x ~153 GB/s per GPU)
XGMI_FIXED_US = 25.0    # assumed fixed cost of one RCCL gather


def emulated_scaling(a, local, torch):
    """Single-frame strong scaling emulated on ONE GPU (WORLD_SIZE=1): for n = 1, 2, 4, 8, every
    rank's share of ONE frame (8-row blocks interleaved, rank k: rows (r // 8) mod n == k; the
    reference's block dispenser scene.cpp:13-48 at GPU granularity) is rendered alone, one share
    at a time, on this GPU.  Reported per n: each share's render ms (median of reps), the max
    (an n-GPU frame waits for its slowest rank), the imbalance (max / mean) and a projected
    speed-up = T(1) / (max share + gather), the gather priced at the RGB8 rows of the largest
    remote share over one xGMI link at an ASSUMED rate (XGMI_LINK_GBS, XGMI_FIXED_US): every
    remote rank sends to rank 0 over its own link."""
    import rtamd
    from rtamd import dist as rd
    from rtamd.configs import CONFIGS, SCENES, option_kwargs
    out = {}
    blk = max(1, a.row_block)
    stream = torch.cuda.current_stream().cuda_stream
    for cfg in [c for c in a.sweep.split(",") if c]:
        scene_rel, W, H, flags = CONFIGS[cfg]
        kw = option_kwargs(flags)
        s = rtamd.load_scene(os.path.join(SCENES, scene_rel), device=local)
        s.upload()
        curve = []
        for n in (1, 2, 4, 8):
            n_max = max(rd.n_rows(H, k, n, blk) for k in range(n))
            buf = torch.zeros((n_max, W, 3), dtype=torch.uint8, device="cuda")
            share_ms, rays = [], 0
            for k in range(n):
                prm = s.params(W, H, kw["bdepth"], kw["intersection_only"], k * blk, H, n, row_block=blk)
                ts = []
                for rep in range(a.sweep_reps + 1):  # rep 0: warm-up (level buffers, launch plans)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    st = s.render_device(prm, 0, buf.data_ptr(), stream)
                    torch.cuda.synchronize()
                    if rep > 0:
                        ts.append(time.perf_counter() - t0)
                share_ms.append(statistics.median(ts) * 1e3)
                rays += st.rays
            remote_rows = max([rd.n_rows(H, k, n, blk) for k in range(1, n)] or [0])
            gather_ms = 0.0 if n == 1 else (remote_rows * W * 3 / (XGMI_LINK_GBS * 1e9) * 1e3 + XGMI_FIXED_US / 1e3)
            proj = max(share_ms) + gather_ms
            curve.append({"n_gpus": n, "render_ms_per_rank": [round(x, 3) for x in share_ms],
                          "max_ms": round(max(share_ms), 3), "imbalance": round(max(share_ms) / (sum(share_ms) / n), 3),
                          "gather_ms_assumed": round(gather_ms, 4), "projected_ms": round(proj, 3), "rays": int(rays)})
        base = curve[0]["projected_ms"]
        for r in curve:
            r["projected_speedup"] = round(base / r["projected_ms"], 3)
            r["projected_efficiency"] = round(base / r["projected_ms"] / r["n_gpus"], 3)
        out[cfg] = {"emulated": True, "scene": scene_rel, "width": W, "height": H, "bounce_depth": kw["bdepth"],
                    "partition": f"{blk}-row blocks interleaved (row r -> rank (r // {blk}) mod n); each rank's share "
                                 "rendered alone on this one GPU, one share at a time",
                    "gather_model": f"largest remote share's RGB8 rows / {XGMI_LINK_GBS:g} GB/s per xGMI link + "
                                    f"{XGMI_FIXED_US:g} us (assumed, not measured)",
                    "curve": curve,
                    "batch_partition_8way": emulated_batch_partition(a, s, W, H, kw, blk, cfg, torch)}
        s.close()
    return out


BATCH_FRAMES = {"C5_refraction3_4096_bd8": 16}  # frames per emulated batch step (default 48, bench.py's own)


def emulated_batch_partition(a, s, W, H, kw, blk, cfg, torch, n=8):
    """The throughput form of an n-GPU node for a sweep config (VERDICT r4 "next" 3): every
    rank renders its row blocks of the SAME F frames in one rt_render_batch_device call (the
    bench's partition mode: rotated, frame f's blocks of residue (rank + f) mod n, so that with
    F a multiple of n every rank renders the same rows in total), emulated on this one GPU one
    rank's share at a time; the node's
    step takes the slowest share or the assumed gather of its F x rows of RGB8, whichever is
    longer: the bench overlaps a step's gather with the next step's render (main(), side
    stream, double-buffered RGB8), so in steady state the two run concurrently; the serial
    sum is reported beside it.  Reported beside the one-GPU batch of the same F whole frames."""
    from rtamd import dist as rd
    F = BATCH_FRAMES.get(cfg, 48)
    stream = torch.cuda.current_stream().cuda_stream

    def timed(prm_list, rows):
        outs = torch.empty((len(prm_list), rows, W, 3), dtype=torch.uint8, device="cuda")
        ts, rays = [], 0
        for rep in range(a.sweep_reps + 1):  # rep 0: warm-up (level buffers, launch plans)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st = s.render_batch_device(prm_list, [], [outs[f].data_ptr() for f in range(len(prm_list))], stream)
            torch.cuda.synchronize()
            if rep > 0:
                ts.append(time.perf_counter() - t0)
            rays = st.rays
        return statistics.median(ts) * 1e3, rays

    whole_ms, whole_rays = timed([s.params(W, H, kw["bdepth"], kw["intersection_only"], 0, H, 1)] * F, H)
    share_ms, rays = [], 0
    bblk = a.batch_block if a.batch_block > 0 else rd.band_rows(H, n)
    for k in range(n):  # rank k's rotated share (rtamd.dist.batch_rows), as bench.py's partition step renders it
        sel = rd.batch_rows(H, k, n, F, bblk)
        if not a.step_order:
            sel = [sel[f] for f in rd.batch_order(k, n, F)]
        rows = max(rd.n_rows(H, q, n, bblk) for q in range(n))
        ms, r = timed([s.params(W, H, kw["bdepth"], kw["intersection_only"], b, e, st, row_block=bl)
                       for (b, e, st, bl) in sel], rows)
        share_ms.append(round(ms, 3))
        rays += r
    remote_rows = max(rd.n_rows(H, k, n, bblk) for k in range(1, n))
    gather_ms = F * remote_rows * W * 3 / (XGMI_LINK_GBS * 1e9) * 1e3 + XGMI_FIXED_US / 1e3
    node_ms = max(max(share_ms), gather_ms)
    serial_ms = max(share_ms) + gather_ms
    return {"frames_per_step": F, "n_gpus": n, "rows_per_block": bblk,
            "partition": f"{bblk}-row blocks ({'one contiguous band per rank' if bblk == rd.band_rows(H, n) else 'interleaved'}), "
                         f"rotated per frame: frame f's blocks of residue (rank + f) mod {n} on rank k",
            "one_gpu_batch_ms": round(whole_ms, 3),
            "one_gpu_mrays_per_s": round(whole_rays / whole_ms / 1e3, 1),
            "share_ms_per_rank": share_ms, "max_share_ms": max(share_ms),
            "imbalance": round(max(share_ms) / (sum(share_ms) / n), 3), "gather_ms_assumed": round(gather_ms, 3),
            "projected_node_mrays_per_s": round(rays / node_ms / 1e3, 1),
            "projected_speedup": round(whole_ms / node_ms, 3),
            "projected_speedup_gather_not_overlapped": round(whole_ms / serial_ms, 3),
            "per_gpu_mrays_per_s_of_share": round(rays / n / (sum(share_ms) / n) / 1e3, 1)}


def strong_scaling(a, world, rank, local, groups, dist, torch):
    """ONE frame of each sweep config, row-interleaved over n = 1, 2, 4, 8 <= world ranks and
    gathered to rank 0 over RCCL (RGB8), timed end to end; ranks >= n idle."""
    import rtamd
    from rtamd import dist as rd
    from rtamd.configs import CONFIGS, SCENES, option_kwargs
    out = {}
    for cfg in [c for c in a.sweep.split(",") if c]:
        scene_rel, W, H, flags = CONFIGS[cfg]
        kw = option_kwargs(flags)
        s = rtamd.load_scene(os.path.join(SCENES, scene_rel), device=local)
        s.upload()
        stream = torch.cuda.current_stream().cuda_stream
        rows_curve = []
        blk = max(1, a.row_block)
        for n, grp in groups:
            n_max = max(rd.n_rows(H, k, n, blk) for k in range(n))
            buf = torch.zeros((n_max, W, 3), dtype=torch.uint8, device="cuda")
            frame = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda") if rank == 0 else None
            bufs = [torch.empty_like(buf) for _ in range(n)] if rank == 0 and n > 1 else None
            prm = s.params(W, H, kw["bdepth"], kw["intersection_only"], rank * blk, H, n, row_block=blk) \
                if rank < n else None
            samples = []
            for rep in range(a.sweep_reps + 1):  # rep 0: warm-up (level buffers for this row count)
                if world > 1:
                    dist.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                rays, t_render = 0, 0.0
                if rank < n:
                    st = s.render_device(prm, 0, buf.data_ptr(), stream)
                    torch.cuda.synchronize()
                    t_render = time.perf_counter() - t0
                    rays = st.rays
                    if n > 1:
                        rd.gather_rows(buf, H, dst=0, out=frame, bufs=bufs, group=grp, group_size=n, group_rank=rank,
                                       block=blk)
                    elif rank == 0:
                        frame.copy_(buf)
                    torch.cuda.synchronize()
                t_total = time.perf_counter() - t0
                v = torch.tensor([t_render, t_total, float(rays)], dtype=torch.float64, device="cuda")
                if world > 1:
                    allv = [torch.empty_like(v) for _ in range(world)]
                    dist.all_gather(allv, v)
                    allv = [x.tolist() for x in allv[:n]]
                else:
                    allv = [v.tolist()]
                if rep > 0:
                    samples.append(allv)
            if rank == 0:
                tot = [max(r[1] for r in smp) for smp in samples]
                med = statistics.median_low(tot)
                pick = samples[tot.index(med)]
                rend = [r[0] * 1e3 for r in pick]
                rays = sum(r[2] for r in pick)
                rows_curve.append({"n_gpus": n, "ms": round(med * 1e3, 3), "mrays_per_s": round(rays / med / 1e6, 1),
                                   "render_ms_per_rank": [round(x, 3) for x in rend],
                                   "imbalance": round(max(rend) / (sum(rend) / len(rend)), 3),
                                   "gather_ms": round((med - max(r[0] for r in pick)) * 1e3, 3), "rays": int(rays)})
        if rank == 0:
            base = rows_curve[0]["ms"]
            for r in rows_curve:
                r["speedup"] = round(base / r["ms"], 3)
                r["efficiency"] = round(base / r["ms"] / r["n_gpus"], 3)
            out[cfg] = {"scene": scene_rel, "width": W, "height": H, "bounce_depth": kw["bdepth"],
                        "partition": f"{blk}-row blocks interleaved (row r -> rank (r // {blk}) mod n), RGB8 rows "
                                     "gathered to rank 0 over "
                                     + ("RCCL" if dist.is_initialized() and dist.get_backend() == "nccl" else
                                        "the process group" if world > 1 else "nothing (one rank)"),
                        "curve": rows_curve}
        s.close()
    return out


def rank_topology(a, world, rank, local, dist, torch):
    """Which GPU every rank drives, so that a multi-GPU line proves itself: the PCI address of
    each rank's device, gathered to every rank, and the RCCL communicator's size.  Over RCCL
    (backend nccl) two ranks on one GPU make the scaling figures meaningless: the run stops
    with exit code 3 before any timing (gloo rehearsals may share a GPU on purpose)."""
    p = torch.cuda.get_device_properties(local)
    me = "%04x:%02x:%02x" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
    if world > 1:
        ids = [None] * world
        with stdout_to_stderr():
            grp = dist.new_group(backend="gloo")  # host-side exchange: no RCCL communicator yet
            dist.all_gather_object(ids, me, group=grp)
            dist.destroy_process_group(grp)
    else:
        ids = [me]
    nccl = world > 1 and dist.get_backend() == "nccl"
    topo = {"backend": dist.get_backend() if world > 1 else None, "world_size": world,
            "rccl_nranks": world if nccl else None, "rank_pci_bus_ids": ids,
            "distinct_gpus": len(set(ids))}
    if nccl and len(set(ids)) != world:
        if rank == 0:
            sys.stderr.write("bench.py: %d RCCL ranks drive only %d distinct GPUs (%s): every rank needs a GPU of its "
                             "own for a scaling measurement\n" % (world, len(set(ids)), ", ".join(ids)))
        sys.exit(3)
    return topo


def main():
    a = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import torch
    import torch.distributed as dist
    import rtamd
    from rtamd import dist as rd
    from rtamd.configs import CONFIGS, SCENES, option_kwargs

    # more ranks than visible GPUs share them (a gloo rehearsal); over RCCL rank_topology then
    # stops the run with a message instead of a device-ordinal error
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        with stdout_to_stderr():
            # nccl without device_id: its communicator is made at the first collective, after
            # rank_topology has checked that every rank drives a GPU of its own
            dist.init_process_group(a.backend)
    topology = rank_topology(a, world, rank, local, dist, torch)
    if world > 1:
        with stdout_to_stderr():
            dist.barrier(device_ids=[local] if a.backend == "nccl" else None)  # the connections are made here
    scene_rel, W, H, flags = CONFIGS[a.config]
    kw = option_kwargs(flags)
    scene = os.path.join(SCENES, scene_rel)
    traffic_path = a.traffic or latest_traffic()

    if a.solo_only:  # the profiled command of the roofline's time base
        solo = solo_pass(scene, W, H, kw, a.solo_frames, local)
        if rank == 0:
            print(json.dumps({"solo_only": True, "config": a.config,
                              "roofline": roofline(solo, a.solo_frames, traffic_path, None, latest_valu())}),
                  flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    s = rtamd.load_scene(scene, device=local)
    s.upload()
    B = max(1, a.frames_per_step)
    partition = a.mode == "partition"
    # this rank's rows of every frame (partition: the rotated assignment of rtamd.dist.batch_rows,
    # frame f's blocks of residue (rank + f) mod ways, so that every rank does the same work per
    # step) or whole frames (replica)
    ways = world if a.emulate_ranks <= 1 else a.emulate_ranks * world
    blk = a.batch_block if a.batch_block > 0 else rd.band_rows(H, ways)
    frame_rows = rd.batch_rows(H, rank, ways, max(1, a.frames_per_step), blk) if partition else \
        [(0, H, 1, 1)] * max(1, a.frames_per_step)
    rows = frame_rows[0]
    n_loc = sum(rd.n_rows(H, (rank + f) % ways, ways, blk) for f in range(len(frame_rows))) / len(frame_rows) \
        if partition else H
    # gather buffers: the longest rank's row count
    n_buf = max(rd.n_rows(H, k, ways, blk) for k in range(ways)) if partition else H
    outs = [torch.empty((n_buf, W, 3), dtype=torch.float64, device="cuda") for _ in range(B)]
    # RGB8 double-buffered: the gathers of step i (side stream) overlap the render of step i+1
    # (one tensor per buffer set: partition mode gathers all the step's frames in ONE collective)
    out8s = [torch.zeros((B, n_buf, W, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
    gathered = [None, None]
    comm = torch.cuda.Stream() if world > 1 else torch.cuda.current_stream()
    prms = [s.params(W, H, kw["bdepth"], kw["intersection_only"], r[0], r[1], r[2], row_block=r[3]) for r in frame_rows]
    prm = prms[0]
    # the frames in the order the rank hands them to the batch call (rtamd.dist.batch_order:
    # every rank's chunks hold the image's blocks in the same order); outputs stay per frame
    order = rd.batch_order(rank, ways, B) if partition and not a.step_order else list(range(B))
    prms_ordered = [prms[f] for f in order]
    stream = torch.cuda.current_stream().cuda_stream
    gbufs = torch.empty((world, B, n_buf, W, 3), dtype=torch.uint8, device="cuda") \
        if rank == 0 and world > 1 and partition else None
    n_frames_rank0 = B if partition else B * world
    frames = torch.empty((n_frames_rank0, H, W, 3), dtype=torch.uint8, device="cuda") if rank == 0 else None

    totals = {"rays": 0, "trace_rays": 0, "zero": 0, "ms": [0.0] * 3, "launches": [0] * 3}
    work = {}
    n_steps = [0]

    def step(record):
        k = n_steps[0] % 2
        n_steps[0] += 1
        if gathered[k] is not None:  # the gathers that read these buffers two steps ago
            torch.cuda.current_stream().wait_event(gathered[k])
        st = s.render_batch_device(prms_ordered, [outs[f].data_ptr() for f in order],
                                   [out8s[k][f].data_ptr() for f in order], stream)
        rendered = torch.cuda.Event()
        rendered.record()
        with torch.cuda.stream(comm):
            comm.wait_event(rendered)
            if partition and ways != world:  # emulated share: no assembly
                pass
            elif partition:  # every frame assembled on rank 0 from all ranks' rows: one gather per step
                rd.gather_rows_batch(out8s[k], H, dst=0, out=frames, bufs=gbufs, block=blk, rotate=True)
            else:
                for f in range(B):
                    if world > 1:  # whole frames of every rank to rank 0
                        rd.gather_frames(out8s[k][f], dst=0,
                                         out=[frames[f * world + r] for r in range(world)] if rank == 0 else None)
                    else:
                        frames[f].copy_(out8s[k][f])
            gathered[k] = torch.cuda.Event()
            gathered[k].record(comm)
        if record:
            totals["rays"] += st.trace_rays + st.shadow_rays
            totals["trace_rays"] += st.trace_rays
            totals["zero"] += st.shadow_rays_zero_terms
            for j in range(3):
                totals["ms"][j] += st.stage_ms[j]
                totals["launches"][j] += st.stage_launches[j]
            # the batch's B renders do identical work; the traversal counts (node visits ...)
            # come from the solo pass's counting call (the timed kernels do not count)
            work.update({"trace_rays": st.trace_rays // B, "shadow_rays": st.shadow_rays // B,
                         "shadow_rays_zero_terms": st.shadow_rays_zero_terms // B})

    for _ in range(a.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    torch.cuda.synchronize()
    t_rank = time.perf_counter() - t0  # this rank's own work done (before waiting for the others)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the timed path's own output, checked against the reference (after the timed region):
    # rank 0's assembled RGB8 frame of the last step, and its f64 image when it rendered whole frames
    parity = None
    if rank == 0 and ways == world:
        last = (n_steps[0] - 1) % 2
        f8 = frames[n_frames_rank0 - 1] if frames is not None else None
        f64 = outs[B - 1] if (not partition or world == 1) else None
        parity = frame_parity(a.config, f8, f64)
        parity["frame"] = f"frame {n_frames_rank0 - 1} of the last timed step (buffer set {last})"
    # wall-clock of ONE frame's rows on this rank (one render call, nothing else in flight)
    lat = []
    for _ in range(max(0, a.latency_warmup) if a.latency_frames > 0 else 0):
        s.render_device(prm, outs[0].data_ptr(), out8s[0][0].data_ptr(), stream)
    for _ in range(max(0, a.latency_frames)):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        s.render_device(prm, outs[0].data_ptr(), out8s[0][0].data_ptr(), stream)  # (frame 0 of set 0)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t1)
    lat = sorted(lat)[len(lat) // 2] if lat else float("nan")
    vals = [elapsed, float(totals["rays"]), float(totals["trace_rays"]), lat, float(totals["zero"]), t_rank] + \
        totals["ms"] + [float(x) for x in totals["launches"]]
    agg = torch.tensor(vals, dtype=torch.float64, device="cuda")
    if world > 1:
        allv = [torch.empty_like(agg) for _ in range(world)]
        dist.all_gather(allv, agg)
        allv = [x.tolist() for x in allv]
    else:
        allv = [agg.tolist()]
    elapsed = max(v[0] for v in allv)  # max over ranks
    rays = sum(v[1] for v in allv)
    trace_rays = sum(v[2] for v in allv)
    latency = max(v[3] for v in allv)
    zero_rays = sum(v[4] for v in allv)
    rank_ms = [v[5] / a.steps * 1e3 for v in allv]
    conc_launches = [sum(v[9 + j] for v in allv) for j in range(3)]

    sweep = {}
    groups = []
    n = 1
    while n <= world:
        with stdout_to_stderr():
            groups.append((n, dist.new_group(list(range(n))) if world > 1 and n > 1 else None))
        n *= 2
    if a.sweep and world == 1 and a.emulate_ranks <= 1:
        sweep = emulated_scaling(a, local, torch)
    elif a.sweep:
        sweep = strong_scaling(a, world, rank, local, groups, dist, torch)
    solo = solo_pass(scene, W, H, kw, a.solo_frames, local) if rank == 0 and a.solo_frames > 0 else None

    if rank == 0:
        fps = B if partition else B * world  # frames per step
        value = rays / elapsed / 1e6
        # the throughput schedule replays launch plans without per-kernel events (api.cpp Plan):
        # only the launch counts are known there; kernel times come from the solo pass
        concurrent = {"launches_per_frame": {STAGES[j]: conc_launches[j] / a.steps / fps for j in range(3)}}
        res = {
            "metric": "Mrays/s (primary+secondary) and wall-clock at 1920x1080; HBM GB/s vs peak",
            "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong" if partition else "weak",
            "mrays_trace": round(trace_rays / elapsed / 1e6, 3),
            # rays that went through a traversal: the shadow rays decided by zero Phong terms
            #  count in `value` like every other ray the reference casts
            "mrays_traversed": round((rays - zero_rays) / elapsed / 1e6, 3),
            "vs_baseline": None, "dtype": "f64", "data": "synthetic: shipped reference scene data (bunny.obj), "
                                                        "deterministic, no RNG",
            "config": {"workload": a.config, "scene": scene_rel, "width": W, "height": H,
                       "bounce_depth": kw["bdepth"], "frames_per_step": fps,
                       "rays_per_frame": int(rays / a.steps / fps),
                       "ms_per_frame": round(elapsed / a.steps / fps * 1e3, 3),
                       "frame_latency_ms": round(latency * 1e3, 3),
                       "frame_latency_how": f"median of {a.latency_frames} single-frame render_device calls (f64 + RGB8 "
                                            f"into HBM) after the timed steps and {a.latency_warmup} untimed ones",
                       "row_block": blk if partition else None,
                       "parallelism": (f"EMULATED rank share: rank 0's {n_loc:g} of {H} rows per frame of an {ways}-way "
                                       f"partition, {fps} frames/step on 1 GPU (development measure, not a job)"
                                       if ways != world else
                                       f"{fps} frames/step, each split into {blk}-row blocks over {world} GPU(s) "
                                       f"({'one contiguous band per GPU' if blk == rd.band_rows(H, world) else 'interleaved'}), "
                                       f"rotated per frame (frame f: blocks of residue (rank + f) mod {world} on each rank, "
                                       f"{n_loc:g} rows of {H} per frame on rank 0), pipelined renders per GPU, "
                                       f"{'RCCL' if a.backend == 'nccl' else 'gloo (rehearsal)'} gather "
                                       "of every frame's RGB8 rows to rank 0" if partition and world > 1 else
                                       f"1 GPU, {fps} frames/step pipelined (rt_render_batch_device)" if world == 1
                                       else f"frame-parallel: {B} whole frames per GPU per step, gathered to rank 0")},
            "per_rank": {"ms_per_step": [round(x, 3) for x in rank_ms],
                         "imbalance": round(max(rank_ms) / (sum(rank_ms) / len(rank_ms)), 3)},
            "roofline": roofline(solo, a.solo_frames, traffic_path, concurrent, latest_valu()) if solo else None,
            "parity": parity,
            "work_per_frame_rank0": work,
            "traversal_work_per_frame": solo["work_per_frame"] if solo else None,
            "strong_scaling": sweep,
            "topology": topology,
            # HBM the timed scene's level buffers hold after the run, their peak during it, and the
            # RTAMD_LEVEL_BUDGET they were held to (0: none)
            "level_buffers": level_buffers(s),
        }
        if res["roofline"]:
            # the dominant kernel's solo time per step must fit in the step (a consistent time base)
            dom = res["roofline"]["kernel"]
            res["roofline"]["solo_ms_per_step"] = round(res["roofline"]["solo_ms_per_frame"][dom] * fps / world, 3)
        if world == 1 and not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(s, scene, W, H, kw["bdepth"], a.cpu_seconds)
            res["cpu_baseline"]["cpu_model"] = cpu_model()
            ci = core_info()
            res["cpu_baseline"].update({"nproc": ci["nproc"], "affinity": ci["affinity"], "host_cpus": ci})
            one = reference_single_thread(s, scene, W, H, kw["bdepth"], a.cpu_seconds / 3)
            if one:
                res["cpu_baseline"]["single_thread"] = one
            same = same_algorithm_baseline(scene, W, H, kw["bdepth"], a.cpu_seconds / 3)
            if same:
                res["cpu_baseline"]["same_algorithm"] = same
        print(json.dumps(res), flush=True)
    s.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
