#!/usr/bin/env python
"""Benchmark of the ray-trace hot path on MI355X: Mrays/s at 1920x1080 (BASELINE.json).

Workload (BASELINE.json configs[2], the metric's 1920x1080 single-GPU config):
excess_inputs/bunny.rti (4,968-triangle bunny + reflective floor +
mirror spheres), 1920x1080, --bdepth 4.  A step renders frames of that scene through
the C-ABI (librtamd.so); rays = traceRay calls (primary + reflection + refraction) +
shadow rays, counted by the kernels and equal to the reference's counts.

Multi-GPU (torchrun, one rank per GPU, RCCL): a step renders a batch of N frames, each
row-interleaved over all N ranks and assembled on rank 0 by an RCCL gather of its RGB8
rows over xGMI (rtamd.dist.gather_batch).  The interleave rotates with the frame (frame
f's rows of residue k are rendered by rank (k - f) mod N), so each rank renders every row
once per step in ONE render call: per-GPU work is one frame per step (weak scaling) and
each GPU pays the per-call latency of the level chain once per step, not once per frame.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3_bunny_1920x1080_bd4]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
NODE_BYTES, TRI_BYTES, NRM_BYTES = 64, 72, 72   # SURVEY.md §8d algorithmic bytes (64-B fp32-box node)
RAY_IO_BYTES, PIXEL_BYTES = 64 + 64, 24
FP64_PEAK_TFLOPS = 78.6     # MI355X vector FP64
# algorithmic fp64 flops: node visit = two 28-flop slab tests; a triangle
# test 38 flops to the a-reject, +67 for one that reaches the normal + facing test; a
# sphere test 30 + two 28-flop transforms + 12 for the re-normalisation
NODE_FLOPS, TRI_FLOPS, CAND_FLOPS, SPHERE_FLOPS = 56, 38, 67, 98


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend (nccl = RCCL; gloo only to rehearse N ranks on fewer GPUs)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3_bunny_1920x1080_bd4")
    ap.add_argument("--frames-per-gpu", type=int, default=4,
                    help="frames per GPU per step, pipelined over the scene's lanes (rt_render_batch_device)")
    ap.add_argument("--latency-frames", type=int, default=5,
                    help="single-frame renders timed after the run (wall-clock latency of one frame)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "traffic_round1.json"),
                    help="PMC-measured HBM bytes per trace launch (rocprofv3 FETCH_SIZE/WRITE_SIZE), if present")
    return ap.parse_args()


def _cores():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))  # the GPU box's CPU share is 16


def cpu_baseline(s, scene, w, h, bdepth, target_s):
    """CPU leg on this host's cores over a bounded, evenly spaced row sample of the same frame.

    Prefers the UNMODIFIED reference (oracle/_ref/refharness, built from /root/reference/src
    by `make -C oracle ref`; its fork-parallel pixel loop = one reference process per core);
    falls back to the bit-exact CPU restatement oracle/ (\"port\").  Rays in the sample are
    the kernels' counts for the same rows (equal to the reference's, see tests)."""
    import subprocess
    import rtamd
    cores = _cores()
    harness = os.path.join(REPO, "oracle", "_ref", "refharness")
    kind = "reference" if os.access(harness, os.X_OK) else "port"
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
            return {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": cores, "kind": kind,
                    "sample": f"{what}, brute-force face loop, on {n} rows (every {step}th) of the same {w}x{h} "
                              f"frame: {rays} rays in {dt:.1f} s wall (incl. scene parse)"}
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


def main():
    a = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import torch
    import torch.distributed as dist
    import rtamd
    from cases import CONFIGS, SCENES, option_kwargs

    if a.backend == "gloo":
        local = local % torch.cuda.device_count()  # rehearsal: several ranks may share a GPU
    torch.cuda.set_device(local)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    scene_rel, W, H, flags = CONFIGS[a.config]
    kw = option_kwargs(flags)
    scene = os.path.join(SCENES, scene_rel)
    s = rtamd.load_scene(scene, device=local)
    s.upload()
    n_max = -(-H // world)
    F = max(1, a.frames_per_gpu)
    outs = [torch.empty((H, W, 3), dtype=torch.float64, device="cuda") for _ in range(F)]
    # RGB8 output double-buffered: the gathers of step i (side stream) overlap the render of i+1
    out8s = [[torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(F)] for _ in range(2)]
    gathered = [None, None]
    comm = torch.cuda.Stream() if world > 1 else torch.cuda.current_stream()
    prm = s.params(W, H, kw["bdepth"], kw["intersection_only"], 0, H, 1)  # every row, once per step
    stream = torch.cuda.current_stream().cuda_stream
    gather = [torch.empty((n_max, W, 3), dtype=torch.uint8, device="cuda") for _ in range(world)] \
        if rank == 0 and world > 1 else None
    frames = [torch.empty((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(world)] if rank == 0 else None
    from rtamd import dist as rd

    totals = {"rays": 0, "trace_rays": 0, "zero": 0, "ms": [0.0, 0.0, 0.0], "launches": [0, 0, 0], "bytes": [0, 0, 0],
              "flops": [0, 0, 0]}
    work = {}

    n_steps = [0]

    def step(record):
        # F x N frames per step (weak scaling): F renders of every row on this rank, pipelined
        # in one batch call; each render holds this rank's rows of N row-interleaved frames,
        # assembled on rank 0 by one RCCL gather of RGB8 rows per frame, on a side stream
        k = n_steps[0] % 2
        n_steps[0] += 1
        if gathered[k] is not None:  # the gathers that read these buffers two steps ago
            torch.cuda.current_stream().wait_event(gathered[k])
        st = s.render_batch_device([prm] * F, [o.data_ptr() for o in outs], [o.data_ptr() for o in out8s[k]],
                                   stream)
        rendered = torch.cuda.Event()
        rendered.record()
        with torch.cuda.stream(comm):
            comm.wait_event(rendered)
            for f in range(F):
                rd.gather_batch(out8s[k][f], H, dst=0, frames=frames, bufs=gather)
            gathered[k] = torch.cuda.Event()
            gathered[k].record(comm)
        if record:
            totals["rays"] += st.trace_rays + st.shadow_rays
            totals["trace_rays"] += st.trace_rays
            totals["zero"] += st.shadow_rays_zero_terms
            for k in range(3):
                totals["ms"][k] += st.stage_ms[k]
                totals["launches"][k] += st.stage_launches[k]
            # SURVEY.md §8d algorithmic bytes, attributed to the kernel that moves them
            for k, nrays in ((0, st.trace_rays), (1, st.shadow_rays)):
                totals["bytes"][k] += (nrays * RAY_IO_BYTES + st.stage_node_visits[k] * NODE_BYTES +
                                       st.stage_tri_tests[k] * TRI_BYTES + st.stage_candidates[k] * NRM_BYTES)
                totals["flops"][k] += (st.stage_node_visits[k] * NODE_FLOPS + st.stage_tri_tests[k] * TRI_FLOPS +
                                       st.stage_candidates[k] * CAND_FLOPS + st.stage_sphere_tests[k] * SPHERE_FLOPS)
            totals["bytes"][2] += st.pixels * PIXEL_BYTES
            per = lambda xs: [x // F for x in xs]  # the batch's F renders do identical work
            work.update({"trace_rays": st.trace_rays // F, "shadow_rays": st.shadow_rays // F,
                         "shadow_rays_zero_terms": st.shadow_rays_zero_terms // F,
                         "node_visits": per(st.stage_node_visits), "tri_tests": per(st.stage_tri_tests),
                         "candidates": per(st.stage_candidates), "sphere_tests": per(st.stage_sphere_tests),
                         "bvh_traversals": per(st.stage_bvh_traversals),
                         "max_node_visits_per_ray": list(st.stage_max_node_visits)})

    for _ in range(a.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # wall-clock of ONE frame (this rank's rows, one render call, nothing else in flight)
    lat = []
    for _ in range(max(0, a.latency_frames)):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        s.render_device(prm, outs[0].data_ptr(), out8s[0][0].data_ptr(), stream)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t1)
    lat = sorted(lat)[len(lat) // 2] if lat else float("nan")
    agg = torch.tensor([elapsed, float(totals["rays"])] + totals["ms"] + [float(x) for x in totals["launches"]] +
                       [float(x) for x in totals["bytes"]] + [float(x) for x in totals["flops"]] +
                       [float(totals["trace_rays"]), lat, float(totals["zero"])], dtype=torch.float64, device="cuda")
    if world > 1:
        t_max = agg[0:1].clone()
        l_max = agg[15:16].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        dist.all_reduce(l_max, op=dist.ReduceOp.MAX)
        dist.all_reduce(agg, op=dist.ReduceOp.SUM)
        agg[0], agg[15] = t_max[0], l_max[0]
    v = agg.tolist()
    elapsed, rays, stage_ms, stage_launches, stage_bytes = v[0], v[1], v[2:5], v[5:8], v[8:11]
    stage_flops, trace_rays, latency, zero_rays = v[11:14], v[14], v[15], v[16]
    fps = world * F  # frames per step
    if rank == 0:
        value = rays / elapsed / 1e6
        names = ["k_closest", "k_shadow", "k_shade"]
        dom = max(range(3), key=lambda k: stage_ms[k])  # the dominant kernel
        kms, launches, nbytes = stage_ms[dom], stage_launches[dom], stage_bytes[dom]
        achieved = (nbytes / launches) / ((kms / launches) * 1e-3) / 1e9 if launches else 0.0
        gflops = stage_flops[dom] / (kms * 1e-3) / 1e9 if kms else 0.0
        traffic = None
        if os.path.exists(a.traffic):
            try:
                traffic = json.load(open(a.traffic)).get("hbm_bytes_per_launch", {}).get(names[dom])
            except Exception:
                traffic = None
        res = {
            "metric": "Mrays/s (primary+secondary) and wall-clock at 1920x1080; HBM GB/s vs peak",
            "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "mrays_trace": round(trace_rays / elapsed / 1e6, 3),
            # rays that went through a traversal: the shadow rays decided by zero Phong terms
            #  count in `value` like every other ray the reference casts
            "mrays_traversed": round((rays - zero_rays) / elapsed / 1e6, 3),
            "vs_baseline": None, "dtype": "f64", "data": "synthetic: shipped reference scene data (bunny.obj), "
                                                        "deterministic, no RNG",
            "config": {"workload": a.config, "scene": scene_rel, "width": W, "height": H,
                       "bounce_depth": kw["bdepth"], "frames_per_step": fps, "frames_per_gpu_per_step": F,
                       "rays_per_frame": int(rays / a.steps / fps),
                       "ms_per_frame": round(elapsed / a.steps / fps * 1e3, 3),
                       "frame_latency_ms": round(latency * 1e3, 3),
                       "parallelism": (f"{fps} frames/step: {F} pipelined renders per GPU, each holding its rows of "
                                       f"{world} frames row-interleaved x{world} (rotated), RCCL gather of RGB8 rows")
                       if world > 1 else f"1 GPU, {F} frames/step pipelined (rt_render_batch_device)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": names[dom], "avg_launch_ms": round(kms / launches, 4) if launches else None,
                         "fp64": {"achieved": round(gflops / 1e3, 3), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                                  "frac": round(gflops / 1e3 / FP64_PEAK_TFLOPS, 4)},
                         "note": "algorithmic bytes per SURVEY.md §8d (ray I/O + LBVH nodes + triangles + normals), "
                                 "mostly L2/MALL-resident scene reads; kernel times are HIP-event spans of launches "
                                 "that run concurrently with other levels' kernels; see DESIGN.md",
                         "stages": {names[k]: {"ms_per_frame": round(stage_ms[k] / a.steps / fps, 4),
                                               "launches_per_frame": stage_launches[k] / a.steps / fps,
                                               "GBps": round(stage_bytes[k] / (stage_ms[k] * 1e-3) / 1e9, 1)
                                               if stage_ms[k] else None} for k in range(3)},
                         "work_per_frame_rank0": work},
        }
        if world == 1 and not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(s, scene, W, H, kw["bdepth"], a.cpu_seconds)
            same = same_algorithm_baseline(scene, W, H, kw["bdepth"], a.cpu_seconds / 3)
            if same:
                res["cpu_baseline"]["same_algorithm"] = same
        print(json.dumps(res), flush=True)
    s.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
