"""Every BASELINE.json config on one GPU: the render into HBM (as bench.py) and the drop-in's
whole process (`bin/rtamd <scene> -w -h -o out.png`, the reference's `as2` invocation,
main.cpp:40-85, whose wall-clock is the reference's only published figure,
notes/notes-02.txt:8).

For each config one JSON line: ms_per_frame (back-to-back renders into HBM, no host copy),
frame_latency_ms (median of single renders, each synchronised), and cli_wall_ms (median
process wall-clock of the CLI, spawn to exit) with cli_phases, the CLI's own --timing split
of its host time (HIP runtime start, parse, LBVH build, HBM upload, render, device-to-host
copy, PNG encode + write, teardown).

usage: python tools/config_bench.py [repeats] [cli_runs]"""
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import rtamd  # noqa: E402
from cases import CONFIGS, SCENES, option_kwargs  # noqa: E402

CLI = os.path.join(REPO, "cs184-raytracer_amd", "bin", "rtamd")


def cli_run(scene, w, h, flags, runs):
    """Median wall-clock of `runs` CLI processes and the phases of that run."""
    walls, phases = [], []
    with tempfile.TemporaryDirectory() as d:
        for _ in range(runs):
            t0 = time.perf_counter()
            subprocess.run([CLI, os.path.join(SCENES, scene), "-w", str(w), "-h", str(h), *flags, "-o",
                            os.path.join(d, "out.png"), "--timing", os.path.join(d, "t.json")],
                           check=True, capture_output=True)
            walls.append((time.perf_counter() - t0) * 1e3)
            phases.append(json.load(open(os.path.join(d, "t.json"))))
    k = walls.index(statistics.median_low(walls))
    flat = {n: v for n, v in phases[k].items() if n != "detail"}
    flat.update({"detail." + n: v for n, v in phases[k].get("detail", {}).items()})
    return round(walls[k], 2), {n: round(v, 3) for n, v in flat.items()}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    cli_runs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    for name, (scene, w, h, flags) in CONFIGS.items():
        kw = option_kwargs(flags)
        s = rtamd.load_scene(os.path.join(SCENES, scene))
        s.upload()
        out = torch.empty((h, w, 3), dtype=torch.float64, device="cuda")
        out8 = torch.empty((h, w, 3), dtype=torch.uint8, device="cuda")
        prm = s.params(w, h, kw["bdepth"], kw["intersection_only"], 0, h, 1)
        for _ in range(2):  # warm-up (allocations, the launch plan)
            st = s.render_device(prm, out.data_ptr(), out8.data_ptr())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            st = s.render_device(prm, out.data_ptr(), out8.data_ptr())
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        lat = []
        for _ in range(max(5, reps)):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            s.render_device(prm, out.data_ptr(), out8.data_ptr())
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t1)
        info = s.info()
        s.close()
        rec = {"config": name, "width": w, "height": h, "flags": flags, "ms_per_frame": round(dt * 1e3, 3),
               "frame_latency_ms": round(statistics.median(lat) * 1e3, 4),
               "rays": st.rays, "trace_rays": st.trace_rays, "shadow_rays": st.shadow_rays,
               "Mrays_per_s": round(st.rays / dt / 1e6, 1),
               # HBM the scene and the ray-level buffers hold after these renders (two lanes
               # for a multi-chunk frame keep two sets of level buffers)
               "scene_bytes": info.device_bytes, "level_bytes": info.level_bytes}
        if cli_runs > 0 and os.access(CLI, os.X_OK):
            rec["cli_wall_ms"], rec["cli_phases"] = cli_run(scene, w, h, flags, cli_runs)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
