"""Renders one BASELINE.json config `reps` times into HBM (for rocprofv3 timelines).

usage: python tools/one_config.py <config> [reps] [k/n]   (k/n: rank k's 8-row-block share of an
n-way partition, as bench.py's strong-scaling sweep renders it)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
import torch  # noqa: E402
import rtamd  # noqa: E402
from rtamd.configs import CONFIGS, SCENES, option_kwargs  # noqa: E402

name = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
scene, w, h, flags = CONFIGS[name]
kw = option_kwargs(flags)
s = rtamd.load_scene(os.path.join(SCENES, scene))
out = torch.empty((h, w, 3), dtype=torch.float64, device="cuda")
out8 = torch.empty((h, w, 3), dtype=torch.uint8, device="cuda")
prm = s.params(w, h, kw["bdepth"], kw["intersection_only"], 0, h, 1)
if len(sys.argv) > 3:
    k, n = (int(v) for v in sys.argv[3].split("/"))
    prm = s.params(w, h, kw["bdepth"], kw["intersection_only"], k * 8, h, n, row_block=8)
ts = []
for _ in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.render_device(prm, out.data_ptr(), out8.data_ptr())
    ts.append(time.perf_counter() - t0)
print(name, [round(t * 1e3, 3) for t in ts])
s.close()
