"""Single-frame latency of C3 after batches on the same scene (bench.py's order): a batch of
48 frames rendered 3 times, then `reps` single frames; prints the single-frame times (ms).
usage: python tools/lat_after_batch.py [reps]   (RTAMD_BATCH_LANES etc. from the environment)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
import torch  # noqa: E402
import rtamd  # noqa: E402
from rtamd.configs import CONFIGS, SCENES, option_kwargs  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
scene, W, H, flags = CONFIGS["C3_bunny_1920x1080_bd4"]
kw = option_kwargs(flags)
s = rtamd.load_scene(os.path.join(SCENES, scene))
s.upload()
F = 48
out8 = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
prm = s.params(W, H, kw["bdepth"], kw["intersection_only"], 0, H, 1)
for _ in range(3):
    s.render_batch_device([prm] * F, [], [out8[f].data_ptr() for f in range(F)], stream)
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.render_device(prm, 0, out8[0].data_ptr(), stream)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
print("single frames after batches (ms):", [round(t, 3) for t in ts], "median", round(sorted(ts)[len(ts) // 2], 3))
s.close()
