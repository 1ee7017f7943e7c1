"""Batch throughput of one config with every frame cut into `world` bands handed to the batch
call in a given band order (jobs of one frame's row range each, outputs at the band's rows):
does the order in which a chunk holds the image's rows change the rate?  (round 6: the
8-way shares of bench.py's partition, profiles/round6/ab/README.md)

usage: python tools/order_probe.py <config> [frames] [reps] [order,order,...]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
import torch  # noqa: E402
import rtamd  # noqa: E402
from rtamd import dist as rd  # noqa: E402
from rtamd.configs import CONFIGS, SCENES, option_kwargs  # noqa: E402

name = sys.argv[1]
F = int(sys.argv[2]) if len(sys.argv) > 2 else 48
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 8
scene, W, H, flags = CONFIGS[name]
kw = option_kwargs(flags)
s = rtamd.load_scene(os.path.join(SCENES, scene))
s.upload()
n = 8
bh = rd.band_rows(H, n)
bands = [(k * bh, min(H, (k + 1) * bh)) for k in range(n)]
out8 = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
orders = {"whole": None, "natural": list(range(n)), "shift4": [4, 5, 6, 7, 0, 1, 2, 3],
          "reverse": list(range(n - 1, -1, -1)), "interleave": [0, 4, 1, 5, 2, 6, 3, 7],
          "outside_in": [0, 7, 1, 6, 2, 5, 3, 4], "middle_out": [3, 4, 2, 5, 1, 6, 0, 7]}
# per-band cost: every frame's band k alone (48 jobs of one band), ms per call
band_ms = []
for k in range(n):
    b, e = bands[k]
    prms = [s.params(W, H, kw["bdepth"], kw["intersection_only"], b, e, 1)] * F
    ptrs = [out8[f, b].data_ptr() for f in range(F)]
    ts = []
    for rep in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.render_batch_device(prms, [], ptrs, stream)
        torch.cuda.synchronize()
        if rep:
            ts.append(time.perf_counter() - t0)
    band_ms.append(round(sorted(ts)[len(ts) // 2] * 1e3, 3))
print(name, "band ms", band_ms, flush=True)
orders["lpt"] = sorted(range(n), key=lambda k: -band_ms[k])     # most expensive first
orders["spt"] = sorted(range(n), key=lambda k: band_ms[k])      # cheapest first
if len(sys.argv) > 4:
    orders = {k: orders[k] for k in sys.argv[4].split(",")}
res = {}
for rnd in range(2):
    for tag, order in orders.items():
        if order is None:
            prms = [s.params(W, H, kw["bdepth"], kw["intersection_only"], 0, H, 1)] * F
            ptrs = [out8[f].data_ptr() for f in range(F)]
        else:
            prms, ptrs = [], []
            for f in range(F):
                for k in order:
                    b, e = bands[k]
                    prms.append(s.params(W, H, kw["bdepth"], kw["intersection_only"], b, e, 1))
                    ptrs.append(out8[f, b].data_ptr())
        ts = []
        for rep in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st = s.render_batch_device(prms, [], ptrs, stream)
            torch.cuda.synchronize()
            if rep:
                ts.append(time.perf_counter() - t0)
        ts.sort()
        ms = ts[len(ts) // 2] * 1e3
        res.setdefault(tag, []).append(round(st.rays / ms / 1e3, 1))
        print(name, rnd, tag, round(ms, 3), "ms", round(st.rays / ms / 1e3, 1), "Mrays/s", flush=True)
print("summary", name, res)
s.close()
