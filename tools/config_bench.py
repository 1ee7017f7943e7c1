"""Mrays/s of every BASELINE.json config on one GPU (render into HBM, as bench.py).

usage: python tools/config_bench.py [repeats]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import rtamd  # noqa: E402
from cases import CONFIGS, SCENES, option_kwargs  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for name, (scene, w, h, flags) in CONFIGS.items():
    kw = option_kwargs(flags)
    s = rtamd.load_scene(os.path.join(SCENES, scene))
    s.upload()
    out = torch.empty((h, w, 3), dtype=torch.float64, device="cuda")
    out8 = torch.empty((h, w, 3), dtype=torch.uint8, device="cuda")
    prm = s.params(w, h, kw["bdepth"], kw["intersection_only"], 0, h, 1)
    st = s.render_device(prm, out.data_ptr(), out8.data_ptr())  # warm-up (allocations)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        st = s.render_device(prm, out.data_ptr(), out8.data_ptr())
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print(json.dumps({"config": name, "width": w, "height": h, "flags": flags, "ms_per_frame": round(dt * 1e3, 3),
                      "rays": st.rays, "trace_rays": st.trace_rays, "shadow_rays": st.shadow_rays,
                      "Mrays_per_s": round(st.rays / dt / 1e6, 1)}), flush=True)
    s.close()
