"""Level-buffer HBM of the BASELINE configs (rt_scene_info.level_bytes after the renders, and
the peak during them) with the frame time and the f64 image hash against the reference's
golden (tests/golden/ref_hashes.json).  RTAMD_LEVEL_BUDGET in the environment applies.

usage: python tools/level_bytes.py [frames] [config ...]"""
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
import torch  # noqa: E402
import rtamd  # noqa: E402
from rtamd.configs import CONFIGS, SCENES, option_kwargs  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 3
names = sys.argv[2:] or list(CONFIGS)
gold = json.load(open(os.path.join(REPO, "tests", "golden", "ref_hashes.json")))["configs"]
for name in names:
    scene, w, h, flags = CONFIGS[name]
    kw = option_kwargs(flags)
    s = rtamd.load_scene(os.path.join(SCENES, scene))
    s.upload()
    out = torch.empty((h, w, 3), dtype=torch.float64, device="cuda")
    prm = s.params(w, h, kw["bdepth"], kw["intersection_only"], 0, h, 1)
    ts = []
    for _ in range(frames):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.render_device(prm, out.data_ptr())
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    sha = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
    inf = s.info()
    print(json.dumps({"config": name, "level_bytes": inf.level_bytes, "level_gib": round(inf.level_bytes / 2**30, 3),
                      "level_peak_gib": round(inf.level_bytes_peak / 2**30, 3), "budget": inf.level_budget,
                      "ms": [round(t, 3) for t in ts], "parity": sha == gold[name]["f64_sha256"]}), flush=True)
    s.close()
