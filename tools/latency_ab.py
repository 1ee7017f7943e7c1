"""Single-frame latency A/B: median ms per frame of BASELINE.json configs under environment
variants (each variant in its own process, since the library reads its knobs at scene
creation), rounds alternating on one box.

usage: python tools/latency_ab.py <rounds> <config|scene.rti[:WxH][+bdN][@k/n][,...]> [VAR=V[,VAR=V]] ...
       (the first variant is always the default environment)"""
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys, time, json
sys.path.insert(0, os.path.join(%r, "cs184-raytracer_amd"))
import torch, rtamd
from rtamd.configs import CONFIGS, SCENES, option_kwargs
res = {}
for name in sys.argv[1].split(","):
    cfg, _, share = name.partition("@")
    cfg, _, bd = cfg.partition("+bd")  # +bdN: another bounce depth
    cfg, _, size = cfg.partition(":")  # cfg:WxH renders the config's scene and options at another size
    if cfg.endswith(".rti"):  # a shipped scene by file name (excess_inputs/ or inputs/), 1024^2, depth 10
        sub = "excess_inputs" if os.path.exists(os.path.join(SCENES, "excess_inputs", cfg)) else "inputs"
        scene, w, h, flags = os.path.join(sub, cfg), 1024, 1024, []
    else:
        scene, w, h, flags = CONFIGS[cfg]
    if size:
        w, h = (int(v) for v in size.split("x"))
    kw = option_kwargs(flags)
    if bd:
        kw["bdepth"] = int(bd)
    s = rtamd.load_scene(os.path.join(SCENES, scene))
    out = torch.empty((h, w, 3), dtype=torch.float64, device="cuda")
    out8 = torch.empty((h, w, 3), dtype=torch.uint8, device="cuda")
    prm = s.params(w, h, kw["bdepth"], kw["intersection_only"], 0, h, 1)
    if share:  # rank k's 8-row-block share of an n-way partition (bench.py's strong-scaling sweep)
        k, n = (int(v) for v in share.split("/"))
        prm = s.params(w, h, kw["bdepth"], kw["intersection_only"], k * 8, h, n, row_block=8)
    reps = int(sys.argv[2])
    ts = []
    for i in range(reps + 5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.render_device(prm, out.data_ptr(), out8.data_ptr())
        torch.cuda.synchronize()
        if i >= 5:
            ts.append(time.perf_counter() - t0)
    ts.sort()
    res[name] = round(ts[len(ts) // 2] * 1e3, 4)
    s.close()
print(json.dumps(res))
""" % REPO


def main():
    rounds = int(sys.argv[1])
    configs = sys.argv[2]
    variants = [""] + sys.argv[3:]
    reps = int(os.environ.get("REPS", "40"))
    acc = {v: {} for v in variants}
    for r in range(rounds):
        for v in variants:
            env = dict(os.environ)
            for kv in filter(None, v.split(",")):
                k, val = kv.split("=", 1)
                env[k] = val
            p = subprocess.run([sys.executable, "-c", CHILD, configs, str(reps)], env=env, capture_output=True,
                               text=True, timeout=300)
            if p.returncode:
                sys.stderr.write(p.stderr)
                sys.exit(p.returncode)
            res = json.loads(p.stdout.strip().splitlines()[-1])
            print(r, v or "default", json.dumps(res), flush=True)
            for c, ms in res.items():
                acc[v].setdefault(c, []).append(ms)
    for v in variants:
        print("median", v or "default", json.dumps({c: statistics.median(m) for c, m in acc[v].items()}))


if __name__ == "__main__":
    main()
