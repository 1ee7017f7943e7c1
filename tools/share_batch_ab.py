"""Batch of F frames' row shares (one rank's k/n share, the bench's partition mode) or whole
frames, one rt_render_batch_device call, median ms over reps, under environment variants
(each in its own process), rounds alternating on one box.

usage: python tools/share_batch_ab.py <rounds> <config>[@k/n][:F][,...] [VAR=V[,VAR=V]] ..."""
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import os, sys, time, json, statistics
sys.path.insert(0, os.path.join(%r, "cs184-raytracer_amd"))
import torch, rtamd
from rtamd.configs import CONFIGS, SCENES, option_kwargs
res = {}
for name in sys.argv[1].split(","):
    spec, _, nf = name.partition(":")
    F = int(nf or 48)
    cfg, _, share = spec.partition("@")
    scene, w, h, flags = CONFIGS[cfg]
    kw = option_kwargs(flags)
    s = rtamd.load_scene(os.path.join(SCENES, scene))
    prm = s.params(w, h, kw["bdepth"], kw["intersection_only"], 0, h, 1)
    rows = h
    if share:
        k, n = (int(v) for v in share.split("/"))
        prm = s.params(w, h, kw["bdepth"], kw["intersection_only"], k * 8, h, n, row_block=8)
        rows = sum(min(8, h - r) for r in range(k * 8, h, n * 8))
    outs = torch.empty((F, rows, w, 3), dtype=torch.uint8, device="cuda")
    ptrs = [outs[f].data_ptr() for f in range(F)]
    stream = torch.cuda.current_stream().cuda_stream
    ts = []
    for i in range(int(sys.argv[2]) + 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = s.render_batch_device([prm] * F, [], ptrs, stream)
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(time.perf_counter() - t0)
    res[name] = {"ms": round(statistics.median(ts) * 1e3, 3), "mrays_s": round(st.rays / statistics.median(ts) / 1e6, 1)}
    s.close()
print(json.dumps(res))
""" % REPO


def main():
    rounds, configs = int(sys.argv[1]), sys.argv[2]
    variants = [""] + sys.argv[3:]
    reps = int(os.environ.get("REPS", "7"))
    acc = {v: {} for v in variants}
    for r in range(rounds):
        for v in variants:
            env = dict(os.environ)
            for kv in filter(None, v.split(",")):
                k, val = kv.split("=", 1)
                env[k] = val
            p = subprocess.run([sys.executable, "-c", CHILD, configs, str(reps)], env=env, capture_output=True, text=True,
                               timeout=300)
            if p.returncode:
                sys.stderr.write(p.stderr)
                sys.exit(p.returncode)
            res = json.loads(p.stdout.strip().splitlines()[-1])
            print(r, v or "default", json.dumps(res), flush=True)
            for c, m in res.items():
                acc[v].setdefault(c, []).append(m["ms"])
    for v in variants:
        print("median", v or "default", json.dumps({c: statistics.median(m) for c, m in acc[v].items()}))


if __name__ == "__main__":
    main()
