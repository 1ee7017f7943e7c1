"""CLI (bin/rtamd) wall-clock and phase A/B under environment variants, rounds alternating on one
box: median process wall and median of each --timing phase per config and variant.

usage: python tools/cli_ab.py <rounds> <config[,config...]> [VAR=V[,VAR=V]] ...
       (the first variant is always the default environment)"""
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
from rtamd.configs import CONFIGS, SCENES  # noqa: E402

CLI = os.path.join(REPO, "cs184-raytracer_amd", "bin", "rtamd")


def main():
    rounds, configs = int(sys.argv[1]), sys.argv[2].split(",")
    variants = [""] + sys.argv[3:]
    res = {v: {c: [] for c in configs} for v in variants}
    with tempfile.TemporaryDirectory() as d:
        for _ in range(rounds):
            for v in variants:
                env = dict(os.environ)
                for kv in filter(None, v.split(",")):
                    k, val = kv.split("=", 1)
                    env[k] = val
                for c in configs:
                    scene, w, h, flags = CONFIGS[c]
                    t0 = time.perf_counter()
                    subprocess.run([CLI, os.path.join(SCENES, scene), "-w", str(w), "-h", str(h), *flags, "-o",
                                    os.path.join(d, "o.png"), "--timing", os.path.join(d, "t.json")], env=env,
                                   check=True, capture_output=True, timeout=120)
                    ph = json.load(open(os.path.join(d, "t.json")))
                    ph["wall_ms"] = (time.perf_counter() - t0) * 1e3
                    res[v][c].append(ph)
    for v in variants:
        out = {}
        for c in configs:
            keys = res[v][c][0].keys()
            out[c] = {k: round(statistics.median(r[k] for r in res[v][c]), 2) for k in keys}
        print("median", v or "default", json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
