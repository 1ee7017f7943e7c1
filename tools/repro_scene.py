"""Renders one scene on the GPU under environment variants (each in its own process: the
library reads its knobs at scene creation) and counts the pixels that differ from the CPU
oracle, render by render (a parity-failure bisection aid).

usage: python tools/repro_scene.py scene.rti W H bdepth io(0/1) [VAR=V[,VAR=V]] ..."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import os, sys, json
import numpy as np
sys.path.insert(0, os.path.join(%r, "cs184-raytracer_amd")); sys.path.insert(0, os.path.join(%r, "oracle"))
import rtamd, pyoracle
path, w, h, bd, io = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), bool(int(sys.argv[5]))
want, _ = pyoracle.render(path, w, h, bdepth=bd, intersection_only=io)
s = rtamd.load_scene(path)
o = rtamd.Options(renderWidth_=w, renderHeight_=h, bounceDepth_=bd, intersectionOnly_=io)
res = []
for k in range(3):
    got = s.renderScene(options=o)
    d = (np.ascontiguousarray(got).view(np.uint64) != np.ascontiguousarray(want).view(np.uint64)).any(axis=2)
    ys, xs = np.nonzero(d)
    res.append({"diff": int(d.sum()), "first": [(int(y), int(x)) for y, x in zip(ys[:6], xs[:6])],
                "max_got": float(np.max(got)), "max_want": float(np.max(want))})
s.close()
print(json.dumps(res))
""" % (REPO, REPO)

path, w, h, bd, io = sys.argv[1:6]
for v in [""] + sys.argv[6:]:
    env = dict(os.environ)
    for kv in filter(None, v.split(",")):
        k, val = kv.split("=", 1)
        env[k] = val
    p = subprocess.run([sys.executable, "-c", CHILD, path, w, h, bd, io], env=env, capture_output=True, text=True,
                       timeout=300)
    print(v or "default", p.stdout.strip() if p.returncode == 0 else "FAILED " + p.stderr[-500:], flush=True)
