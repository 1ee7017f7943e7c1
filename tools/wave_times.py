"""Per-wave timing of single frames (diagnostic build with -DRT_DIAG_WAVETIME=1:
tools/build_variant.sh wt -DRT_DIAG_WAVETIME=1): for each traversal launch of the last of a
few renders, the launch's span, the histogram of its waves' durations, when its waves start
(a second round of waves starts late), and its slowest waves with their packet node
iterations, face tests and 8x8 tile (level-0 packets).

usage: RTAMD_LIB=cs184-raytracer_amd/rtamd/var/librtamd_wt.so \\
       python tools/wave_times.py <config>[@k/n] [...] > profiles/round5/wave_times_<name>.json"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
import torch  # noqa: E402
import rtamd  # noqa: E402
from rtamd.configs import CONFIGS, SCENES, option_kwargs  # noqa: E402

REC = np.dtype([("t0", "<u8"), ("t1", "<u8"), ("tag", "<u4"), ("item", "<u4"), ("nodes", "<u4"), ("faces", "<u4")])
KERNEL = {1: "k_closest", 2: "k_fused", 3: "k_shadow"}
MAXREC = 1 << 18


def records(L):
    buf = np.zeros(MAXREC, dtype=REC)
    n = L.rt_debug_wave_times(0, buf.ctypes.data_as(ctypes.c_void_p), MAXREC)
    if n < 0:
        raise RuntimeError(rtamd.lib().rt_last_error())
    return buf[:n]


def main():
    L = rtamd.lib()
    L.rt_debug_wave_times.restype = ctypes.c_int
    L.rt_debug_wave_times.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    out = {}
    for name in sys.argv[1:]:
        cfg, _, share = name.partition("@")
        scene, w, h, flags = CONFIGS[cfg]
        kw = option_kwargs(flags)
        s = rtamd.load_scene(os.path.join(SCENES, scene))
        img = torch.empty((h, w, 3), dtype=torch.float64, device="cuda")
        prm = s.params(w, h, kw["bdepth"], kw["intersection_only"], 0, h, 1)
        if share:
            k, n = (int(v) for v in share.split("/"))
            prm = s.params(w, h, kw["bdepth"], kw["intersection_only"], k * 8, h, n, row_block=8)
        for _ in range(4):
            s.render_device(prm, img.data_ptr())
            torch.cuda.synchronize()
            r = records(L)  # the last render's records
        s.close()
        if not len(r):
            raise SystemExit("no wave records: not an RT_DIAG_WAVETIME build")
        t00 = int(r["t0"].min())
        res = {"waves": int(len(r)), "frame_span_us": round((int(r["t1"].max()) - t00) / 100, 2), "launches": []}
        for tag in sorted(set(r["tag"].tolist())):
            q = r[r["tag"] == tag]
            dur = (q["t1"] - q["t0"]).astype(np.float64) / 100  # us
            start = (q["t0"] - t00).astype(np.float64) / 100
            end = (q["t1"] - t00).astype(np.float64) / 100
            order = np.argsort(-dur)[:10]
            ent = {"kernel": KERNEL.get(tag & 15, str(tag & 15)), "packet": bool(tag >> 4 & 1), "level": int(tag >> 8),
                   "waves": int(len(q)), "first_start_us": round(float(start.min()), 2),
                   "last_end_us": round(float(end.max()), 2),
                   "wave_us": {p: round(float(np.percentile(dur, v)), 2) for p, v in
                               (("p10", 10), ("p50", 50), ("p90", 90), ("p99", 99), ("max", 100))},
                   "start_us": {p: round(float(np.percentile(start, v)), 2) for p, v in
                                (("p50", 50), ("p90", 90), ("max", 100))},
                   "nodes_per_wave": {p: float(np.percentile(q["nodes"], v)) for p, v in (("p50", 50), ("p90", 90), ("max", 100))},
                   "hist_us": np.histogram(dur, bins=10)[0].tolist(),
                   "hist_edges_us": [round(float(e), 1) for e in np.histogram(dur, bins=10)[1]],
                   "slowest": [{"us": round(float(dur[i]), 2), "start_us": round(float(start[i]), 2),
                                "item": int(q["item"][i]), "tile": int(q["item"][i]) // 64,
                                "nodes": int(q["nodes"][i]), "faces": int(q["faces"][i])} for i in order]}
            # correlation of a wave's duration with its node iterations
            if q["nodes"].max() > 0:
                ent["corr_us_nodes"] = round(float(np.corrcoef(dur, q["nodes"].astype(np.float64))[0, 1]), 3)
            res["launches"].append(ent)
        out[name] = res
        print(json.dumps({name: res}), flush=True)


if __name__ == "__main__":
    main()
