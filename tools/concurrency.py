"""Kernel concurrency of a rocprofv3 kernel trace (the throughput schedule): over the span
of the trace's last `frac` of kernels, the fraction of time with >= 1 kernel running and
the time-weighted histogram of running kernels.
usage: python tools/concurrency.py <kernel_trace.csv> [frac]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
ev = ev[int(len(ev) * (1 - frac)):]
t0, t1 = ev[0][0], max(e[1] for e in ev)
pts = []
for s, e, _ in ev:
    pts.append((s, 1))
    pts.append((e, -1))
pts.sort()
hist = {}
cur, last = 0, t0
for t, d in pts:
    if t > last:
        hist[cur] = hist.get(cur, 0) + (t - last)
    cur += d
    last = t
span = t1 - t0
print(f"span {span / 1e6:.3f} ms over {len(ev)} kernels; idle {hist.get(0, 0) / span:.3f}")
for k in sorted(hist):
    print(f"  {k:2d} running: {hist[k] / span:.3f}")
