"""Per-kernel timeline of the last rendered frame from a rocprofv3 kernel trace CSV.
usage: python tools/frame_timeline.py <kernel_trace.csv>"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))


def name(r):
    m = re.search(r"(k_[a-z0-9_]+(?:<[a-z0-9, ]+>)?)\(", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"][:20]


names = [name(r) for r in rows]
outs = [i for i, n in enumerate(names) if n.startswith("k_output")]
a, b = outs[-2] + 1, outs[-1]
t0 = int(rows[a]["Start_Timestamp"])
busy = 0
for i in range(a, b + 1):
    r = rows[i]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{names[i]:20s} grid={r['Grid_Size_X']:>9s} start={(s - t0) / 1e3:8.1f}us dur={(e - s) / 1e3:8.1f}us")
span = int(rows[b]["End_Timestamp"]) - t0
print(f"frame span {span / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us ({100 * busy / span:.0f}%)")
