"""Per-kernel vector instructions (wave-instructions) per frame from tools/valu_breakdown.sh
output: one column per build.   usage: python tools/valu_table.py gpurun_out/<tag> [frames]"""
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 6
cols = {}
for path in sorted(glob.glob(os.path.join(root, "*", "pmc_counter_collection.csv"))):
    v = os.path.basename(os.path.dirname(path))
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        m = re.search(r"(k_[a-z0-9_]+(?:<[a-z]+>)?)\(", r["Kernel_Name"])
        if m:
            acc[(m.group(1), r["Counter_Name"])] += float(r["Counter_Value"])
    cols[v] = acc
names = ["default"] + sorted(k for k in cols if k != "default")
kernels = sorted({k for c in cols.values() for (k, _) in c})
for ctr in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES"):
    print(f"{ctr} per frame (millions)")
    print("%-18s" % "kernel" + "".join("%12s" % n[:11] for n in names))
    tot = collections.Counter()
    for k in kernels:
        row = [cols[n].get((k, ctr), 0.0) / frames / 1e6 for n in names]
        for n, x in zip(names, row):
            tot[n] += x
        print("%-18s" % k + "".join("%12.2f" % x for x in row))
    print("%-18s" % "total" + "".join("%12.2f" % tot[n] for n in names))
