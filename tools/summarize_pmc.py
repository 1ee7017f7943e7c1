"""Summarises rocprofv3 --pmc CSVs per kernel (mean counter value per dispatch).
usage: python tools/summarize_pmc.py gpurun_out/<tag>/p*/pmc_counter_collection.csv"""
import collections
import csv
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        m = re.search(r"(k_[a-z0-9_]+(?:<[a-z]+>)?)\(", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:24]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-28s n=%-4d mean=%.4g  sum=%.4g" % (c, len(v), sum(v) / len(v), sum(v)))
