"""Per-kernel scalar-memory and instruction-fetch table of tools/profile_sqc.sh's passes:
counters summed over every dispatch of a variant (tools/kname.py names); the derived latency
counters (cycles, per dispatch) averaged over dispatches; kernel time from each pass's trace.

usage: python tools/sqc_table.py gpurun_out/<tag> > profiles/round5/sqc.json"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kname import parse  # noqa: E402

LAT = ("SmemLatency", "InstrFetchLatency", "VmemLatency")


def main():
    d = sys.argv[1]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    lat = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(float)
    for p in sorted(glob.glob(os.path.join(d, "p*", ""))):
        for cc in glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True):
            per = collections.defaultdict(float)
            keys = {}
            for r in csv.DictReader(open(cc)):
                v = parse(r["Kernel_Name"])[1]
                if not v:
                    continue
                per[(v, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
                keys[r["Dispatch_Id"]] = v
            for (v, _, c), x in per.items():
                (lat[v][c].append(x) if c in LAT else tot[v].__setitem__(c, tot[v][c] + x))
        if p.endswith("p1/"):
            for kt in glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True):
                for r in csv.DictReader(open(kt)):
                    v = parse(r["Kernel_Name"])[1]
                    if v:
                        dur[v] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {"source": d, "kernels": {}}
    for v in sorted(dur, key=lambda k: -dur[k]):
        c = tot[v]
        row = {"s": round(dur[v], 6)}
        for k in LAT:
            if lat[v][k]:
                row[k] = round(sum(lat[v][k]) / len(lat[v][k]), 1)
        if c.get("SQ_WAVE_CYCLES"):
            row["smem_per_kcycle"] = round(1e3 * c["SQ_INSTS_SMEM"] / c["SQ_WAVE_CYCLES"], 2)
        if c.get("SQC_DCACHE_REQ"):
            row["dcache_hit"] = round(c["SQC_DCACHE_HITS"] / c["SQC_DCACHE_REQ"], 3)
            row["dcache_miss"] = round(c["SQC_DCACHE_MISSES"] / c["SQC_DCACHE_REQ"], 3)
            row["dcache_miss_dup"] = round(c["SQC_DCACHE_MISSES_DUPLICATE"] / c["SQC_DCACHE_REQ"], 3)
        if c.get("SQC_ICACHE_REQ"):
            row["icache_hit"] = round(c["SQC_ICACHE_HITS"] / c["SQC_ICACHE_REQ"], 3)
            row["icache_miss"] = round(c["SQC_ICACHE_MISSES"] / c["SQC_ICACHE_REQ"], 4)
        if dur[v]:
            # per-second rates over the 8 XCDs (the SQC counters sum every instance)
            for k in ("SQC_DCACHE_REQ", "SQC_ICACHE_REQ", "SQC_TC_STALL", "SQC_DCACHE_BUSY_CYCLES",
                      "SQC_ICACHE_BUSY_CYCLES", "SQC_TC_DATA_READ_REQ", "SQC_TC_INST_REQ"):
                if k in c:
                    row[k + "_per_us"] = round(c[k] / dur[v] / 1e6, 1)
        row["raw"] = {k: c[k] for k in sorted(c)}
        out["kernels"][v] = row
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
