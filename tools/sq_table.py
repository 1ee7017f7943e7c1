"""Per-kernel SQ issue/stall table of a single-frame profile (tools/profile_c5.sh): kernel time
share from the kernel trace, and from the --pmc passes (summed over every dispatch of the
variant, tools/kname.py names) VALU busy, s_waitcnt wait and issue-stall fractions of wave
time, and lane utilisation.

usage: python tools/sq_table.py gpurun_out/<tag> > profiles/<round>/<name>.json"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kname import parse  # noqa: E402

N_CU = 256


def one(pattern):
    f = glob.glob(pattern, recursive=True)
    return f[0] if f else None


def main():
    d = sys.argv[1]
    ms = collections.defaultdict(float)
    calls = collections.Counter()
    for r in csv.DictReader(open(one(os.path.join(d, "kt", "**", "*kernel_trace.csv")))):
        v = parse(r["Kernel_Name"])[1]
        if v:
            ms[v] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            calls[v] += 1
    total = sum(ms.values())
    # counters per pass: SQ_ACTIVE_INST_VALU is collected in both passes, so every ratio takes
    # its numerator and denominator from the same pass (round 4's table summed the two passes'
    # SQ_ACTIVE_INST_VALU, doubling valu_busy and halving lane_util)
    ctr = {sub: collections.defaultdict(lambda: collections.defaultdict(float)) for sub in ("sq", "sq2")}
    dur = collections.defaultdict(float)
    for sub in ("sq", "sq2"):
        cc = one(os.path.join(d, sub, "**", "*counter_collection.csv"))
        if not cc:
            continue
        for r in csv.DictReader(open(cc)):
            v = parse(r["Kernel_Name"])[1]
            if v:
                ctr[sub][v][r["Counter_Name"]] += float(r["Counter_Value"])
        kt = one(os.path.join(d, sub, "**", "*kernel_trace.csv"))
        if kt and sub == "sq":
            seen = set()
            for r in csv.DictReader(open(kt)):
                v = parse(r["Kernel_Name"])[1]
                if v and r["Dispatch_Id"] not in seen:
                    seen.add(r["Dispatch_Id"])
                    dur[v] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {"source": d, "kernel_ms_total": round(total, 3), "kernels": {}}
    for v in sorted(ms, key=lambda k: -ms[k]):
        c, c2 = ctr["sq"].get(v, {}), ctr["sq2"].get(v, {})
        row = {"launches": calls[v], "ms": round(ms[v], 3), "share": round(ms[v] / total, 4)}
        if c.get("SQ_WAVE_CYCLES"):
            row.update({"valu_busy": round(c["SQ_ACTIVE_INST_VALU"] / (N_CU * dur[v] * 2.4e9), 3) if dur[v] else None,
                        "wait_any": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3),
                        "wait_inst_any": round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 3),
                        "valu_instr": c["SQ_INSTS_VALU"], "salu_per_valu": round(c["SQ_INSTS_SALU"] / c["SQ_INSTS_VALU"], 3)})
        if c2.get("SQ_THREAD_CYCLES_VALU") and c2.get("SQ_ACTIVE_INST_VALU"):
            row["lane_util"] = round(c2["SQ_THREAD_CYCLES_VALU"] / c2["SQ_ACTIVE_INST_VALU"] / 64, 3)
        out["kernels"][v] = row
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
