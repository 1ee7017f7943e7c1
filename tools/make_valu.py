"""VALU roof data from a tools/profile_round2.sh run: vector instructions per launch of every
kernel family in the solo pass, and the chip's sustained VALU issue rate (calibration).

usage: python tools/make_valu.py gpurun_out/<tag> profiles/<round>     -> <round>/valu.json

- solo: rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES over `bench.py --solo-only`
  (every kernel alone); SQ_INSTS_VALU counts wave64 vector instructions (issue events).
- calibration: the same counters over tools/valu_calibration.py: k_valu_peak runs chains of
  independent v_fma_f32 (and v_fma_f64) on every CU, 16 waves per CU; instructions / kernel
  duration (kernel trace of the same pass) is the sustained issue rate.  The f32 rate is the
  roof's peak: no vector instruction issues faster, so achieved / peak is an upper bound of
  the traversal kernels' issue-slot use (their fp64 work issues at the f64 rate or slower)."""
import collections
import csv
import json
import os
import re
import sys


def family(name):
    m = re.search(r"(k_[a-z0-9_]+)(?:<[^>]*>)?\(", name)
    return m.group(1) if m else None


def load(d):
    dur = {}
    for r in csv.DictReader(open(os.path.join(d, "pmc_kernel_trace.csv"))):
        dur[r["Dispatch_Id"]] = (r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    ctr = collections.defaultdict(dict)
    for r in csv.DictReader(open(os.path.join(d, "pmc_counter_collection.csv"))):
        ctr[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    return dur, ctr


def main():
    src, dst = sys.argv[1], sys.argv[2]
    dur, ctr = load(os.path.join(src, "valu_cal"))
    cal = {}
    for t in ("float", "double"):
        ids = sorted((int(i) for i, (n, _) in dur.items() if f"k_valu_peak<{t}>" in n))
        # dispatches: warm-up, 16 waves/CU, warm-up, 32 waves/CU
        for waves, i in ((16, str(ids[1])), (32, str(ids[3]))):
            instr, secs = ctr[i]["SQ_INSTS_VALU"], dur[i][1]
            cal[f"{t}_{waves}w"] = {"wave_instr": instr, "seconds": secs, "wave_instr_per_s": instr / secs}
    dur, ctr = load(os.path.join(src, "valu"))
    per = collections.defaultdict(list)
    waves = collections.defaultdict(list)
    for i, (n, _) in dur.items():
        f = family(n)
        if f and i in ctr:
            per[f].append(ctr[i]["SQ_INSTS_VALU"])
            waves[f].append(ctr[i].get("SQ_WAVES", 0.0))
    out = {"method": "rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES over `bench.py --solo-only --solo-frames 3` "
                     "(wave64 vector instructions per launch, mean per kernel family); peak = sustained v_fma_f32 "
                     "issue rate of tools/valu_calibration.py (k_valu_peak, 16 waves on every CU)",
           "valu_per_launch": {f: round(sum(v) / len(v)) for f, v in sorted(per.items())},
           "waves_per_launch": {f: round(sum(v) / len(v)) for f, v in sorted(waves.items())},
           "launches_profiled": {f: len(v) for f, v in sorted(per.items())},
           "peak_wave_instr_per_s": max(cal["float_16w"]["wave_instr_per_s"], cal["float_32w"]["wave_instr_per_s"]),
           "calibration": cal}
    os.makedirs(dst, exist_ok=True)
    json.dump(out, open(os.path.join(dst, "valu.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
