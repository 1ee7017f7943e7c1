"""VALU instruction mix per kernel (tools/profile_mix.sh output) and the issue-cycle bound it
implies: usage python tools/make_mix.py gpurun_out/<tag> [out_dir]"""
import csv
import collections
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kname import parse  # noqa: E402


def load(d):
    f = [x for x in os.listdir(d) if x.endswith("counter_collection.csv")][0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for r in csv.DictReader(open(os.path.join(d, f))):
        k = parse(r["Kernel_Name"])[1]
        if not k:  # counting instantiations (bench.py solo pass)
            continue
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[k].add(r["Dispatch_Id"])
    return per, {k: len(v) for k, v in launches.items()}


def main():
    src = sys.argv[1]
    m1, n1 = load(os.path.join(src, "m1"))
    m2, n2 = load(os.path.join(src, "m2"))
    m3, n3 = load(os.path.join(src, "m3"))
    out = {"method": "rocprofv3 --kernel-trace --pmc, tools/profile_mix.sh: m1/m2 over bench.py --solo-only "
                     "--solo-frames 4 (per kernel), m3 over bench.py --steps 2 --warmup 1 (whole batch schedule)",
           "kernels": {}}
    for k in sorted(m1):
        a, b = m1[k], m2.get(k, {})
        v = a["SQ_INSTS_VALU"]
        f64 = sum(a[f"SQ_INSTS_VALU_{x}_F64"] for x in ("ADD", "MUL", "FMA", "TRANS"))
        f32 = sum(b.get(f"SQ_INSTS_VALU_{x}_F32", 0) for x in ("ADD", "MUL", "FMA", "TRANS"))
        row = {"launches": n1[k], "valu": v, "f64_add": a["SQ_INSTS_VALU_ADD_F64"], "f64_mul": a["SQ_INSTS_VALU_MUL_F64"],
               "f64_fma": a["SQ_INSTS_VALU_FMA_F64"], "f64_trans": a["SQ_INSTS_VALU_TRANS_F64"],
               "int32": a["SQ_INSTS_VALU_INT32"], "int64": a["SQ_INSTS_VALU_INT64"], "cvt": a["SQ_INSTS_VALU_CVT"],
               "f32": f32, "f32_trans": b.get("SQ_INSTS_VALU_TRANS_F32", 0), "salu": b.get("SQ_INSTS_SALU", 0),
               "smem": b.get("SQ_INSTS_SMEM", 0), "waves": b.get("SQ_WAVES", 0)}
        row["other"] = v - f64 - row["int32"] - row["int64"] - row["cvt"] - f32
        row["frac"] = {x: round(row[x] / v, 4) for x in ("f64_add", "f64_mul", "f64_fma", "f64_trans", "int32",
                                                         "int64", "cvt", "f32", "other")} if v else {}
        out["kernels"][k] = row
    tot = collections.defaultdict(float)
    for k, a in m3.items():
        for c, x in a.items():
            tot[c] += x
    out["bench_schedule_totals"] = {"launches": sum(n3.values()), **dict(tot)}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2:
        json.dump(out, open(os.path.join(sys.argv[2], "valu_mix.json"), "w"), indent=1)


main()
