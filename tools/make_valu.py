"""VALU roof data from a tools/profile_round3.sh run: per kernel, vector instructions per
launch, VALU-busy and stall fractions from the SQ counters, and the chip's calibrated VALU
issue peak.

usage: python tools/make_valu.py gpurun_out/<tag> profiles/<round>     -> <round>/valu.json

- valu: rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES
  SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE
  over `bench.py --solo-only` (every kernel alone).
- valu_cal: the same counters over tools/valu_calibration.py (k_valu_peak: 32 independent
  chains x4 of v_fma_f32, v_pk_fma_f32 or v_fma_f64 on every SIMD at 1, 2, 4, 8 waves).
- sq2 (optional): SQ_THREAD_CYCLES_VALU ... (lane utilisation, scalar/vector/LDS instruction mix).

Units (rocprofv3 sums every counter over its instances): SQ_WAVE_CYCLES, SQ_WAIT_*,
SQ_ACTIVE_INST_* are quad-cycles summed over waves (MI355X_MICROARCH.md, "s_memtime tick vs
SQ PMC units"); GRBM_GUI_ACTIVE is GPU-busy cycles summed over the XCDs, so GRBM_GUI_ACTIVE /
n_xcd / duration is the shader clock.  VALU busy = SQ_ACTIVE_INST_VALU / (CU_NUM x GRBM
cycles per XCD), the VALUBusy derived metric of rocprofv3 (100 x SQ_ACTIVE_INST_VALU / CU_NUM /
GRBM_GUI_ACTIVE): the fraction of SIMD-cycles spent issuing vector instructions."""
import collections
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kname import parse  # noqa: E402

N_XCD, N_CU, N_SIMD = 8, 256, 1024


def variant(name):
    """k_shadow<true, true> etc. (tools/kname.py); None for the counting instantiations."""
    return parse(name)[1]


def family(v):
    return v.split("<")[0] if v else None


def load(d):
    dur = {}
    kt = [f for f in os.listdir(d) if f.endswith("kernel_trace.csv")]
    for r in csv.DictReader(open(os.path.join(d, kt[0]))):
        dur[r["Dispatch_Id"]] = (r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    ctr = collections.defaultdict(dict)
    cc = [f for f in os.listdir(d) if f.endswith("counter_collection.csv")]
    for r in csv.DictReader(open(os.path.join(d, cc[0]))):
        ctr[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        if r["Dispatch_Id"] not in dur:
            dur[r["Dispatch_Id"]] = (r["Kernel_Name"], None)
    return dur, ctr


def derived(c, secs):
    g = lambda k: c.get(k, float("nan"))
    grbm = g("GRBM_GUI_ACTIVE") / N_XCD  # GPU-busy cycles of one XCD
    # busy on the kernel's own duration at 2.4 GHz: GRBM_GUI_ACTIVE of a short dispatch also
    # counts the collection window around it (its clock would read > 3 GHz)
    cyc = secs * 2.4e9 if secs else grbm
    out = {"valu_wave_instr": g("SQ_INSTS_VALU"), "seconds": secs,
           "clock_ghz": grbm / secs / 1e9 if secs else None,
           "valu_busy": g("SQ_ACTIVE_INST_VALU") / (N_CU * cyc),
           "wait_inst_any": g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES"),
           "wait_any": g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"),
           "active_inst_any": g("SQ_ACTIVE_INST_ANY") / g("SQ_WAVE_CYCLES"),
           "salu_per_valu": g("SQ_INSTS_SALU") / g("SQ_INSTS_VALU")}
    if secs and grbm:
        # cycles of one SIMD per wave64 vector instruction, if every SIMD issued for the whole launch
        out["simd_cycles_per_valu"] = grbm * N_SIMD / g("SQ_INSTS_VALU")
        out["valu_busy_cycles_per_valu"] = 4 * g("SQ_ACTIVE_INST_VALU") / g("SQ_INSTS_VALU")
    return out


def mean(rows, key):
    v = [r[key] for r in rows if r.get(key) is not None]
    return sum(v) / len(v) if v else None


def main():
    src, dst = sys.argv[1], sys.argv[2]
    dur, ctr = load(os.path.join(src, "valu_cal"))
    cal = {}
    kinds = {"0": "v_fma_f32", "1": "v_pk_fma_f32", "2": "v_fma_f64"}
    for k, instr in kinds.items():
        ids = sorted(int(i) for i, (n, _) in dur.items() if f"k_valu_peak<{k}>" in n)
        # dispatches per kind: (warm-up, measured) at 1, 2, 4, 8 waves per SIMD
        for w, i in zip((1, 2, 4, 8), ids[1::2]):
            i = str(i)
            d = derived(ctr[i], dur[i][1])
            d["wave_instr_per_s"] = d["valu_wave_instr"] / d["seconds"]
            cal[f"{instr}_{w}w"] = {k2: (round(v, 4) if isinstance(v, float) else v) for k2, v in d.items()}
    best = max(cal, key=lambda k: cal[k]["wave_instr_per_s"])
    best64 = max((k for k in cal if "f64" in k), key=lambda k: cal[k]["wave_instr_per_s"])
    # The roof: the chip's wave64 issue rate of 4-cycle VALU instructions (v_fma_f64,
    # v_pk_fma_f32: 4 SIMD cycles each, measured above), 1024 SIMDs at 2.4 GHz = 614.4 G/s,
    # the rate behind the guide's 78.6 TF vector FP64.  Plain 32-bit VALU (v_fma_f32) issues
    # at 2 cycles with >= 2 waves per SIMD (MI355X_MICROARCH.md:473; measured 2.2 here), so
    # for the traversal kernels' mix (mostly fp64) achieved / 614.4 G is an upper bound of
    # their issue-slot use.
    peak = N_SIMD * 2.4e9 / 4
    dur, ctr = load(os.path.join(src, "valu"))
    per = collections.defaultdict(list)
    for i, (n, secs) in dur.items():
        v = variant(n)
        if v and i in ctr and secs:
            per[v].append(derived(ctr[i], secs))
    sq2 = {}
    p2 = os.path.join(src, "sq2")
    if os.path.isdir(p2):
        d2, c2 = load(p2)
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        for i, (n, _) in d2.items():
            v = variant(n)
            if v and i in c2:
                for k, x in c2[i].items():
                    acc[v][k] += x
        for v, c in acc.items():
            w = c.get("SQ_WAVES", 0) or float("nan")
            sq2[v] = {"lane_util": round(c["SQ_THREAD_CYCLES_VALU"] / c["SQ_ACTIVE_INST_VALU"] / 64, 3),
                      "smem_per_wave": round(c["SQ_INSTS_SMEM"] / w, 1), "vmem_rd_per_wave": round(c["SQ_INSTS_VMEM_RD"] / w, 1),
                      "lds_per_wave": round(c["SQ_INSTS_LDS"] / w, 1),
                      "scalar_active_frac_of_valu_active": round(c["SQ_ACTIVE_INST_SCA"] / c["SQ_ACTIVE_INST_VALU"], 3),
                      "vmem_active_frac_of_valu_active": round(c["SQ_ACTIVE_INST_VMEM"] / c["SQ_ACTIVE_INST_VALU"], 3)}
    kernels = {}
    fam = collections.defaultdict(list)
    for v, rows in sorted(per.items()):
        instr = sum(r["valu_wave_instr"] for r in rows)
        secs = sum(r["seconds"] for r in rows)
        kernels[v] = {"launches": len(rows), "valu_per_launch": round(instr / len(rows)),
                      "us_per_launch": round(secs / len(rows) * 1e6, 2),
                      "issue_rate_g": round(instr / secs / 1e9, 2), "issue_frac_of_peak": round(instr / secs / peak, 4),
                      **{k: round(mean(rows, k), 4) for k in ("valu_busy", "wait_inst_any", "wait_any", "active_inst_any",
                                                               "salu_per_valu", "clock_ghz", "valu_busy_cycles_per_valu")},
                      **({"sq2": sq2[v]} if v in sq2 else {})}
        fam[family(v)].extend(rows)
    out = {"method": "rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES "
                     "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE over `bench.py "
                     "--solo-only --solo-frames 4` (every kernel alone) and over tools/valu_calibration.py; peak = the 4-cycle "
                     "wave64 issue rate (peak_what); valu_busy on the kernel's duration at 2.4 GHz",
           "valu_per_launch": {f: round(sum(r["valu_wave_instr"] for r in rows) / len(rows)) for f, rows in sorted(fam.items())},
           "valu_busy": {f: round(mean(rows, "valu_busy"), 4) for f, rows in sorted(fam.items())},
           "wait_inst_any": {f: round(mean(rows, "wait_inst_any"), 4) for f, rows in sorted(fam.items())},
           "wait_any": {f: round(mean(rows, "wait_any"), 4) for f, rows in sorted(fam.items())},
           "launches_profiled": {f: len(rows) for f, rows in sorted(fam.items())},
           "peak_wave_instr_per_s": peak,
           "peak_what": "1024 SIMDs x 2.4 GHz / 4 cycles per wave64 instruction (v_fma_f64 / v_pk_fma_f32 rate; "
                        "the guide's 78.6 TF vector FP64); measured sustained: " + best64 + " " +
                        str(round(cal[best64]["wave_instr_per_s"] / 1e9, 1)) + " G/s; plain v_fma_f32 (2-cycle, "
                        "MI355X_MICROARCH.md:473): " + best + " " + str(round(cal[best]["wave_instr_per_s"] / 1e9, 1)) +
                        " G/s",
           "f32_dual_rate_wave_instr_per_s": cal[best]["wave_instr_per_s"],
           "f64_sustained_wave_instr_per_s": cal[best64]["wave_instr_per_s"],
           "calibration": cal, "kernels": kernels}
    os.makedirs(dst, exist_ok=True)
    json.dump(out, open(os.path.join(dst, "valu.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
