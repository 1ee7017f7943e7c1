"""Per-kernel HBM traffic and launch durations from a tools/profile_round2.sh run.

usage: python tools/make_traffic.py gpurun_out/<tag> profiles/<round>

Writes <round>/traffic.json (read by bench.py) and copies the rocprofv3 summaries
(kernel stats of the solo pass and of the default bench) next to it.

FETCH_SIZE and WRITE_SIZE come from separate rocprofv3 --pmc passes over the solo pass
(`bench.py --solo-only`: every kernel alone), in kB per dispatch.  The FETCH_SIZE
correction is measured, not assumed: the calibration pass (tools/fetch_calibration.py)
reads a 1 GiB buffer once at 1, 4, 8 and 16 bytes per lane (the widths of the path's
ray/hit/flag loads), and bytes / counted bytes is the factor (MI355X_MICROARCH.md: only the
16-B case was calibrated there).  Kernels are grouped by family (k_shadow<true> and
k_shadow<false> -> k_shadow), the unit bench.py reports its roofline for."""
import collections
import csv
import json
import os
import re
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kname import parse  # noqa: E402

CALIB_BYTES = 1 << 30


def family(name):
    """Kernel family; None for the counting instantiations (tools/kname.py)."""
    return parse(name)[0]


def per_dispatch(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        f = family(r["Kernel_Name"])
        if f and r["Counter_Name"] == counter:
            acc[f].append(float(r["Counter_Value"]))
    return acc


def calibration(path):
    """FETCH_SIZE (kB) of the measured reads: dispatches alternate evict (16 B) / measured."""
    rows = [r for r in csv.DictReader(open(path)) if "k_stream_read" in r["Kernel_Name"]
            and r["Counter_Name"] == "FETCH_SIZE"]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    measured = rows[1::2]
    out = {}
    for width, r in zip([1, 4, 8, 16], measured):
        counted = float(r["Counter_Value"]) * 1024
        out[str(width)] = {"fetch_kB": float(r["Counter_Value"]), "bytes_read": CALIB_BYTES,
                           "factor": round(CALIB_BYTES / counted, 4)}
    return out


def durations(path):
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        f = family(r["Kernel_Name"])
        if f:
            dur[f].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return {f: round(sum(d) / len(d), 4) for f, d in sorted(dur.items())}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    cal = calibration(f"{src}/calib/pmc_counter_collection.csv")
    factors = sorted({v["factor"] for v in cal.values()})
    # one factor for every width the path uses (1, 4, 8 B per lane; 16 B not used): the
    # largest, so the traffic is an upper bound if they ever differ
    factor = max(v["factor"] for w, v in cal.items() if w in ("1", "4", "8"))
    fetch = per_dispatch(f"{src}/fetch/pmc_counter_collection.csv", "FETCH_SIZE")
    write = per_dispatch(f"{src}/write/pmc_counter_collection.csv", "WRITE_SIZE")
    out = {"method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over `bench.py "
                     "--solo-only --solo-frames 4` (every kernel alone); per kernel family, mean per launch; "
                     f"FETCH_SIZE x {factor} (measured: tools/fetch_calibration.py, 1 GiB read at 1/4/8/16 B per "
                     "lane), WRITE_SIZE as counted (exact for streaming stores, MI355X_MICROARCH.md); kB x 1024",
           "fetch_calibration": cal, "fetch_factor": factor, "fetch_factors_seen": factors,
           "hbm_bytes_per_launch": {}, "fetch_kB_per_launch_raw": {}, "write_kB_per_launch_raw": {},
           "launches_profiled": {},
           "avg_launch_ms_solo_kernel_trace": durations(f"{src}/solo/solo_kernel_trace.csv"),
           "avg_launch_ms_bench_kernel_trace": durations(f"{src}/kt/kt_kernel_trace.csv")}
    for f in sorted(set(fetch) & set(write)):
        fk = sum(fetch[f]) / len(fetch[f])
        wk = sum(write[f]) / len(write[f])
        out["fetch_kB_per_launch_raw"][f] = round(fk, 3)
        out["write_kB_per_launch_raw"][f] = round(wk, 3)
        out["hbm_bytes_per_launch"][f] = round((factor * fk + wk) * 1024)
        out["launches_profiled"][f] = len(fetch[f])
    json.dump(out, open(f"{dst}/traffic.json", "w"), indent=1)
    shutil.copy(f"{src}/solo/solo_kernel_stats.csv", f"{dst}/solo_kernel_stats.csv")
    shutil.copy(f"{src}/kt/kt_kernel_stats.csv", f"{dst}/kernel_stats.csv")
    print(json.dumps({k: out[k] for k in ("fetch_factor", "hbm_bytes_per_launch", "avg_launch_ms_solo_kernel_trace")},
                     indent=1))


if __name__ == "__main__":
    main()
