"""Host + device timeline of the last rendered frame from a rocprofv3 --hip-trace --kernel-trace
directory (tools/host_trace.sh): every HIP API call and kernel of the call, on one clock,
relative to the call's first API call.

usage: python tools/host_timeline.py <rocprofv3 output dir>"""
import csv
import glob
import os
import re
import sys


def rows(pattern):
    out = []
    for f in glob.glob(os.path.join(sys.argv[1], "**", pattern), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


api = sorted(rows("*hip_api_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
ker = sorted(rows("*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))


def kname(r):
    m = re.search(r"(k_[a-z0-9_]+(?:<[a-z, ]+>)?)\(", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"][:24]


# frames end with the statistics reduction; the last frame starts after the API call that
# waited for the previous one (the synchronisation that returned after k_stats_finish)
fin = [r for r in ker if "k_stats_finish" in r["Kernel_Name"]]
prev_end, last_end = int(fin[-2]["End_Timestamp"]), int(fin[-1]["End_Timestamp"])
# the render call's API calls: after the previous frame's synchronisation returned
calls = [r for r in api if int(r["Start_Timestamp"]) > prev_end and int(r["Start_Timestamp"]) <= last_end + 200000]
sync_after = [r for r in calls if r["Function"] in ("hipStreamSynchronize", "hipDeviceSynchronize")]
t0 = int(calls[0]["Start_Timestamp"])
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api", r["Function"]) for r in calls]
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "gpu", kname(r)) for r in ker
       if prev_end < int(r["Start_Timestamp"]) <= last_end]
ev.sort()
for s, e, k, n in ev:
    print(f"{k} {n:34s} start={(s - t0) / 1e3:8.1f}us dur={(e - s) / 1e3:7.1f}us")
first_k = min(s for s, e, k, n in ev if k == "gpu")
last_api = max(e for s, e, k, n in ev if k == "api")
print(f"first API call -> first kernel start {(first_k - t0) / 1e3:.1f} us; last kernel end "
      f"{(last_end - t0) / 1e3:.1f} us; last API call returns {(last_api - t0) / 1e3:.1f} us")
print(f"API calls {len(calls)}; host time in API calls {sum(e - s for s, e, k, n in ev if k == 'api') / 1e3:.1f} us")
