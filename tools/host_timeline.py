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
    m = re.search(r"(k_[a-z0-9_]+(?:<[a-z0-9, ]+>)?)\(", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"][:24]


# frames: tools/one_config.py synchronises before every render (hipDeviceSynchronize) and
# rt_scene_destroy once more at the end; the last frame lies between the last two
syncs = [r for r in api if r["Function"] == "hipDeviceSynchronize"]
prev_end, last_end = int(syncs[-2]["Start_Timestamp"]), int(syncs[-1]["Start_Timestamp"])
calls = [r for r in api if prev_end <= int(r["Start_Timestamp"]) < last_end]
t0 = int(calls[0]["Start_Timestamp"])
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api", r["Function"]) for r in calls]
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "gpu",
        "%-26s q%s s%s" % (kname(r), r.get("Queue_Id", "?"), r.get("Stream_Id", "?"))) for r in ker
       if prev_end < int(r["Start_Timestamp"]) <= last_end]
ev.sort()
for s, e, k, n in ev:
    print(f"{k} {n:34s} start={(s - t0) / 1e3:8.1f}us dur={(e - s) / 1e3:7.1f}us")
first_k = min(s for s, e, k, n in ev if k == "gpu")
last_api = max(e for s, e, k, n in ev if k == "api")
last_k = max(e for s, e, k, n in ev if k == "gpu")
print(f"first API call -> first kernel start {(first_k - t0) / 1e3:.1f} us; last kernel end "
      f"{(last_k - t0) / 1e3:.1f} us; last API call returns {(last_api - t0) / 1e3:.1f} us")
print(f"API calls {len(calls)}; host time in API calls {sum(e - s for s, e, k, n in ev if k == 'api') / 1e3:.1f} us")
