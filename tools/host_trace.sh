#!/bin/bash
# Host + kernel timeline of single frames: rocprofv3 --hip-trace --kernel-trace (no counters)
# over tools/one_config.py, so every HIP API call of a render call and every kernel sit on one
# clock (where the host time of a call goes: launches, event records, cross-stream waits,
# the final synchronisation).  Then tools/host_timeline.py summarises the last frames.
#   tools/host_trace.sh <tag> C1_simple_sphere_256 C4_airboat_sub_1920x1080 ...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for a in "$@"; do
	cfg=${a%%@*}; share=""; [[ $a == *@* ]] && share=${a#*@}
	c=$(echo $a | tr '@/' '__')
	timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace -d $O/$c -o tr --output-format csv -- python $R/tools/one_config.py $cfg 12 $share > $O/$c.log 2>&1 || exit 1
	python $R/tools/host_timeline.py $O/$c > $O/$c.host.txt || exit 2
	tail -3 $O/$c.host.txt
done
