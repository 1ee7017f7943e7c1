#!/bin/bash
# Kernel timelines of single frames (rocprofv3 --kernel-trace over tools/one_config.py):
#   tools/latency_trace.sh <tag> C1_simple_sphere_256 C4_airboat_sub_1920x1080 ...
#   (<config>@k/n: rank k's row-block share of an n-way partition, tools/one_config.py)
# then: python tools/frame_timeline.py gpurun_out/<tag>/<config>/*kernel_trace.csv
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
	timeout -k 10 120 rocprofv3 --kernel-trace -d $O/$c -o kt --output-format csv -- python $R/tools/one_config.py $cfg 6 $share > $O/$c.log 2>&1 || exit 1
	python $R/tools/frame_timeline.py $(ls $O/$c/*kernel_trace.csv $O/$c/*/*kernel_trace.csv 2>/dev/null | head -1) > $O/$c.timeline.txt || exit 2
	tail -1 $O/$c.timeline.txt
done
