#!/bin/bash
# Solo (serialised) per-kernel times of one C3 frame: RTAMD_SERIAL=1 puts the shading
# kernels on the chain's stream, rocprofv3 --kernel-trace records every launch, and
# tools/frame_timeline.py prints the last frame.   usage: tools/solo_timeline.sh <tag>
set -o pipefail
TAG=${1:-solo}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp RTAMD_SERIAL=1
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --latency-frames 0 --frames-per-step 1 --sweep "" --solo-frames 0 > $O/kt.log 2>&1 || exit 1
python $R/tools/frame_timeline.py $O/kt/kt_kernel_trace.csv > $O/timeline.txt
