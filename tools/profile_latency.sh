#!/bin/bash
# Memory-latency counters (one rocprofv3 --pmc pass each) over tools/tail_trace.py N
# (1/N of the C3 frame): average VMEM/SMEM/LDS instruction latency = SQ_INST_LEVEL_x /
# SQ_INSTS_x (cycles), L2 hit rate.   usage: tools/profile_latency.sh <tag> <N>
set -o pipefail
TAG=${1:-lat}
N=${2:-8}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAVES -d $O/p1 -o pmc --output-format csv -- python $R/tools/tail_trace.py $N > $O/p1.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES -d $O/p2 -o pmc --output-format csv -- python $R/tools/tail_trace.py $N > $O/p2.log 2>&1 || exit 2
echo done
