#!/bin/bash
# Scalar-memory / instruction-fetch counters of the solo pass (round 5: why the packet kernels
# gain nothing from a fifth wave per SIMD).  One PMC pass per group, each its own run.
#   usage: tools/profile_sqc.sh <tag> [extra bench.py args]
#   then:  python tools/sqc_table.py gpurun_out/<tag> > profiles/round5/sqc.json
set -o pipefail
TAG=${1:-sqc}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
i=0
for P in "SmemLatency SQ_INSTS_SMEM SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
         "InstrFetchLatency VmemLatency" \
         "SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE" \
         "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_TC_STALL" \
         "SQC_DCACHE_BUSY_CYCLES SQC_ICACHE_BUSY_CYCLES SQC_TC_DATA_READ_REQ SQC_TC_INST_REQ"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $O/p$i -o pmc --output-format csv -- python $R/bench.py --solo-only --solo-frames 4 "$@" > $O/p$i.log 2>&1 || { echo "pass $i ($P) failed"; tail -5 $O/p$i.log; exit 2; }
done
echo done
