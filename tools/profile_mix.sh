#!/bin/bash
# VALU instruction mix of the traversal kernels (which vector instructions are 64-bit, i.e.
# 4-cycle, and which are 32-bit) over the solo pass, and the VALU/SALU totals of the bench's
# own batch schedule (counts are schedule-independent; PMC serialises the dispatches, so the
# bench's timing comes from its own run).
#   usage: tools/profile_mix.sh <tag>;  then: python tools/make_mix.py gpurun_out/<tag> profiles/round3
set -o pipefail
TAG=${1:-mix}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
M1="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
M2="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES"
M3="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $M1 -d $O/m1 -o pmc --output-format csv -- python $R/bench.py --solo-only --solo-frames 4 > $O/m1.log 2>&1 || exit 2
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $M2 -d $O/m2 -o pmc --output-format csv -- python $R/bench.py --solo-only --solo-frames 4 > $O/m2.log 2>&1 || exit 3
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $M3 -d $O/m3 -o pmc --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --latency-frames 0 --sweep "" --solo-frames 0 > $O/m3.log 2>&1 || exit 4
timeout -k 10 120 python $R/tools/valu_calibration.py ${CAL_N:-2000} --mix > $O/cal_mix.log 2>&1 || exit 5
echo done
