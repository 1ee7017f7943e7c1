#!/bin/bash
# C5 (refraction3 4096^2, depth 8, spheres only) single frames: kernel trace + stats, and the
# SQ issue/stall counters per kernel (one rocprofv3 --pmc pass each, kernel trace only).
#   usage: tools/profile_c5.sh <tag>   then: python tools/make_valu.py ... (sq only: see DESIGN §5)
set -o pipefail
TAG=${1:-c5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"
SQ2="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAVES GRBM_GUI_ACTIVE"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python $R/tools/one_config.py C5_refraction3_4096_bd8 4 > $O/kt.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $SQ -d $O/sq -o pmc --output-format csv -- python $R/tools/one_config.py C5_refraction3_4096_bd8 3 > $O/sq.log 2>&1 || exit 2
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $SQ2 -d $O/sq2 -o pmc --output-format csv -- python $R/tools/one_config.py C5_refraction3_4096_bd8 3 > $O/sq2.log 2>&1 || exit 3
echo done
