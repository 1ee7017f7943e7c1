#!/bin/bash
# Roofline recipe (run on the MI355X box via gpurun):
#   1. kernel trace + stats of the solo pass (the roofline's time base) and of the default bench
#   2. HBM bytes: FETCH_SIZE and WRITE_SIZE in separate PMC passes over the solo pass, and the
#      FETCH_SIZE calibration (tools/fetch_calibration.py)
#   3. SQ issue/stall counters (+ GRBM_GUI_ACTIVE) over the solo pass, and over the VALU issue
#      calibration (k_valu_peak: v_fma_f32 / v_pk_fma_f32 / v_fma_f64 at 1-8 waves per SIMD)
#   usage: tools/profile_roofline.sh <tag>
#   then:  python tools/make_traffic.py gpurun_out/<tag> profiles/round<N>
#          python tools/make_valu.py gpurun_out/<tag> profiles/round<N>
set -o pipefail
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"
SQ2="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAVES GRBM_GUI_ACTIVE"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/solo -o solo --output-format csv -- python $R/bench.py --solo-only --solo-frames 4 > $O/solo.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --sweep "" --solo-frames 0 > $O/kt.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o pmc --output-format csv -- python $R/bench.py --solo-only --solo-frames 4 > $O/fetch.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o pmc --output-format csv -- python $R/bench.py --solo-only --solo-frames 4 > $O/write.log 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/calib -o pmc --output-format csv -- python $R/tools/fetch_calibration.py > $O/calib.log 2>&1 || exit 6
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $SQ -d $O/valu -o pmc --output-format csv -- python $R/bench.py --solo-only --solo-frames 4 > $O/valu.log 2>&1 || exit 7
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ -d $O/valu_cal -o pmc --output-format csv -- python $R/tools/valu_calibration.py > $O/valu_cal.log 2>&1 || exit 8
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $SQ2 -d $O/sq2 -o pmc --output-format csv -- python $R/bench.py --solo-only --solo-frames 4 > $O/sq2.log 2>&1 || exit 9
echo done
