#!/bin/bash
# Round-2 profiling recipe (run on the MI355X box via gpurun): kernel trace + stats of the
# solo pass (the roofline's time base) and of the default bench, separate PMC passes for
# HBM bytes (FETCH_SIZE, WRITE_SIZE) over the solo pass, and the FETCH_SIZE calibration.
# Then SQ_INSTS_VALU over the solo pass and over the VALU issue calibration (the VALU roof).
#   usage: tools/profile_round2.sh <tag>   then: python tools/make_traffic.py gpurun_out/<tag> profiles/round2
#                                                 python tools/make_valu.py gpurun_out/<tag> profiles/round2
set -o pipefail
TAG=${1:-prof2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/solo -o solo --output-format csv -- python $R/bench.py --solo-only --solo-frames 4 > $O/solo.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --sweep "" --solo-frames 0 > $O/kt.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o pmc --output-format csv -- python $R/bench.py --solo-only --solo-frames 4 > $O/fetch.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o pmc --output-format csv -- python $R/bench.py --solo-only --solo-frames 4 > $O/write.log 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/calib -o pmc --output-format csv -- python $R/tools/fetch_calibration.py > $O/calib.log 2>&1 || exit 6
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES -d $O/valu -o pmc --output-format csv -- python $R/bench.py --solo-only --solo-frames 4 > $O/valu.log 2>&1 || exit 7
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES -d $O/valu_cal -o pmc --output-format csv -- python $R/tools/valu_calibration.py > $O/valu_cal.log 2>&1 || exit 8
echo done
