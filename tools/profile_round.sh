#!/bin/bash
# GPU profiling recipe (run on the MI355X box via gpurun):
#   bench line, rocprofv3 kernel trace + stats, and separate PMC passes for HBM bytes
#   (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950: MI355X_MICROARCH.md).
# usage: tools/profile_round.sh <tag>   (then copy gpurun_out/<tag>/traffic.json to
#        profiles/traffic_<round>.json and bench.json / kt/kt_kernel_stats.csv to profiles/<round>/)
set -o pipefail
TAG=${1:-round1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/kt.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o pmc --output-format csv -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o pmc --output-format csv -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/write.log 2>&1 || exit 4
cd $R
python tools/make_traffic.py $O $O/traffic.json > /dev/null || exit 5
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --traffic $O/traffic.json > $O/bench.json 2> $O/bench.err || exit 1
echo done
