#!/bin/bash
# Per-config single-frame times, the per-kernel VALU breakdown (default build and the
# no-LBVH diagnostic build) and the lane census of the per-lane kernels, on the GPU box.
# Needs the variant builds: tools/build_variant.sh nobvh -DRT_DIAG_SKIP=1;
# tools/build_variant.sh lanes -DRT_DIAG_LANES=1.
#   usage: tools/round_artifacts.sh <tag>   (writes gpurun_out/<tag>/)
set -o pipefail
TAG=${1:-art}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 150 python $R/tools/config_bench.py 7 > $O/configs.jsonl 2> $O/configs.err || exit 1
timeout -k 10 200 bash $R/tools/valu_breakdown.sh $TAG/vb nobvh > /dev/null || exit 2
python $R/tools/valu_table.py $O/vb > $O/valu_breakdown.txt || exit 3
RTAMD_LIB=$R/cs184-raytracer_amd/rtamd/var/librtamd_lanes.so timeout -k 10 120 python $R/tools/lane_census.py 3 > $O/lane_census.txt 2>/dev/null || exit 4
echo done
