#!/bin/bash
# Vector-instruction counts per kernel per frame (C3, one frame per call) for the default
# build and for variant builds (tools/build_variant.sh), one rocprofv3 --pmc pass each.
#   usage (GPU box): tools/valu_breakdown.sh <out-tag> [variant-tag ...]
#   then: python tools/valu_table.py gpurun_out/<out-tag>
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in default "$@"; do
	if [ $v = default ]; then unset RTAMD_LIB; else export RTAMD_LIB=$R/cs184-raytracer_amd/rtamd/var/librtamd_$v.so; fi
	timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES -d $O/$v -o pmc --output-format csv -- python $R/tools/one_config.py ${CONFIG:-C3_bunny_1920x1080_bd4} ${FRAMES:-6} > $O/$v.log 2>&1 || exit 1
done
echo done
