#!/bin/bash
# A/B/C...: bench.py alternately with the default librtamd.so and variant builds
# (tools/build_variant.sh tags), same box, round-robin.
#   usage: tools/ab_multi.sh <rounds> <variant-tag> [variant-tag ...]
set -o pipefail
N=$1; shift
R=$(pwd)
mkdir -p gpurun_out/abm
for r in $(seq 1 $N); do
	for v in default "$@"; do
		if [ $v = default ]; then unset RTAMD_LIB; else export RTAMD_LIB=$R/cs184-raytracer_amd/rtamd/var/librtamd_$v.so; fi
		timeout -k 10 120 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --latency-frames 0 --sweep "" --solo-frames 0 ${BENCH_ARGS} > gpurun_out/abm/$v.$r.json 2>gpurun_out/abm/$v.$r.err || exit 1
		echo "$v $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" gpurun_out/abm/$v.$r.json)"
	done
done
