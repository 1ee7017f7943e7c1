#!/bin/bash
# A/B/C...: bench.py alternately with the default librtamd.so and variant builds
# (tools/build_variant.sh tags) or environment settings ("env:VAR=VALUE[,VAR=VALUE]"),
# same box, round-robin.
#   usage: tools/ab_multi.sh <rounds> <variant> [variant ...]
set -o pipefail
N=$1; shift
R=$(pwd)
mkdir -p gpurun_out/abm
for r in $(seq 1 $N); do
	for v in default "$@"; do
		envset=""
		unset RTAMD_LIB
		if [[ $v == env:* ]]; then envset=$(echo "${v#env:}" | tr ',' ' ');
		elif [ $v != default ]; then export RTAMD_LIB=$R/cs184-raytracer_amd/rtamd/var/librtamd_$v.so; fi
		env $envset timeout -k 10 120 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --latency-frames 0 --sweep "" --solo-frames 0 ${BENCH_ARGS} > gpurun_out/abm/$(echo $v | tr -c "a-zA-Z0-9.\n" _).$r.json 2>gpurun_out/abm/$(echo $v | tr -c "a-zA-Z0-9.\n" _).$r.err || exit 1
		echo "$v $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" gpurun_out/abm/$(echo $v | tr -c "a-zA-Z0-9.\n" _).$r.json)"
	done
done
