#!/bin/bash
# A/B: bench.py alternately with librtamd.so (B) and an older build (A, RTAMD_LIB), same box.
#   usage: tools/ab_bench.sh <path of A .so> [rounds]
set -o pipefail
A=$1; N=${2:-3}
mkdir -p gpurun_out/ab
for r in $(seq 1 $N); do
	for v in A B; do
		if [ $v = A ]; then export RTAMD_LIB=$A; else unset RTAMD_LIB; fi
		timeout -k 10 120 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --latency-frames 0 --sweep "" --solo-frames 0 > gpurun_out/ab/$v$r.json 2>/dev/null || exit 1
		echo "$v $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" gpurun_out/ab/$v$r.json)"
	done
done
