#!/bin/bash
# A/B of one GPU's share of an e-way row partition (bench.py --emulate-ranks e) under
# environment settings, round-robin on one box (GPU box, from the repo root).
#   usage: tools/emu_ab.sh <rounds> <steps> <warmup> "<e>:<VAR=VALUE[,VAR=VALUE]>" ...
#   e.g.   tools/emu_ab.sh 2 60 3 "8:X=1" "8:RTAMD_BATCH_BALANCE=0"
set -o pipefail
N=$1; ST=$2; WU=$3; shift 3
for r in $(seq 1 $N); do
  for v in "$@"; do
    e=${v%%:*}; vars=${v#*:}
    env $(echo $vars | tr ',' ' ') timeout -k 10 200 python bench.py --steps $ST --warmup $WU --no-cpu-baseline --latency-frames 0 --sweep "" --solo-frames 0 --emulate-ranks $e > gpurun_out/emu.json 2>gpurun_out/emu.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/emu.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
  done
done
