#!/bin/bash
# One GPU call: the -m gpu suite, then the default bench line (each step time-limited;
# stops at the first failure).  Output under gpurun_out/$1.
set -o pipefail
tag=${1:-check}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cat $out/bench.json | head -c 3000
