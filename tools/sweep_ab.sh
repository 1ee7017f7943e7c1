# A/B of the emulated single-frame strong-scaling sweep (bench.py strong_scaling) under
# environment variants, 2 rounds on one box:  VARIANTS="X=1 VAR=VALUE" bash tools/sweep_ab.sh
set -o pipefail
for r in 1 2; do for v in ${VARIANTS:-X=1 RTAMD_ONE_STREAM_LEVEL1=0}; do
env $v timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --solo-frames 0 --latency-frames 0 --frames-per-step 3 --sweep-reps 5 > gpurun_out/sw.json 2>gpurun_out/sw.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/sw.json'));print('$v',{c:[(p['n_gpus'],p['max_ms']) for p in v['curve']] for c,v in d['strong_scaling'].items()})"
done; done
