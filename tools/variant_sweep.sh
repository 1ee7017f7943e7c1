#!/bin/bash
# Builds librtamd with each EXTRA_HIPFLAGS variant given as an argument and runs the
# 1-GPU bench for it (tuning sweeps on the GPU box).  Restores the default build at the end.
#   tools/variant_sweep.sh "" "-DRT_TRAVERSAL_WAVES=4" ...
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/sweep
for v in "$@"; do
	rm -f cs184-raytracer_amd/build/trace.o
	make -s -C cs184-raytracer_amd -j8 EXTRA_HIPFLAGS="$v" rtamd/librtamd.so > /dev/null
	tag=$(echo "x$v" | tr -c 'a-zA-Z0-9=\n' '_')
	timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sweep/$tag.json
	echo "variant [$v]: $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['unit'], d['ms_per_step'], 'ms', {k: v['ms_per_frame'] for k, v in d['roofline']['stages'].items()})" gpurun_out/sweep/$tag.json)"
done
rm -f cs184-raytracer_amd/build/trace.o
make -s -C cs184-raytracer_amd -j8 rtamd/librtamd.so > /dev/null
