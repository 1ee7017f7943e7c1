#!/bin/bash
# Tuning sweeps on the GPU box: for each argument, either rebuild librtamd with that
# EXTRA_DEFS string (preprocessor defines for host and device code), or (argument "env:VAR=VALUE") run the default build with VAR set,
# and run the 1-GPU bench.  Restores the default build at the end.
#   tools/variant_sweep.sh "" "-DRT_TRAVERSAL_WAVES=4" "env:RTAMD_PACKET_MASK=1" ...
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/sweep
built=none
for v in "$@"; do
	envset=""
	flags="$v"
	if [[ "$v" == env:* ]]; then envset="${v#env:}"; flags=""; fi
	if [[ "$flags" != "$built" ]]; then
		rm -f cs184-raytracer_amd/build/*.o
		make -s -C cs184-raytracer_amd -j8 EXTRA_DEFS="$flags" rtamd/librtamd.so > /dev/null
		built="$flags"
	fi
	tag=$(echo "x$v" | tr -c 'a-zA-Z0-9=\n' '_')
	env $envset timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sweep/$tag.json
	echo "variant [$v]: $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['unit'], d['ms_per_step'], 'ms', {k: v['ms_per_frame'] for k, v in d['roofline']['stages'].items()})" gpurun_out/sweep/$tag.json)"
done
rm -f cs184-raytracer_amd/build/*.o
make -s -C cs184-raytracer_amd -j8 rtamd/librtamd.so > /dev/null
