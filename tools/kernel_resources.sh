#!/bin/bash
# Static resource usage of the traversal kernels (VGPRs, SGPRs, spills, scratch, LDS) for a
# build with extra defines: tools/kernel_resources.sh "-DRT_FOO=1"
DEFS=$1
R=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 --cuda-device-only -c -o /tmp/kr_$$.o \
	$DEFS $R/cs184-raytracer_amd/csrc/trace.hip -Rpass-analysis=kernel-resource-usage 2>&1 |
	sed 's/.*remark: //; s/ \[-Rpass-analysis=kernel-resource-usage\]//' |
	awk '/Function Name:/ {name=$3; keep = (name ~ /k_closest|k_shadow|k_shade|k_fused|k_output/)} keep && /VGPRs:|TotalSGPRs|Spill|Scratch|LDS/ {printf "%s ", $0} keep && /LDS Size/ {print "  <- " name}' |
	sed 's/_ZN5rtamd12_GLOBAL__N_1//'
rm -f /tmp/kr_$$.o
