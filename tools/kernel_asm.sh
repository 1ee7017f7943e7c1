#!/bin/bash
# Device assembly of one kernel (name substring) for a build with extra defines:
#   tools/kernel_asm.sh k_closestILb1 "-DRT_FOO=1" > /tmp/k.s
PAT=$1
DEFS=$2
R=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 --cuda-device-only -S -o /tmp/ka_$$.s \
	$DEFS $R/cs184-raytracer_amd/csrc/trace.hip 2>/dev/null
awk -v pat="$PAT" '$0 ~ "^_ZN.*" pat ".*: *;" || $0 ~ "^_ZN.*" pat ".*:$" {on=1} on {print} on && /s_endpgm/ {exit}' /tmp/ka_$$.s
rm -f /tmp/ka_$$.s
