#!/bin/bash
# Variant librtamd whose trace.hip device code goes through assembly: hipcc -S, optionally
# tools/vop3_select.py (VOP2 v_cndmask_b32 -> VOP3 encoding), assemble, link, bundle, and the
# host side compiled against that code object.
#   usage: tools/build_vop3_variant.sh <tag> <rewrite 0|1> ["<defines>"]
set -e
TAG=$1; RW=$2; DEFS=$3
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/cs184-raytracer_amd
B=$P/build/var_$TAG
mkdir -p $B $P/rtamd/var
L=/opt/rocm/lib/llvm/bin
H="-O3 -fPIC -std=c++17 -ffp-contract=off -Wall --offload-arch=gfx950 -munsafe-fp-atomics $DEFS"
/opt/rocm/bin/hipcc $H --cuda-device-only -S -o $B/trace-gfx950.s $P/csrc/trace.hip 2>&1 | grep -v hip-link || true
if [ "$RW" = 1 ]; then python3 $R/tools/vop3_select.py $B/trace-gfx950.s $B/trace-gfx950.v.s; else cp $B/trace-gfx950.s $B/trace-gfx950.v.s; fi
$L/clang -target amdgcn-amd-amdhsa -mcpu=gfx950 -c -o $B/trace-gfx950.o $B/trace-gfx950.v.s
$L/lld -flavor gnu -m elf64_amdgpu --no-undefined -shared -o $B/trace-gfx950.hsaco $B/trace-gfx950.o
$L/clang-offload-bundler -type=o -bundle-align=4096 -targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--gfx950 \
	-input=/dev/null -input=$B/trace-gfx950.hsaco -output=$B/trace.hipfb
/opt/rocm/bin/hipcc $H --cuda-host-only -Xclang -fcuda-include-gpubinary -Xclang $B/trace.hipfb -c -o $B/trace.o $P/csrc/trace.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $P/rtamd/var/librtamd_$TAG.so $B/trace.o $P/build/api.o $P/build/scene_host.o \
	$P/build/bvh.o $P/build/png.o -lz -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
echo "$P/rtamd/var/librtamd_$TAG.so"
