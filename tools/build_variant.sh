#!/bin/bash
# Builds a variant of librtamd (with the diag hooks of librtamd_diag.so) with extra preprocessor defines into
# cs184-raytracer_amd/rtamd/var/librtamd_<tag>.so (here, on the CPU; the .so travels to the
# GPU box with the tree; load it there with RTAMD_LIB=...).  The default build is untouched.
#   usage: tools/build_variant.sh <tag> "<defines>"      e.g. tools/build_variant.sh nobvh -DRT_DIAG_SKIP=1
#   EXTRA_HIP="<flags>": device compiler flags for the HIP sources only (e.g. -mllvm options)
set -e
TAG=$1
DEFS=$2
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/cs184-raytracer_amd
B=$P/build/var_$TAG
mkdir -p $B $P/rtamd/var
rm -f $B/*.o
FL="-O3 -fPIC -std=c++17 -ffp-contract=off -Wall $DEFS"
HIPCC=/opt/rocm/bin/hipcc
$HIPCC $FL $EXTRA_HIP --offload-arch=gfx950 -munsafe-fp-atomics -c -o $B/trace.o $P/csrc/trace.hip &
$HIPCC $FL --offload-arch=gfx950 -munsafe-fp-atomics -c -o $B/api.o $P/csrc/api.cpp &
$HIPCC $FL --offload-arch=gfx950 -munsafe-fp-atomics -c -o $B/diag.o $P/csrc/diag.cpp &
for f in scene_host bvh png; do
	g++ $FL -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c -o $B/$f.o $P/csrc/$f.cpp &
done
wait
$HIPCC --offload-arch=gfx950 -shared -o $P/rtamd/var/librtamd_$TAG.so $B/trace.o $B/api.o $B/diag.o $B/scene_host.o $B/bvh.o $B/png.o -lz -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
echo "$P/rtamd/var/librtamd_$TAG.so"
