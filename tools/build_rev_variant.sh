#!/bin/bash
# Builds librtamd from the sources of a git revision (A/B of code changes on one box) into
# cs184-raytracer_amd/rtamd/var/librtamd_<tag>.so; load it there with RTAMD_LIB=...
#   usage: tools/build_rev_variant.sh <tag> <git-rev> ["<defines>"]
set -e
TAG=$1
REV=$2
DEFS=$3
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/rtamd_rev.XXXXXX)
git -C $R archive $REV cs184-raytracer_amd/csrc include | tar -x -C $T
P=$T/cs184-raytracer_amd
B=$T/build
mkdir -p $B $R/cs184-raytracer_amd/rtamd/var
FL="-O3 -fPIC -std=c++17 -ffp-contract=off -Wall $DEFS"
HIPCC=/opt/rocm/bin/hipcc
$HIPCC $FL $EXTRA_HIP --offload-arch=gfx950 -munsafe-fp-atomics -c -o $B/trace.o $P/csrc/trace.hip &
$HIPCC $FL --offload-arch=gfx950 -munsafe-fp-atomics -c -o $B/api.o $P/csrc/api.cpp &
for f in scene_host bvh png; do
	g++ $FL -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c -o $B/$f.o $P/csrc/$f.cpp &
done
wait
$HIPCC --offload-arch=gfx950 -shared -o $R/cs184-raytracer_amd/rtamd/var/librtamd_$TAG.so $B/trace.o $B/api.o $B/scene_host.o $B/bvh.o $B/png.o -lz -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
rm -rf $T
echo "$R/cs184-raytracer_amd/rtamd/var/librtamd_$TAG.so"
