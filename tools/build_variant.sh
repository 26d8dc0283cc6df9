#!/bin/bash
# Build an A/B variant of librtamd.so with extra device flags, out of tree
# (a copy of raytracing-project_amd under /tmp), into
# raytracing-project_amd/lib/exp/librtamd_<name>.so (tools/gpu/ab_lib.sh).
# Usage: tools/build_variant.sh <name> -DFOO=1 ...
set -e
NAME=$1; shift
REPO=$(cd "$(dirname "$0")/.." && pwd)
B=/tmp/rtamd_variant_$NAME
rm -rf "$B" && mkdir -p "$B"
cp -r "$REPO/raytracing-project_amd" "$B/" && cp -r "$REPO/include" "$B/"
rm -rf "$B/raytracing-project_amd/build" "$B/raytracing-project_amd/lib/exp"
make -C "$B/raytracing-project_amd" -j8 lib/librtamd.so \
  HIP_FLAGS="-std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -munsafe-fp-atomics -Wall -Wno-unused-function $*" > "$B/build.log" 2>&1
mkdir -p "$REPO/raytracing-project_amd/lib/exp"
cp "$B/raytracing-project_amd/lib/librtamd.so" "$REPO/raytracing-project_amd/lib/exp/librtamd_$NAME.so"
rm -rf "$B"
echo "built lib/exp/librtamd_$NAME.so ($*)"
