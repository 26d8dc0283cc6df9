#!/bin/bash
# Build experimental librtamd variants into raytracing-project_amd/lib/exp/ (diagnostics; load with RTAMD_LIB=...).
# Only the FP64 kernels are rebuilt with the extra flags; the rest is the in-tree build.
# The product's trace-kernel backend options are kept (EXP_UNIFORM= drops the uniform-region one).
# Usage: tools/build_exp.sh NAME "extra hipcc flags"
set -e
cd "$(dirname "$0")/../raytracing-project_amd"
mkdir -p lib/exp build/exp
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -munsafe-fp-atomics -mllvm --amdgpu-set-wave-priority ${EXP_UNIFORM--mllvm --structurizecfg-skip-uniform-regions} \
  -I../include -Icsrc/host -Icsrc/device $2 -c csrc/device/rt_kernels_f64.hip -o build/exp/rt_kernels_f64_$1.o 2>/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/exp/librtamd_$1.so build/rt_render.o \
  build/exp/rt_kernels_f64_$1.o build/rt_kernels_f32.o build/rt_kernels_big.o build/mt_jump.o build/rt_dist.o build/mt_poly.o build/scene_compile.o \
  -Llib -lrt_host -ldl -Wl,-rpath,'$ORIGIN/..'
echo built lib/exp/librtamd_$1.so
