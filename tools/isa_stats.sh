#!/bin/bash
# Static instruction statistics of one trace kernel (host-side, no GPU):
# SGPR count, SGPR spill traffic through VGPR lanes (v_writelane / v_readlane),
# VALU / SALU / s_nop / branch counts.  A proxy for A/B builds; the GPU PMC
# passes (tools/gpu/abl_pmc.sh) give the dynamic counts.
# Usage: tools/isa_stats.sh [kernel-substring] [extra hipcc flags...]
cd "$(dirname "$0")/../raytracing-project_amd" || exit 1
K=${1:-k_std_leanILb0ELb1E}
shift
OUT=/tmp/isa_stats_$$.s
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -munsafe-fp-atomics \
  -mllvm --amdgpu-set-wave-priority -mllvm --structurizecfg-skip-uniform-regions \
  -I../include -Icsrc/host -Icsrc/device "$@" --cuda-device-only -S csrc/device/rt_kernels_f64.hip -o $OUT 2>/dev/null || exit 1
awk -v K="$K" '
  $0 ~ "^_Z.*" K ".*:" && !start {start=1; next}
  start && /^\t\.end_amdhsa_kernel/ {start=0; done=1}
  start && /^\t\.amdhsa_kernel/ {start=0}
  start && /^\tv_/ {valu++}
  start && /^\ts_/ && !/^\ts_nop/ && !/^\ts_waitcnt/ {salu++}
  start && /^\ts_nop/ {nop++}
  start && /v_writelane_b32/ {wl++}
  start && /v_readlane_b32 s[0-9]+, v[0-9]+, [0-9]+$/ {rl++}
  start && /s_cbranch|s_branch/ {br++}
  start && /scratch_/ {scr++}
  done && /TotalNumSgprs|NumVgprs:|ScratchSize:/ && !seen[$2]++ {print}
  END {printf "VALU %d  SALU %d  s_nop %d  writelane %d  readlane(imm) %d  branches %d  scratch ops %d\n", valu, salu, nop, wl, rl, br, scr}
' $OUT | tail -5
rm -f $OUT
