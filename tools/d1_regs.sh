#!/bin/bash
# VGPRs / occupancy / spills / scratch bytes of every k_arn_d1 instance (extra hipcc flags as arguments)
R=$(cd "$(dirname "$0")/.." && pwd)
hipcc --offload-arch=gfx950 -O3 -std=c++17 -c --cuda-device-only "$@" -Rpass-analysis=kernel-resource-usage \
  -I $R/include $R/tensorkrylov.jl_amd/csrc/tk_kernels.hip -o /tmp/_d1regs.o 2>&1 | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/Function Name: _ZN2tk8k_arn_d1/ {split($0,a,"_ZN2tk8k_arn_d1"); n=substr(a[2],1,12)} n && / VGPRs:/ {v=$NF} n && /ScratchSize/ {sc=$NF} n && /Occupancy/ {o=$NF} n && /VGPRs Spill/ {print n, "vgpr", v, "occ", o, "spill", $NF, "scratch", sc; n=""}'
