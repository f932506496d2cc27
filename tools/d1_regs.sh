#!/bin/bash
# VGPRs / occupancy / spills of every k_arn_d1 instance (extra hipcc flags as arguments)
R=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && hipcc --offload-arch=gfx950 -O3 -std=c++17 -c --cuda-device-only "$@" -Rpass-analysis=kernel-resource-usage \
  -I $R/include $R/tensorkrylov.jl_amd/csrc/tk_kernels.hip -o /tmp/_d1regs.o > /tmp/_d1regs.txt 2>&1
python3 $R/tools/d1_regs.py /tmp/_d1regs.txt
