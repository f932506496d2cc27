#!/bin/bash
# build an A/B variant of libtkhip.so into tools/_build/libtkhip_NAME.so
# usage: tools/build_variant.sh NAME [GIT_REV|-] [-DFLAG=V ...]   ("-" = working tree)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; rev=${2:--}; shift 2 || shift $#
mkdir -p $R/tools/_build
src=$R
if [ "$rev" != "-" ]; then
  src=$(mktemp -d)
  for f in include/tk.h tensorkrylov.jl_amd/csrc/tk_kernels.hip tensorkrylov.jl_amd/csrc/tk_abi.cpp tensorkrylov.jl_amd/csrc/tk_host.cpp tensorkrylov.jl_amd/csrc/tk_host.h tensorkrylov.jl_amd/csrc/tk_solver.cpp tensorkrylov.jl_amd/csrc/tk_internal.h tensorkrylov.jl_amd/csrc/tk_xsched.h; do
    mkdir -p $src/$(dirname $f); git -C $R show $rev:$f > $src/$f 2>/dev/null || rm -f $src/$f
  done
fi
hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -Xarch_host -mavx2 -Xarch_host -mfma -Wno-unused-value -Wno-unused-result "$@" \
  -I $src/include $src/tensorkrylov.jl_amd/csrc/tk_kernels.hip $src/tensorkrylov.jl_amd/csrc/tk_abi.cpp $( [ -f $src/tensorkrylov.jl_amd/csrc/tk_host.cpp ] && echo $src/tensorkrylov.jl_amd/csrc/tk_host.cpp ) $( [ -f $src/tensorkrylov.jl_amd/csrc/tk_solver.cpp ] && echo $src/tensorkrylov.jl_amd/csrc/tk_solver.cpp ) -pthread -lrccl \
  -o $R/tools/_build/libtkhip_$name.so
