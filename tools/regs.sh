#!/bin/bash
# Register / occupancy report of the stencil kernels of one variant (iso3 iso2 ani3 ani2),
# filtered by an optional regex on the mangled name; EXTRA="-D..." adds flags.  usage: bash tools/regs.sh iso3 [regex]
V=${1:-iso3}; RE=${2:-.}
ANI=$([[ $V == ani* ]] && echo 1 || echo 0); DIM=${V: -1}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Inonlinear-solvers_amd/csrc \
  $EXTRA -DNLS_ANI=$ANI -DNLS_DIM=$DIM -DNLS_TABLE=stencil_table_$V -c nonlinear-solvers_amd/csrc/nls_stencil.hip \
  -o /tmp/regs_$V.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|AGPRs|Spill|Occupancy" | paste - - - - - - |
  sed -E 's/[^ ]*nls_stencil.hpp:[0-9:]* remark://g; s/\[-Rpass-analysis=kernel-resource-usage\]//g; s/Function Name: //' |
  awk '{$1=$1; print}' | grep -E "$RE"
