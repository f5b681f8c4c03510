#!/bin/bash
set -e
O=gpurun_out/l2; mkdir -p $O
for kz in 8 32; do
  NLS_KZ_ALPHA2=$kz timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/rb4_kz$kz.json
  NLS_KZ_ALPHA2=$kz NLS_AMD_LIB=$GRAFT_REPO_ROOT/nonlinear-solvers_amd/lib_v/libnls_amd.so timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/rb2_kz$kz.json
  NLS_KZ_ALPHA2=$kz NLS_AMD_LIB=$GRAFT_REPO_ROOT/nonlinear-solvers_amd/lib_v2/libnls_amd.so timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/rb1_kz$kz.json
done
