#!/bin/bash
# Round 3: isotropic passes at two workgroups per CU up to J = 6 / 8 (late J ring) vs base.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/nonlinear-solvers_amd
for r in 1 2; do
  for v in base v4 v5; do
    if [ $v = base ]; then unset NLS_AMD_LIB; else export NLS_AMD_LIB=$L/lib_$v/libnls_amd.so; fi
    timeout -k 10 200 python -u tools/p2_probe.py 512 16 3 > gpurun_out/ab_${v}_$r.log 2>&1 || exit 1
  done
done
unset NLS_AMD_LIB
for f in gpurun_out/ab_*.log; do echo "== $f"; grep "J= [468] \|update per step" $f; done
