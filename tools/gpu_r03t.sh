#!/bin/bash
# Round 3: interior fast path of the k_p2d stencil rows (A/B vs NLS_P2D_FAST=0), iso
# 512^3 per pass and G2 256^3 per pass; then the split-boundary variants.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/nonlinear-solvers_amd/lib_nofast/libnls_amd.so
for r in 1 2; do
  timeout -k 10 200 python -u tools/p2_probe.py 512 16 3 > gpurun_out/fast_iso_$r.log 2>&1 || exit 1
  NLS_AMD_LIB=$V timeout -k 10 200 python -u tools/p2_probe.py 512 16 3 > gpurun_out/nofast_iso_$r.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/g2_probe.py "" NLS_AMD_LIB=$V "" NLS_AMD_LIB=$V > gpurun_out/fast_g2.log 2>&1 || exit 1
for f in gpurun_out/fast_iso_*.log gpurun_out/nofast_iso_*.log; do echo "== $f"; grep "J=\|update per step" $f; done
cat gpurun_out/fast_g2.log
timeout -k 10 300 python -u tools/slab_probe.py 2 13 5 > gpurun_out/slab_probe4.txt 2>&1 || exit 1
grep -v "version\|Hostname\|Librccl" gpurun_out/slab_probe4.txt | cut -c1-110
