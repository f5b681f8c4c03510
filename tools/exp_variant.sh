#!/bin/bash
# A/B of a compile-time variant library (nonlinear-solvers_amd/lib_v, built with
# extra -D flags) against the default one, on the given bench workloads.
# usage: bash tools/exp_variant.sh tag workload [workload ...]
set -e
TAG=$1; shift
mkdir -p gpurun_out/var_$TAG
for w in "$@"; do
  for rep in 1 2; do
    timeout -k 10 240 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/var_$TAG/${w}_base$rep.json
    NLS_AMD_LIB=$GRAFT_REPO_ROOT/nonlinear-solvers_amd/lib_v/libnls_amd.so timeout -k 10 240 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/var_$TAG/${w}_var$rep.json
  done
done
