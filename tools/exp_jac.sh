#!/bin/bash
# A/B of the device eigensolve (k_reduce_final): one-barrier register Jacobi (default)
# vs a variant library built with other flags into lib_jac1 (tools/build_variant.sh); parity tests first.
set -e
export TMPDIR=/tmp
O=gpurun_out/jac
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_fused.py \
  -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in new old; do
  L=$PWD/nonlinear-solvers_amd/lib/libnls_amd.so
  [ $v = old ] && L=$PWD/nonlinear-solvers_amd/lib_jac1/libnls_amd.so
  for w in nlse2d_4096 g2_3d_256; do
  NLS_AMD_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_${v}_$w -o run -- \
    python3 bench.py --no-cpu-baseline --steps 4 --warmup 1 --workload $w > $O/bench_${v}_$w.json 2>&1
  done
done
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; grep -E "reduce_final|k_tail" "$f" | cut -c1-200; done
