#!/bin/bash
# eigensolve phase timings (wall_clock64) of the two Jacobi variants
set -e
O=gpurun_out/jacdbg
mkdir -p $O
for v in dbg; do
  for w in nlse2d_4096 g2_3d_256; do
    NLS_AMD_LIB=$PWD/nonlinear-solvers_amd/lib_$v/libnls_amd.so timeout -k 10 200 \
      python bench.py --no-cpu-baseline --steps 2 --warmup 1 --workload $w > $O/${v}_$w.log 2>&1
  done
done
grep -h "jacobi" $O/*.log | sort | uniq -c | head -40
