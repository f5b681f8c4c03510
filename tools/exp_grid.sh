#!/bin/bash
# Grid-size sweep of the stencil passes (NLS_GRID_MULT x occupancy x CUs workgroups;
# large grids use the parallel k_colsum reduction).
set -e
mkdir -p gpurun_out/grid
NLS_GRID_MULT=64 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_g2.py tests/test_gpu_multirank.py -x -q -p no:cacheprovider > gpurun_out/grid/pytest_g64.log 2>&1
for g in 1 2 4 8 16 32 64; do
  NLS_GRID_MULT=$g timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/grid/g$g.json
done
for g in 1 64; do
  NLS_GRID_MULT=$g timeout -k 10 240 python bench.py --workload g2_3d_256 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/grid/g2_g$g.json
done
