#!/bin/bash
# default (mult 16) vs persistent grid (mult 1) on the 2D / SG / G2 workloads
set -e
mkdir -p gpurun_out/grid2
for w in nlse2d_4096 sg2d_8192 g2_3d_256 nlse3d_512; do
  for g in 1 16; do
    NLS_GRID_MULT=$g timeout -k 10 240 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/grid2/${w}_g$g.json
  done
done
