#!/bin/bash
set -e
O=gpurun_out/qa3; mkdir -p $O
for a in 1 0; do
  NLS_FUSED_ALPHA=$a timeout -k 10 200 python bench.py --n 256 --no-cpu-baseline --steps 10 > $O/n256_a$a.json
  NLS_FUSED_ALPHA=$a timeout -k 10 200 python bench.py --workload nlse2d_4096 --no-cpu-baseline --steps 10 > $O/n2d_a$a.json
  NLS_FUSED_ALPHA=$a timeout -k 10 200 python bench.py --workload kg_3d_256 --no-cpu-baseline --steps 10 > $O/kg_a$a.json
  NLS_FUSED_ALPHA=$a timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 > $O/n512_a$a.json
done
