#!/bin/bash
# Tile-depth sweep of the fused tail kernels at 512^3 m=16 (k_alpha_l2: NLS_KZ_ALPHA2,
# k_final_fused: NLS_KZ_FUSED), timing classes from bench.py.
set -e
O=gpurun_out/ftune; mkdir -p $O
for a in 4 8 16 32; do
  NLS_KZ_ALPHA2=$a timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 > $O/a$a.json
done
for f in 8 16 64 128; do
  NLS_KZ_FUSED=$f timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 > $O/f$f.json
done
