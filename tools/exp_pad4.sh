#!/bin/bash
set -e
O=gpurun_out/pad4; mkdir -p $O
for w in nlse2d_4096 sg2d_8192 g2_3d_256; do
for pad in 256 4096 2048; do
  NLS_VEC_PAD=$pad timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --steps 6 > $O/${w}_p$pad.json
done
done
for pad in 256 4096; do
  NLS_VEC_PAD=$pad timeout -k 10 200 python bench.py --n 256 --no-cpu-baseline --steps 10 > $O/n256_p$pad.json
done
