#!/bin/bash
# alpha tile depth sweep (3D 512^3, 2D 4096^2)
set -e
mkdir -p gpurun_out/kza
for kz in 2 4 8; do
  NLS_KZ_ALPHA=$kz timeout -k 10 240 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/kza/3d_kz$kz.json
done
for kz in 4 8 16 32; do
  NLS_KZ_ALPHA=$kz timeout -k 10 240 python bench.py --workload nlse2d_4096 --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/kza/2d_kz$kz.json
done
timeout -k 10 240 python bench.py --n 256 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/kza/3d256_default.json
