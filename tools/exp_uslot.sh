#!/bin/bash
# u placement (slot m + offset) repeatability, and basis stride pad sweep
set -e
mkdir -p gpurun_out/uslot3
for i in 1 2 3; do
  for off in 128 2048; do
    NLS_U_SLOT=1 NLS_U_OFF=$off timeout -k 10 240 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/uslot3/off${off}_$i.json
  done
done
for pad in 128 384 512 768 1280; do
  NLS_U_SLOT=1 NLS_U_OFF=128 NLS_VEC_PAD=$pad timeout -k 10 240 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/uslot3/pad$pad.json
done
