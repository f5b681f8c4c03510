#!/bin/bash
# Vector-stride pad sweep at 512^3 (elements of 16 B): update / tail times per pad.
set -e
O=gpurun_out/pad3; rm -rf $O; mkdir -p $O
hostname > $O/host.txt 2>/dev/null || true
for rep in 1 2; do
for pad in 256 4096 1048576 67108864 8192 2048; do
  NLS_VEC_PAD=$pad timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/p${pad}_r$rep.json
done
done
