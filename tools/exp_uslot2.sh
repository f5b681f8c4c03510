#!/bin/bash
set -e
O=gpurun_out/uslot2; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/base_r$rep.json
  NLS_U_SLOT=1 timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/uslot_r$rep.json
  NLS_VEC_PAD=2048 timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/p2048_r$rep.json
done
