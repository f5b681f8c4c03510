#!/bin/bash
set -e
O=gpurun_out/uslot3; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/base_r$rep.json
  for off in 1024 2048 3072; do
    NLS_U_SLOT=1 NLS_U_OFF=$off timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/u${off}_r$rep.json
  done
done
