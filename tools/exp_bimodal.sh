#!/bin/bash
# Run-to-run distribution of the fused tail kernel time at 512^3 (separate processes),
# u in its own allocation vs in the basis allocation (NLS_U_SLOT=1), alpha_l2 tile depth 32.
set -e
O=gpurun_out/bimodal; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 > $O/base$i.json
  NLS_U_SLOT=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 > $O/uslot$i.json
  NLS_KZ_ALPHA2=32 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 > $O/a32_$i.json
done
