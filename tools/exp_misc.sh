#!/bin/bash
set -e
O=gpurun_out/misc; mkdir -p $O
timeout -k 10 200 python bench.py --n 256 --no-cpu-baseline --steps 10 > $O/b256.json
NLS_FORCE_RCCL=1 timeout -k 10 200 python bench.py --n 256 --no-cpu-baseline --steps 10 > $O/b256_rccl.json 2>/dev/null
