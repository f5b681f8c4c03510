#!/bin/bash
set -e
O=gpurun_out/misc; mkdir -p $O
timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/perj.json
NLS_FORCE_RCCL=1 timeout -k 10 240 python bench.py --no-cpu-baseline --steps 6 > $O/bench_rccl1.json 2> $O/bench_rccl1.err
