#!/bin/bash
# Per-GPU proxy of the 8-GPU strong-scaling slab (512^3 / 8 = 256^3 cells):
# bench at n=256, plus a kernel trace to measure idle gaps between launches.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/small
timeout -k 10 300 python bench.py --n 256 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/small/bench256.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/small/trace -o run -- python3 bench.py --n 256 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/small/trace.log 2>&1
