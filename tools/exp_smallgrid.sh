#!/bin/bash
# Small-grid step latency: where is the time at sizes far below the chip
# (the reference's own test sizes, SURVEY configs[0] = 2D 256^2)?
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sg
for n in 128 256 512 1024; do
  for kz in 0 4 8; do
    if [ $kz = 0 ]; then unset NLS_KZ; else export NLS_KZ=$kz; fi
    timeout -k 10 120 python bench.py --workload nlse2d_4096 --n $n --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/sg/2d_${n}_kz$kz.json
  done
done
unset NLS_KZ
for n in 32 64 128; do
  for kz in 0 4 8; do
    if [ $kz = 0 ]; then unset NLS_KZ; else export NLS_KZ=$kz; fi
    timeout -k 10 120 python bench.py --n $n --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/sg/3d_${n}_kz$kz.json
  done
done
unset NLS_KZ
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sg/trace -o run -- python3 bench.py --workload nlse2d_4096 --n 256 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/sg/trace.log 2>&1
