#!/bin/bash
# GPU tests, then A/B of the fused tail (NLS_FUSED_TAIL=1 default vs 0) on the bench workloads.
set -e
mkdir -p gpurun_out/fused
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/fused/pytest.log 2>&1
for w in nlse3d_512 nlse2d_4096 g2_3d_256; do
  timeout -k 10 240 python bench.py --workload $w --no-cpu-baseline > gpurun_out/fused/${w}_on.json
  NLS_FUSED_TAIL=0 timeout -k 10 240 python bench.py --workload $w --no-cpu-baseline > gpurun_out/fused/${w}_off.json
done
