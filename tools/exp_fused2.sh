#!/bin/bash
# GPU tests, then A/B of the fused tails (NLS_FUSED_TAIL=1 default vs 0) on the other workloads.
set -e
mkdir -p gpurun_out/fused2
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/fused2/pytest.log 2>&1
for w in sg2d_8192 kg_3d_256 sewi_3d_256 nlse3d_512; do
  timeout -k 10 240 python bench.py --workload $w --no-cpu-baseline --steps 6 > gpurun_out/fused2/${w}_on.json
  NLS_FUSED_TAIL=0 timeout -k 10 240 python bench.py --workload $w --no-cpu-baseline --steps 6 > gpurun_out/fused2/${w}_off.json
done
