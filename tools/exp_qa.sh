#!/bin/bash
# Folded-alpha check: the new tests first, then all GPU tests, then A/B benches.
set -e
O=gpurun_out/qa; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 120 --timeout-method thread > $O/pytest_fused.log 2>&1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for w in nlse3d_512 nlse2d_4096 sg2d_8192 g2_3d_256; do
  timeout -k 10 240 python bench.py --workload $w --no-cpu-baseline --steps 6 > $O/${w}_on.json
  NLS_FUSED_ALPHA=0 timeout -k 10 240 python bench.py --workload $w --no-cpu-baseline --steps 6 > $O/${w}_off.json
done
