#!/bin/bash
set -e
O=gpurun_out/qa6; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
NLS_FUSED_ALPHA=1 NLS_DEBUG_ALPHA=1 timeout -k 10 300 python tools/qa_diag2.py > $O/diag2.log 2>&1
timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/perj_on.json
NLS_FUSED_ALPHA=0 timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/perj_off.json
for a in 1 0; do
  NLS_FUSED_ALPHA=$a timeout -k 10 200 python bench.py --n 256 --no-cpu-baseline --steps 10 > $O/n256_a$a.json
  NLS_FUSED_ALPHA=$a timeout -k 10 200 python bench.py --workload nlse2d_4096 --no-cpu-baseline --steps 10 > $O/n2d_a$a.json
done
