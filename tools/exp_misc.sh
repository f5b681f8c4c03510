#!/bin/bash
set -e
O=gpurun_out/misc; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_all.log 2>&1
python -c "import torch; f,t=torch.cuda.mem_get_info(); print('free',f/1e9,'total',t/1e9)" > $O/mem.txt 2>&1
timeout -k 10 500 python bench.py --workload cq3d_1024 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_cq1024.json 2> $O/bench_cq1024.err
