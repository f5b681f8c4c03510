#!/bin/bash
# collective-path overhead on one GPU: 256^3 (the 8-GPU slab size) plain vs 1-rank RCCL,
# boundary-plane launches on the halo stream (default) vs in order (NLS_BND_SIDE=0)
set -e
O=gpurun_out/coll
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_mr.log 2>&1 || { tail -30 $O/pytest_mr.log; exit 1; }
tail -1 $O/pytest_mr.log
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --n 256 --steps 10 --warmup 2 > $O/plain$i.json 2>&1
NLS_FORCE_RCCL=1 timeout -k 10 200 python bench.py --no-cpu-baseline --n 256 --steps 10 --warmup 2 > $O/rccl$i.json 2>&1
NLS_BND_PRIO=1 NLS_FORCE_RCCL=1 timeout -k 10 200 python bench.py --no-cpu-baseline --n 256 --steps 10 --warmup 2 > $O/rcclprio$i.json 2>&1
NLS_BND_SIDE=0 NLS_FORCE_RCCL=1 timeout -k 10 200 python bench.py --no-cpu-baseline --n 256 --steps 10 --warmup 2 > $O/rcclinorder$i.json 2>&1
done
