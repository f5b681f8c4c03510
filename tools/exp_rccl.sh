set -e
timeout -k 10 300 python -m pytest tests/test_gpu_multirank.py -x -q -m gpu > gpurun_out/pytest_mr.log 2>&1 || { echo "rc=$?" >> gpurun_out/pytest_mr.log; exit 1; }
NLS_FORCE_RCCL=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/bench_forcerccl.json 2>&1
