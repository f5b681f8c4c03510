set -e
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q -m gpu > gpurun_out/pytest_red.log 2>&1 || { tail -40 gpurun_out/pytest_red.log; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/red.json 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 8 --warmup 2 --workload nlse2d_4096 > gpurun_out/red_2d.json 2>&1
