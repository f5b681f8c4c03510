set -e
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest4.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/v3.json 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 --workload nlse2d_4096 > gpurun_out/v3_2d.json 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 --workload sg2d_8192 > gpurun_out/v3_sg.json 2>&1
