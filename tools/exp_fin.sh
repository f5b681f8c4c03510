set -e
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_drivers.py -x -q -m gpu > gpurun_out/pytest_fin.log 2>&1 || { tail -40 gpurun_out/pytest_fin.log; exit 1; }
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/fin$i.json 2>&1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 8 --warmup 2 --workload nlse2d_4096 > gpurun_out/fin_2d.json 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 --workload sg2d_8192 > gpurun_out/fin_sg.json 2>&1
