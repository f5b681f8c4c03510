set -e
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest2.log 2>&1
for pad in 0 64 256 1088; do
  NLS_VEC_PAD=$pad timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/pad_$pad.json 2>&1
done
