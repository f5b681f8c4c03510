set -e
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest3.log 2>&1
for cfg in "R0G1" "R1G1" "R0G2" "R0G4"; do
  r=${cfg:1:1}; gm=${cfg:3:1}
  NLS_TILE_REMAP=$r NLS_GRID_MULT=$gm timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/v2_$cfg.json 2>&1
done
NLS_VEC_PAD=0 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/v2_pad0.json 2>&1
