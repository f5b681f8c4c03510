set -e
for kz in 16 32 64; do for gm in 1 8; do
  NLS_KZ=$kz NLS_GRID_MULT=$gm timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/tune_kz${kz}_g${gm}.json 2>&1
done; done
