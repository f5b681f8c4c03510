set -e
for cfg in "16 1" "16 64" "32 64" "64 64" "128 64"; do
  set -- $cfg
  NLS_KZ=$1 NLS_GRID_MULT=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/full_kz$1_g$2.json 2>&1
done
