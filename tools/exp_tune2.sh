set -e
for kz in 4 8 12 16; do
  NLS_KZ=$kz timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/t2_3d_kz${kz}.json 2>&1
done
for kz in 4 8 16 32; do
  NLS_KZ=$kz timeout -k 10 200 python bench.py --no-cpu-baseline --steps 8 --warmup 2 --workload nlse2d_4096 > gpurun_out/t2_2d_kz${kz}.json 2>&1
done
