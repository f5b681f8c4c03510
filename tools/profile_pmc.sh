#!/bin/bash
# PMC passes of the headline bench (one counter group per run) and the per-kernel HBM-byte
# summary, then the other BASELINE configurations' bench lines, into gpurun_out/<tag>/
# (the second half of tools/profile_round.sh, for a run split over two gpurun calls).
# usage: bash tools/profile_pmc.sh r03f
TAG=${1:-r03f}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT/pmc
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc/p$i -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > $OUT/pmc/p$i.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py $OUT/pmc nlse3d_512 16 134217728 $OUT/pmc_nlse3d_512.json k_tail 0.2857 || exit 1
timeout -k 10 300 python bench.py --workload nlse2d_4096 --no-cpu-baseline > $OUT/bench_nlse2d_4096.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload sg2d_8192 --no-cpu-baseline --steps 6 > $OUT/bench_sg2d_8192.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload g2_3d_256 --no-cpu-baseline > $OUT/bench_g2_3d_256.json 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload cq3d_1024 --no-cpu-baseline --steps 4 --warmup 1 > $OUT/bench_cq3d_1024.json 2>&1 || exit 1
