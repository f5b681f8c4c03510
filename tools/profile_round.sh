# Full measurement pass for profiles/<tag>: bench (default), rocprofv3 kernel-trace
# stats of the same command, PMC traffic passes.  Usage: bash tools/profile_round.sh r01
set -e
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench_nlse3d_512.json 2> $OUT/bench_nlse3d_512.err
timeout -k 10 300 python bench.py --workload nlse2d_4096 --no-cpu-baseline > $OUT/bench_nlse2d_4096.json 2>&1
timeout -k 10 300 python bench.py --workload sg2d_8192 --no-cpu-baseline --steps 6 > $OUT/bench_sg2d_8192.json 2>&1
timeout -k 10 300 python bench.py --workload g2_3d_256 > $OUT/bench_g2_3d_256.json 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/trace.log 2>&1
bash tools/pmc_run.sh nlse3d_512
