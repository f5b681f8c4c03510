# Final-tree bench set of round 3: every BASELINE configuration plus KG, one box, one process each.
set -o pipefail
mkdir -p gpurun_out/r3b
for w in nlse2d_4096 sg2d_8192 g2_3d_256 kg_3d_256 cq3d_1024 nlse3d_512; do
  timeout -k 10 240 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/r3b/bench_$w.json 2> gpurun_out/r3b/bench_$w.err || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b/prof2d -o run -- python3 bench.py --workload nlse2d_4096 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3b/bench_2d_under_rocprof.json 2> gpurun_out/r3b/prof2d.err
