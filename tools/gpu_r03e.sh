#!/bin/bash
# Round 3: boundary kernels v2 (split into X / Z waves, scalar coefficients) + k_p2g with
# scalar coefficients: parity tests, slab probe, rocprof kernel stats of the G2 bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_g2
timeout -k 10 900 python -u -m pytest -q -m gpu tests/test_gpu_multirank.py tests/test_gpu_oplog.py \
  tests/test_gpu_g2.py tests/test_gpu_pass2.py --timeout 400 --timeout-method thread > gpurun_out/pytest_e.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_e.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/slab_probe.py 0 2 3 4 5 > gpurun_out/slab_probe_e.txt 2>&1 || exit $?
grep -v "version\|Hostname\|Librccl" gpurun_out/slab_probe_e.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g2 -o g2 -- python3 bench.py --workload g2_3d_256 --no-cpu-baseline --steps 5 --warmup 1 --prof-steps 1 > gpurun_out/bench_g2e.json 2> gpurun_out/bench_g2e.err || exit $?
cat gpurun_out/bench_g2e.json
find gpurun_out/prof_g2 -name "*kernel_stats.csv" | head -3
exit $rc
