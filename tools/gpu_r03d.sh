#!/bin/bash
# Round 3: boundary kernels (split slabs) + register two-vector passes (G2, odd shapes):
# parity tests, the slab probe and the G2 bench line.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -m gpu tests/test_gpu_multirank.py tests/test_gpu_oplog.py \
  tests/test_gpu_g2.py tests/test_gpu_pass2.py --timeout 400 --timeout-method thread > gpurun_out/pytest_d.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_d.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload g2_3d_256 --no-cpu-baseline > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err || exit $?
cat gpurun_out/bench_g2.json
timeout -k 10 600 python -u tools/slab_probe.py > gpurun_out/slab_probe_d.txt 2>&1 || exit $?
grep -v "version\|Hostname\|Librccl" gpurun_out/slab_probe_d.txt
exit $rc
