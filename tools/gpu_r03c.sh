#!/bin/bash
# Round 3: split-pass boundary kernels -- slab parity tests, op log, slab probe.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -m gpu tests/test_gpu_multirank.py tests/test_gpu_oplog.py \
  tests/test_gpu_scale_slabs.py tests/test_gpu_c5.py --timeout 400 --timeout-method thread > gpurun_out/pytest_c.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_c.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/slab_probe.py > gpurun_out/slab_probe_c.txt 2>&1 || exit $?
grep -v "version\|Hostname\|Librccl" gpurun_out/slab_probe_c.txt
exit $rc
