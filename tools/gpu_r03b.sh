#!/bin/bash
# Round 3: stiff parity tests with the parity record + the slab probe variants.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/parity.jsonl
NLS_PARITY_LOG=$PWD/gpurun_out/parity.jsonl timeout -k 10 900 python -u -m pytest -v -m gpu \
  tests/test_gpu_stiff.py tests/test_gpu_drivers.py tests/test_gpu_oplog.py \
  --timeout 400 --timeout-method thread > gpurun_out/pytest_b.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_b.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/slab_probe.py > gpurun_out/slab_probe.txt 2>&1 || exit $?
grep -v "version\|Hostname\|Librccl" gpurun_out/slab_probe.txt
exit $rc
