#!/bin/bash
# Round 3, first GPU pass: the GPU suite with the parity record, the headline
# bench line, and the per-rank slab probe (split-launch overhead).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/parity.jsonl
NLS_PARITY_LOG=$PWD/gpurun_out/parity.jsonl timeout -k 10 1500 python -u -m pytest tests --maxfail=10 -v -m gpu \
  --timeout 400 --timeout-method thread > gpurun_out/pytest_all.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_all.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
timeout -k 10 600 python -u tools/slab_probe.py > gpurun_out/slab_probe.txt 2>&1 || exit $?
cat gpurun_out/slab_probe.txt
exit $rc
