#!/bin/bash
# Round 3 (session 2): the GPU suite with the parity record, the headline bench
# line, the G2 / sEWI bench lines and the per-rank slab probe.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/parity.jsonl
NLS_PARITY_LOG=$PWD/gpurun_out/parity.jsonl timeout -k 10 900 python -u -m pytest tests --maxfail=10 -q -m gpu \
  --timeout 400 --timeout-method thread > gpurun_out/pytest_all.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_all.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
for wl in g2_3d_256 sewi_3d_256; do
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline > gpurun_out/bench_$wl.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_$wl.json'));print('$wl', round(d['value'],1), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_roofline']['gpu_kernel_ms_per_step'].items()})"
done
timeout -k 10 400 python -u tools/slab_probe.py > gpurun_out/slab_probe.txt 2>&1 || exit $?
grep -v "version\|Hostname\|Librccl" gpurun_out/slab_probe.txt
exit $rc
