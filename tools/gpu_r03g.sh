#!/bin/bash
# Round 3: lap overlap for the register passes, p2kz rule (>= 1024 tiles): parity + benches.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -m gpu tests/test_gpu_g2.py tests/test_gpu_pass2.py tests/test_gpu_multirank.py \
  tests/test_gpu_oplog.py tests/test_gpu_graph.py --timeout 400 --timeout-method thread > gpurun_out/pytest_g.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_g.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for w in g2_3d_256 nlse2d_4096 sg2d_8192; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.json 2>/dev/null || exit $?
done
NLS_P2_KZ=32 timeout -k 10 300 python -u bench.py --workload nlse2d_4096 --no-cpu-baseline > gpurun_out/bench_nlse2d_4096_kz32.json 2>/dev/null || exit $?
for f in g2_3d_256 nlse2d_4096 nlse2d_4096_kz32 sg2d_8192; do python3 -c "import json;d=json.load(open('gpurun_out/bench_$f.json'));print('$f', round(d['value'],1), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_roofline']['gpu_kernel_ms_per_step'].items()})"; done
timeout -k 10 600 python -u tools/slab_probe.py 0 2 6 7 > gpurun_out/slab_probe_g.txt 2>&1 || exit $?
grep -v "version\|Hostname\|Librccl" gpurun_out/slab_probe_g.txt
exit $rc
