#!/bin/bash
# Round 3: sEWI through the two-vector passes; G2 tile-depth sensitivity.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -m gpu tests/test_gpu_g2.py --timeout 400 --timeout-method thread > gpurun_out/pytest_h.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_h.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload sewi_3d_256 --no-cpu-baseline > gpurun_out/bench_sewi.json 2>/dev/null || exit $?
NLS_PASS2=0 timeout -k 10 300 python -u bench.py --workload sewi_3d_256 --no-cpu-baseline > gpurun_out/bench_sewi_onevec.json 2>/dev/null || exit $?
for kz in 8 16 64; do
  NLS_KZ=$kz timeout -k 10 300 python -u bench.py --workload g2_3d_256 --no-cpu-baseline > gpurun_out/bench_g2_kz$kz.json 2>/dev/null || exit $?
done
for f in sewi sewi_onevec g2_kz8 g2_kz16 g2_kz64; do python3 -c "import json;d=json.load(open('gpurun_out/bench_$f.json'));print('$f', round(d['value'],1), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_roofline']['gpu_kernel_ms_per_step'].items()})"; done
exit $rc
