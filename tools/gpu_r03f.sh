#!/bin/bash
# Round 3: march-form register pass k_p2m (G2): parity, bench A/B (march vs cell), rocprof stats.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_g2m
timeout -k 10 900 python -u -m pytest -q -m gpu tests/test_gpu_g2.py tests/test_gpu_pass2.py tests/test_gpu_multirank.py \
  --timeout 400 --timeout-method thread > gpurun_out/pytest_f.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_f.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload g2_3d_256 --no-cpu-baseline > gpurun_out/bench_g2_march.json 2>/dev/null || exit $?
NLS_P2G_FORM=cell timeout -k 10 300 python -u bench.py --workload g2_3d_256 --no-cpu-baseline > gpurun_out/bench_g2_cell.json 2>/dev/null || exit $?
NLS_PASS2=0 timeout -k 10 300 python -u bench.py --workload g2_3d_256 --no-cpu-baseline > gpurun_out/bench_g2_onevec.json 2>/dev/null || exit $?
for f in march cell onevec; do python3 -c "import json;d=json.load(open('gpurun_out/bench_g2_$f.json'));print('$f', round(d['value'],1), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_roofline']['gpu_kernel_ms_per_step'].items()})"; done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_g2m -o g2m -- python3 bench.py --workload g2_3d_256 --no-cpu-baseline --steps 3 --warmup 1 --prof-steps 1 > /dev/null 2>&1 || exit $?
exit $rc
