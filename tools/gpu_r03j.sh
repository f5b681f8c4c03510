#!/bin/bash
# Round 3: the G2 operator through k_p2d (c staged beside S_J): parity + benches.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -m gpu tests/test_gpu_g2.py -x --timeout 300 --timeout-method thread > gpurun_out/pytest_j.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_j.log
[ $rc -eq 0 ] || exit $rc
for wl in g2_3d_256 sewi_3d_256; do
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline > gpurun_out/bench_$wl.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_$wl.json'));print('$wl', round(d['value'],1), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_roofline']['gpu_kernel_ms_per_step'].items()})"
done
exit 0
