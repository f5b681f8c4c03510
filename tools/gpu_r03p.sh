#!/bin/bash
# Round 3: full GPU suite on the current code + headline, G2 and sEWI bench lines.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests --maxfail=5 -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_p.log 2>&1; rc=$?
tail -8 gpurun_out/pytest_p.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_p.json 2> gpurun_out/bench_p.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/bench_p.json'));print('nlse3d_512', round(d['value'],1), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_roofline']['gpu_kernel_ms_per_step'].items()})"
for wl in g2_3d_256 sewi_3d_256; do
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline > gpurun_out/bench_p_$wl.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_p_$wl.json'));print('$wl', round(d['value'],1), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_roofline']['gpu_kernel_ms_per_step'].items()})"
done
