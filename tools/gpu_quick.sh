# Core parity tests + the headline bench (after a tail/pass change)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pass2.py tests/test_gpu_fused.py tests/test_gpu_g2.py tests/test_gpu_drivers.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_quick.log 2>&1; rc=$?
tail -3 gpurun_out/t_quick.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err; rc=$?
python3 -c "import json;d=json.load(open('gpurun_out/bench_q.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'][:30],d['roofline']['avg_launch_ms'],d['roofline']['frac'],d['step_roofline']['gpu_kernel_ms_per_step'])"
exit $rc
