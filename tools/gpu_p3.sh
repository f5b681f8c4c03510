# Three-vector passes: parity tests, then per-pass timing and the headline bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pass2.py tests/test_gpu_stiff.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_p3.log 2>&1; rc=$?
tail -5 gpurun_out/t_p3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/p2_probe.py 512 16 3 > gpurun_out/p3_probe.log 2>&1; rc=$?
cat gpurun_out/p3_probe.log
[ $rc -eq 0 ] || exit $rc
NLS_PASS3=0 timeout -k 10 200 python -u tools/p2_probe.py 512 16 3 > gpurun_out/p3_probe0.log 2>&1; rc=$?
cat gpurun_out/p3_probe0.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_p3.json 2> gpurun_out/bench_p3.err; rc=$?
cat gpurun_out/bench_p3.json
exit $rc
