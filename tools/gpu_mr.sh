cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_pass2.py > gpurun_out/t_mr.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/t_mr.log | tail -30
exit $rc
