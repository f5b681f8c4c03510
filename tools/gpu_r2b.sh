cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_gautschi.py tests/test_gpu_kg.py tests/test_gpu_parity.py > gpurun_out/t_gg.log 2>&1; rc=$?
tail -25 gpurun_out/t_gg.log
exit $rc
