cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_stiff.py tests/test_gpu_drivers.py > gpurun_out/t_stiff.log 2>&1; rc=$?
tail -30 gpurun_out/t_stiff.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_gpu_c5.py > gpurun_out/t_c5.log 2>&1; rc2=$?
tail -15 gpurun_out/t_c5.log
exit $rc2
