# New G2 cubic-quintic GPU tests first, then the full GPU suite.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_g2.py -x -v -m gpu -k cq --timeout 120 --timeout-method thread > gpurun_out/t_cq.log 2>&1; rc=$?
tail -5 gpurun_out/t_cq.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_all.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_all.log
exit $rc
