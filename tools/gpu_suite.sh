# The full GPU test suite in one process (round-end check).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_all.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_all.log
exit $rc
