set -e
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_all.log 2>&1 || { echo "pytest failed rc=$?" >> gpurun_out/pytest_all.log; exit 1; }
