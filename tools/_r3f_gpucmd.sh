set -o pipefail
mkdir -p gpurun_out/r3f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3f/suite.txt 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3f/smoke.txt 2>&1 && \
timeout -k 10 180 python bench.py > gpurun_out/r3f/bench.json 2> gpurun_out/r3f/bench.err
