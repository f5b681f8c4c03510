#!/bin/bash
# graph/edge tests, then the tile-depth x graph sweep over small grids
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sg2
bash tools/run_checked.sh timeout -k 10 400 python -m pytest tests/test_gpu_graph.py tests/test_gpu_edges.py -q > gpurun_out/sg2/tests.log 2>&1
timeout -k 10 600 python tools/sweep_small.py > gpurun_out/sg2/sweep.jsonl 2> gpurun_out/sg2/sweep.err
