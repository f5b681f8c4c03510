#!/bin/bash
# tile depth (update kz x alpha kz) at the benchmark sizes
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sg3
timeout -k 10 500 python tools/sweep_small.py --sizes "3:256,384,512" --dims 3 --kz 1,2,4,8,16,32 --kza 1,2,4 --graph 0 > gpurun_out/sg3/sweep3d.jsonl 2> gpurun_out/sg3/sweep3d.err
timeout -k 10 400 python tools/sweep_small.py --sizes "2:2048,4096" --dims 2 --kz 1,2,4,8,16 --kza 1,2,4,16 --graph 0 > gpurun_out/sg3/sweep2d.jsonl 2> gpurun_out/sg3/sweep2d.err
