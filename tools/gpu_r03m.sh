#!/bin/bash
# Round 3: G2 256^3 kernel stats under rocprofv3 (ANI k_p2d) + isotropic passes at 256^3.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g2 -o g2 -- python3 bench.py --workload g2_3d_256 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bench_g2_prof.json 2> gpurun_out/prof_g2.err || exit $?
find gpurun_out/prof_g2 -name "*stats*" | head
timeout -k 10 200 python -u tools/p2_probe.py 256 16 3 > gpurun_out/p2_probe_256.txt 2>&1 || exit $?
cat gpurun_out/p2_probe_256.txt
