#!/bin/bash
set -e
O=gpurun_out/qa5; mkdir -p $O
L=$GRAFT_REPO_ROOT/nonlinear-solvers_amd
timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/base.json
NLS_FUSED_ALPHA=0 timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/off.json
NLS_AMD_LIB=$L/lib_v/libnls_amd.so timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/noseam.json
NLS_AMD_LIB=$L/lib_v2/libnls_amd.so timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/nopeek.json
NLS_AMD_LIB=$L/lib_v3/libnls_amd.so timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/noboth.json
