#!/bin/bash
set -e
O=gpurun_out/perj; mkdir -p $O
timeout -k 10 300 python tools/qa_diag2.py > $O/diag2.log 2>&1
timeout -k 10 300 python tools/qa_diag.py > $O/diag.log 2>&1
timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/q4_base.json
NLS_AMD_LIB=$GRAFT_REPO_ROOT/nonlinear-solvers_amd/lib_v/libnls_amd.so timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/q4_rb2.json
NLS_FUSED_ALPHA=0 timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/q4_off.json
