#!/bin/bash
# QA update passes: one row per thread from J = 13 (lib_v) / 12 (lib_v2) vs default, per-J times at 512^3
set -e
O=gpurun_out/qarb
mkdir -p $O
L=$PWD/nonlinear-solvers_amd
timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/base.json
NLS_AMD_LIB=$L/lib_v/libnls_amd.so timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/rb13.json
NLS_AMD_LIB=$L/lib_v2/libnls_amd.so timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/rb12.json
timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/base2.json
