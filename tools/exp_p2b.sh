#!/bin/bash
# pass2 variants at 512^3: kz 64 / 128, one-row waves from J = 12 (default) / 10 (lib_v)
set -e
O=gpurun_out/p2b
mkdir -p $O
L=$PWD/nonlinear-solvers_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_pass2.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/base.json 2>&1
NLS_PASS2=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/p2.json 2>&1
NLS_PASS2=1 NLS_P2_KZ=128 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/p2kz128.json 2>&1
NLS_AMD_LIB=$L/lib_v/libnls_amd.so NLS_PASS2=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/p2rb10.json 2>&1
NLS_PASS2=1 timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/perj_p2.json
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/base2.json 2>&1
