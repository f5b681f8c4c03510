#!/bin/bash
# Round-end check: full GPU suite, then default vs two-vector pass (J=4 one-row waves) at 512^3
set -e
O=gpurun_out/p2c
mkdir -p $O
rm -f $O/*.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/base$i.json 2>&1
NLS_PASS2=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/p2_$i.json 2>&1
done
NLS_PASS2=1 timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/perj_p2.json
