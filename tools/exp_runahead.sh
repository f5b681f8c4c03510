#!/bin/bash
# host run-ahead bound: long single-call step sequences vs short ones
set -e
mkdir -p gpurun_out/ra
: > gpurun_out/ra/all.log
for ra in 0 3; do
  for st in 10 60; do
    echo "ra=$ra steps=$st $(NLS_RUNAHEAD=$ra timeout -k 10 300 python bench.py --n 384 --steps $st --warmup 2 --no-cpu-baseline | cut -c1-220)" >> gpurun_out/ra/all.log
  done
done
python3 - <<'PY'
import numpy as np
n = 384
x = np.linspace(-10, 10, n)
Z, Y, X = np.meshgrid(x, x, x, indexing="ij")
np.save("/tmp/u0_384.npy", (np.exp(-(X**2 + Y**2 + Z**2) / 4) * np.exp(1j * X)).astype(np.complex128))
PY
for ra in 0 3; do
  for ns in 1 10; do
    echo "driver ra=$ra ns=$ns $(NLS_RUNAHEAD=$ra timeout -k 10 300 nonlinear-solvers_amd/bin/nlse_call_3d 384 384 384 10 10 10 /tmp/u0_384.npy /tmp/traj.npy 0.05 50 $ns --m=16)" >> gpurun_out/ra/all.log
  done
done
rm -f /tmp/traj.npy /tmp/u0_384.npy
