#!/bin/bash
# End-to-end driver runs with different snapshot counts (pipeline overlap of D2H + file writes)
set -e
mkdir -p gpurun_out/snap
python3 - <<'PY'
import numpy as np
n = 384
x = np.linspace(-10, 10, n)
Z, Y, X = np.meshgrid(x, x, x, indexing="ij")
u = np.exp(-(X**2 + Y**2 + Z**2) / 4) * np.exp(1j * X)
np.save("/tmp/u0_384.npy", u.astype(np.complex128))
PY
: > gpurun_out/snap/all.log
for ns in 1 10 1 10 25 49; do
  t0=$(date +%s.%N)
  NLS_DRIVER_TIMING=1 timeout -k 10 300 nonlinear-solvers_amd/bin/nlse_call_3d 384 384 384 10 10 10 /tmp/u0_384.npy /tmp/traj.npy 0.05 50 $ns --m=16 > /tmp/o.log 2>&1
  t1=$(date +%s.%N)
  echo "ns=$ns $(cat /tmp/o.log | tr "\n" " ") wall=$(python3 -c "print(round($t1-$t0,3))")" >> gpurun_out/snap/all.log
done
rm -f /tmp/traj.npy /tmp/u0_384.npy
