"""Per-rank cost of the scaling bench's slabs on one GPU: a 512 x 512 x nz grid
(nz = 512/N for N = 1, 2, 4, 8 ranks), single-rank and through the collective code
path on a 1-rank RCCL communicator (NLS_FORCE_RCCL=1: split boundary/interior
launches, all-reduce calls; no neighbour, so no halo bytes).  The N-rank step time
is about the collective row plus the real halo and all-reduce latency.
usage: python tools/slab_probe.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "nonlinear-solvers_amd"))
import nls_amd
n, nz, steps = 512, int(sys.argv[2]), 10
dx = 20.0 / (n - 1)
rng = np.random.default_rng(0)
u = (rng.standard_normal(n * n * nz) + 1j * rng.standard_normal(n * n * nz)) * 1e-3 + 1.0
with nls_amd.Solver(3, n, n, nz, dx, dx, m=16) as s:
    s.set_field(u)
    s.step(1e-3, 2)
    s.sync()
    t0 = time.perf_counter()
    s.step(1e-3, steps)
    s.sync()
    el = (time.perf_counter() - t0) / steps
    s.set_timing(True)
    s.step(1e-3, 3)
    s.sync()
    tm = s.timing()
    s.set_timing(False)
cls = {k: round(v / 3, 3) for k, v in tm["class_ms"].items() if v}
upd = {j: round(tm["update_ms"][j] / 3, 3) for j in range(16) if tm["update_count"][j]}
print(f"nz={nz:3d} rccl={os.environ.get('NLS_FORCE_RCCL', '0')} peer={os.environ.get('NLS_PEER', '0')} kz={os.environ.get('NLS_P2_KZ', 'auto')} {el * 1e3:8.3f} ms/step "
      f"{n * n * nz / el / 1e6:8.0f} Mcells*steps/s  per step {cls}  per step and J {upd}", flush=True)
"""

# (nz, extra environment): the tile depth follows the slab's own plane count (its
# interior on split collective handles), the same as an N-rank handle of 512^3
# computes it; NLS_P2_SPLIT=0 drops the boundary/interior split (the exchange would
# then follow each pass).  Two interleaved rounds: separate processes differ by a few
# per cent from the placement of their allocations.
# NLS_PEER=1: the peer-store passes (one launch per pass, the boundary planes stored by
# k_p2d<..., PEER> itself; on one rank into its own out-of-grid ghost planes, so the row
# carries the stores' cost but not the xGMI latency).
BASE = [
    (64, {}), (64, {"NLS_FORCE_RCCL": "1"}), (64, {"NLS_FORCE_RCCL": "1", "NLS_P2_SPLIT": "0"}),
    (64, {"NLS_FORCE_RCCL": "1", "NLS_PEER": "1"}),
    (128, {}), (128, {"NLS_FORCE_RCCL": "1"}), (128, {"NLS_FORCE_RCCL": "1", "NLS_PEER": "1"}),
]
VARIANTS = BASE + BASE
if len(sys.argv) > 1:  # a subset: python tools/slab_probe.py 0 2 3
    VARIANTS = [VARIANTS[int(i)] for i in sys.argv[1:]]
for nz, extra in VARIANTS:
    env = dict(os.environ, **extra)
    print(f"# {extra}", flush=True)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, str(nz)], env=env, timeout=300)
    if r.returncode:
        sys.exit(r.returncode)
