"""Diagnostic: per-iteration folded vs direct alpha (NLS_DEBUG_ALPHA=1 prints to stderr)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nonlinear-solvers_amd")]
os.environ["NLS_DEBUG_ALPHA"] = "1"
import nls_amd
rng = np.random.default_rng(11)
for (dim, nx, ny, nz, m) in [(3, 21, 19, 17, 16), (2, 64, 64, 1, 16), (3, 64, 8, 4, 12), (3, 16, 16, 16, 12)]:
    n = nx * ny * (nz if dim == 3 else 1)
    dx = 20.0 / (nx - 1)
    u0 = 0.3 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    print(f"=== {dim} {nx} {ny} {nz} m={m}", file=sys.stderr, flush=True)
    with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=0, m=m) as s:
        s.set_field(u0)
        s.step(1e-3, 1)
        s.sync()
