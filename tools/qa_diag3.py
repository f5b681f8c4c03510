"""Diagnostic: folded vs direct alpha on smooth (noise-free) fields, where beta decays."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nonlinear-solvers_amd")]
os.environ["NLS_DEBUG_ALPHA"] = "1"
import nls_amd
for (dim, n, m, w) in [(3, 64, 16, 2.0), (3, 128, 16, 1.0), (2, 256, 16, 2.0), (2, 1024, 25, 1.0), (3, 32, 25, 3.0)]:
    L = 10.0
    x = np.linspace(-L, L, n)
    g = np.meshgrid(*([x] * dim), indexing="ij")
    r2 = sum(t ** 2 for t in g)
    u0 = (np.exp(-r2 / w ** 2) * np.exp(1j * g[-1])).ravel()
    dx = 2 * L / (n - 1)
    print(f"=== {dim} {n} m={m} width={w}", file=sys.stderr, flush=True)
    with nls_amd.Solver(dim, n, n, n if dim == 3 else 1, dx, dx, equation=0, m=m) as s:
        s.set_field(u0)
        s.step(1e-3, 1)
        s.sync()
