"""Print the eigensolver's iteration counts (library built with -DNLS_EIG_DEBUG)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nonlinear-solvers_amd"))
import nls_amd
for dim, n, m in [(2, 64, 16), (2, 64, 32), (3, 32, 16), (2, 64, 10)]:
    rng = np.random.default_rng(0)
    cells = n ** dim
    u = rng.standard_normal(cells) + 1j * rng.standard_normal(cells)
    with nls_amd.Solver(dim, n, n, n if dim == 3 else 1, 20.0 / (n - 1), m=m) as s:
        s.set_field(u)
        s.step(1e-3, 2)
        s.sync()
    print("----", dim, n, m, flush=True)
