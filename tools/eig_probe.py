import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "nonlinear-solvers_amd"))
import nls_amd
n, m = 64, int(sys.argv[1])
dx = 20.0 / (n - 1)
rng = np.random.default_rng(0)
N = n ** 3
u = (rng.standard_normal(N) + 1j * rng.standard_normal(N)) * 1e-3 + 1.0
with nls_amd.Solver(3, n, n, n, dx, dx, equation=nls_amd.NLSE_G2, m=m) as s:
    s.set_coefficients(1.0 + 0.5 * rng.random(N), 0.7 + 0.6 * rng.random(N))
    s.set_field(u)
    for _ in range(3):
        s.step(1e-3, 1)
    s.sync()
