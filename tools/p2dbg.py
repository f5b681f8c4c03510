"""Debug helper: one NLSE step through the two-vector pass (env selects the form)."""
import sys
import numpy as np
sys.path[:0] = ["nonlinear-solvers_amd"]
import nls_amd
nx, ny, nz, m = 64, 16, 12, 16
L = 10.0
dx = 2 * L / (nx - 1)
rng = np.random.default_rng(11)
x, y, z = np.linspace(-L, L, nx), np.linspace(-L, L, ny), np.linspace(-L, L, nz)
Z, Y, X = np.meshgrid(z, y, x, indexing="ij")
u0 = (np.exp(-(X ** 2 + Y ** 2 + Z ** 2) / 4) * np.exp(0.3j * X)).ravel()
u0 = u0 + 1e-3 * (rng.standard_normal(u0.size) + 1j * rng.standard_normal(u0.size))
with nls_amd.Solver(3, nx, ny, nz, dx, dx, m=m) as s:
    s.set_field(u0)
    s.step(1e-3, 1)
    s.sync()
