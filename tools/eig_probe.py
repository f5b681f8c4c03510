"""Eigensolve timing probe: a few steps of small G2 (m = 25) and NLSE (m = 16) handles on
a library built with -DNLS_EIG_DEBUG (k_reduce_final prints its phases per launch).
  NLS_AMD_LIB=nonlinear-solvers_amd/lib_veig/libnls_amd.so python tools/eig_probe.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nonlinear-solvers_amd"))
sys.path.insert(0, ROOT)
import nls_amd  # noqa: E402
from bench import g2_coefficients  # noqa: E402


def run(eq, m, n=32, steps=3):
    L = 10.0
    dx = 2 * L / (n - 1)
    rng = np.random.default_rng(1)
    u = (np.exp(-np.linspace(-3, 3, n) ** 2)[:, None, None] * np.ones((n, n, n))
         + 1e-3 * rng.standard_normal((n, n, n))).astype(np.complex128).ravel()
    with nls_amd.Solver(3, n, n, n, dx, dx, equation=eq, m=m) as s:
        s.set_field(u)
        if eq == nls_amd.NLSE_G2:
            s.set_coefficients(*g2_coefficients(n, L, 0, n))
        for _ in range(steps):
            s.step(1e-3)
            s.sync()
    sys.stdout.flush()


if __name__ == "__main__":
    print(f"# {nls_amd.lib_path()}", flush=True)
    print("## G2 m=25", flush=True)
    run(nls_amd.NLSE_G2, 25)
    print("## NLSE m=16", flush=True)
    run(nls_amd.NLSE_CUBIC, 16)
