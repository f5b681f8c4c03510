"""Diagnostic: relative differences of the folded-alpha / fused-tail variants against
each other and the oracle (prints, no asserts).  GPU."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nonlinear-solvers_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import nls_amd, oracle_py as O
from conftest import rel_l2
from test_gpu_parity import soliton_field

def run(dim, nx, ny, nz, dx, u0, dt, steps, m, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=0, m=m) as s:
            s.set_field(u0)
            s.step(dt, steps)
            return s.get_field()
    finally:
        for k, v in old.items():
            if v is None: del os.environ[k]
            else: os.environ[k] = v

rng = np.random.default_rng(11)
for (dim, nx, ny, nz, m, kind) in [(3, 21, 19, 17, 10, "noise"), (3, 21, 19, 17, 16, "noise"), (3, 24, 24, 24, 16, "soliton"),
                                    (2, 70, 67, 1, 10, "noise"), (2, 64, 64, 1, 16, "soliton"), (3, 67, 35, 33, 16, "noise")]:
    n = nx * ny * (nz if dim == 3 else 1)
    dx = 20.0 / (nx - 1)
    if kind == "noise":
        u0 = 0.3 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    else:
        u0 = soliton_field(dim, nx, ny, nz, 10.0, seed=7)
        u0 = u0 / np.sqrt(np.sum(np.abs(u0) ** 2) * dx ** dim)
    steps, dt = 6, 1e-3
    ref = O.nlse_steps(O.grid(dim, nx, ny, nz, dx, dx), u0, dt, steps, m)
    res = {}
    for tag, env in [("t1a1", {"NLS_FUSED_TAIL": "1", "NLS_FUSED_ALPHA": "1"}), ("t0a1", {"NLS_FUSED_TAIL": "0", "NLS_FUSED_ALPHA": "1"}),
                     ("t1a0", {"NLS_FUSED_TAIL": "1", "NLS_FUSED_ALPHA": "0"}), ("t0a0", {"NLS_FUSED_TAIL": "0", "NLS_FUSED_ALPHA": "0"})]:
        res[tag] = run(dim, nx, ny, nz, dx, u0, dt, steps, m, env)
    print(dim, nx, ny, nz, m, kind, " ".join(f"{k}:oracle={rel_l2(v, ref):.2e}" for k, v in res.items()),
          f"t1a1-t0a0={rel_l2(res['t1a1'], res['t0a0']):.2e} t0a1-t0a0={rel_l2(res['t0a1'], res['t0a0']):.2e} t1a0-t0a0={rel_l2(res['t1a0'], res['t0a0']):.2e}", flush=True)
