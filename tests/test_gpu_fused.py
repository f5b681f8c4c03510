"""GPU checks of the fused tail of the NLSE step (k_alpha_l2 + k_final_fused).

With the fused tail the last Lanczos vector W_{m-1} is never stored: its norm
comes from ||L v_{m-2}||^2 - sum_k |H[m-2][k]|^2 and the vector itself is
recomputed inside the final pass (nls_stencil.hpp k_final_fused).  The step it
replaces is k_update<m-2> + k_final_nlse<m> (NLS_FUSED_TAIL=0, read at handle
creation).  Both must agree to rounding level and both must match the oracle
(eigen_krylov_complex.hpp:10-84, nlse_solver.hpp:53-77) within the north_star
tolerance; the fused kernel must actually run (timing class "final").
"""
import os

import numpy as np
import pytest

import oracle_py as O
from conftest import rel_l2

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _one_vector_path(monkeypatch):
    """These tests compare variants of the one-vector Lanczos passes (fused tail on /
    off, folded alpha on / off); the 3D NLSE runs the two-vector passes by default."""
    monkeypatch.setenv("NLS_PASS2", "0")
nls_amd = pytest.importorskip("nls_amd")


def _field(n, seed):
    rng = np.random.default_rng(seed)
    return rng.standard_normal(n) + 1j * rng.standard_normal(n)


def _run(dim, nx, ny, nz, dx, u0, dt, steps, m, eq, fused, mf=None, cf=None):
    old = os.environ.get("NLS_FUSED_TAIL")
    os.environ["NLS_FUSED_TAIL"] = "1" if fused else "0"
    try:
        with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=eq, m=m) as s:
            if mf is not None:
                s.set_coefficients(mf, cf)
            s.set_field(u0)
            s.set_timing(True)
            for _ in range(steps):
                s.step(dt, 1)
                if mf is not None:
                    s.apply_bc()
            out = s.get_field()
            tm = s.timing()
    finally:
        if old is None:
            del os.environ["NLS_FUSED_TAIL"]
        else:
            os.environ["NLS_FUSED_TAIL"] = old
    return out, tm


@pytest.mark.parametrize("dim,nx,ny,nz", [(3, 21, 19, 17), (2, 70, 67, 1)])
@pytest.mark.parametrize("m", [3, 4, 10, 16, 25])
@pytest.mark.parametrize("eq", [nls_amd.NLSE_CUBIC, nls_amd.NLSE_CQ])
def test_fused_tail_matches_unfused_and_oracle(dim, nx, ny, nz, m, eq):
    n = nx * ny * (nz if dim == 3 else 1)
    dx, dt, steps = 20.0 / (nx - 1), 1e-3, 6
    u0 = 0.3 * _field(n, 11 + m)
    a, ta = _run(dim, nx, ny, nz, dx, u0, dt, steps, m, eq, True)
    b, tb = _run(dim, nx, ny, nz, dx, u0, dt, steps, m, eq, False)
    assert ta["class_count"]["final"] == steps and tb["class_count"]["final"] == 0
    assert rel_l2(a, b) <= 1e-12
    g = O.grid(dim, nx, ny, nz, dx, dx)
    ref = O.nlse_steps(g, u0, dt, steps, m, nonlin=eq)
    assert rel_l2(a, ref) <= 1e-10


@pytest.mark.parametrize("dim,nx,ny,nz", [(3, 18, 16, 15), (2, 50, 47, 1)])
def test_fused_tail_g2_with_bc(dim, nx, ny, nz):
    n = nx * ny * (nz if dim == 3 else 1)
    rng = np.random.default_rng(5)
    dx, dt, steps, m = 0.25, 1e-3, 5, 25 if dim == 3 else 20
    c = rng.uniform(0.6, 1.4, n)
    mf = rng.uniform(0.5, 1.5, n)
    u0 = 0.5 * _field(n, 7)
    a, ta = _run(dim, nx, ny, nz, dx, u0, dt, steps, m, nls_amd.NLSE_G2, True, mf, c)
    b, _ = _run(dim, nx, ny, nz, dx, u0, dt, steps, m, nls_amd.NLSE_G2, False, mf, c)
    assert ta["class_count"]["final"] == steps
    assert rel_l2(a, b) <= 1e-12
    ref = O.nlse_g2_steps(O.grid(dim, nx, ny, nz, dx, dx), c, mf, u0, dt, steps, m, bc=True)
    assert rel_l2(a, ref) <= 1e-10


def test_fused_tail_large_phase():
    """|dt |u|^2 / 2| well beyond pi/4 exercises the quadrant reduction of nl_sincos."""
    nx = ny = 40
    dx = 0.5
    u0 = 30.0 * _field(nx * ny, 3)  # phases up to ~dt * 1e3
    dt = 5e-3
    a, _ = _run(2, nx, ny, 1, dx, u0, dt, 3, 10, nls_amd.NLSE_CUBIC, True)
    ref = O.nlse_steps(O.grid(2, nx, ny, 1, dx, dx), u0, dt, 3, 10)
    assert rel_l2(a, ref) <= 1e-10


# ---- folded alpha (march_q): update pass j also reduces q = (L W_j)^H L (L W_j) and
# the alpha pass of W_{j+1} is skipped (NLS_FUSED_ALPHA, read at handle creation)

def _run_env(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


# shapes with partial x/y/z tiles, two x-tiles (lane-63 gathers), the 3D y-wrap
# across tiles and more planes than one tile depth (peek planes)
SHAPES_QA = [(3, 67, 35, 33), (3, 20, 9, 70), (2, 200, 131, 1), (2, 130, 40, 1)]


@pytest.mark.parametrize("dim,nx,ny,nz", SHAPES_QA)
@pytest.mark.parametrize("eq", ["cubic", "cq", "g2", "sewi", "sg", "kg"])
def test_folded_alpha_matches_alpha_pass(dim, nx, ny, nz, eq):
    n = nx * ny * (nz if dim == 3 else 1)
    rng = np.random.default_rng(17)
    dx = 20.0 / (nx - 1)
    m = {"cubic": 16, "cq": 14, "g2": 12, "sewi": 12, "sg": 10, "kg": 10}[eq]
    steps = 4
    c = rng.uniform(0.6, 1.4, n)
    mf = rng.uniform(0.5, 1.5, n)

    def run():
        if eq in ("cubic", "cq", "g2", "sewi"):
            code = {"cubic": nls_amd.NLSE_CUBIC, "cq": nls_amd.NLSE_CQ}.get(eq, nls_amd.NLSE_G2)
            u0 = 0.3 * _field(n, 5)
            with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=code, m=m) as s:
                if eq in ("g2", "sewi"):
                    s.set_coefficients(mf, c)
                s.set_field(u0)
                s.set_timing(True)
                for i in range(1, steps + 1):
                    if eq == "sewi":
                        s.step_sewi(1e-3, i)
                    else:
                        s.step(1e-3, 1)
                    if eq in ("g2", "sewi"):
                        s.apply_bc()
                return s.get_field(), s.timing()
        u0 = rng.standard_normal(n) * 0.5
        code = nls_amd.SG_GAUTSCHI if eq == "sg" else nls_amd.KG_GAUTSCHI
        with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=code, m=m) as s:
            if eq == "kg":
                s.set_coefficients(mf, c)
                s.set_sg_state(u0, u0.copy())
            else:
                s.set_sg_state(u0, u0.copy(), -np.ones(n))
            s.set_timing(True)
            for _ in range(steps):
                s.step(1e-2, 1)
                if eq == "kg":
                    s.apply_bc()
            return s.get_field(), s.timing()

    rng_state = rng.bit_generator.state
    a, ta = _run_env({"NLS_FUSED_ALPHA": "1"}, run)
    rng.bit_generator.state = rng_state
    b, tb = _run_env({"NLS_FUSED_ALPHA": "0"}, run)
    assert ta["class_count"]["alpha"] < tb["class_count"]["alpha"]
    assert np.all(np.isfinite(a))
    assert rel_l2(a, b) <= 1e-12


@pytest.mark.parametrize("dim,nx,ny,nz", SHAPES_QA)
def test_folded_alpha_nlse_matches_oracle(dim, nx, ny, nz):
    n = nx * ny * (nz if dim == 3 else 1)
    dx, dt, steps, m = 20.0 / (nx - 1), 1e-3, 5, 16
    u0 = 0.3 * _field(n, 23)
    a, ta = _run_env({"NLS_FUSED_ALPHA": "1"},
                     lambda: _run(dim, nx, ny, nz, dx, u0, dt, steps, m, nls_amd.NLSE_CUBIC, True))
    ref = O.nlse_steps(O.grid(dim, nx, ny, nz, dx, dx), u0, dt, steps, m)
    assert rel_l2(a, ref) <= 1e-10


@pytest.mark.parametrize("dim,nx,ny,nz", [(2, 70, 67, 1), (3, 21, 19, 17)])
def test_multi_step_call_equals_single_steps(dim, nx, ny, nz):
    """One-vector path: the fused tail's u store only on a call's last step changes no
    bit of the trajectory (5-step call vs 1-step calls)."""
    dx = 0.4
    u0 = _field(nx * ny * nz, 4)
    out = []
    for calls in ((5,), (1, 1, 1, 1, 1)):
        with nls_amd.Solver(dim, nx, ny, nz, dx, dx, m=12) as s:
            s.set_field(u0)
            for k in calls:
                s.step(1e-3, k)
            out.append(s.get_field())
    assert np.array_equal(out[0], out[1])
