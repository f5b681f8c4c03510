"""The fused tail through the dynamic tile queue (Geo::tq, nls_stencil.hpp march) and
its tile depths, against the static tile grid on the SAME handle (nls_debug_knob).

The tail reduces nothing, so which workgroup takes which tile, and how deep the tiles
are, must not change a single bit of the trajectory.  Several steps per call also check
that the queue's counters return to zero after every launch (a launch that started
from a stale counter would skip tiles and leave garbage in the next start vector).
Covers the NLSE tail (G1 2D/3D, cubic-quintic), the G2 tail with m(x) and c(x), the
sEWI combination tails, and the SG / KG Gautschi tails.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
nls_amd = pytest.importorskip("nls_amd")

TAIL_DYN, KZ_FUSED = 1, 2
VARIANTS = [(0, 0), (1, 0), (1, 4), (1, 16), (0, 4)]  # (queue, tile depth; 0 = stencil depth)


def _field(n, seed=0, cplx=True):
    rng = np.random.default_rng(seed)
    x = np.linspace(-3, 3, n)
    base = np.exp(-x ** 2) + 0.1 * rng.standard_normal(n)
    return base * (1 + 0.3j) if cplx else base


def _variants(s, reset, run):
    out = []
    for dyn, kz in VARIANTS:
        s.debug_knob(TAIL_DYN, dyn)
        s.debug_knob(KZ_FUSED, kz)
        reset()
        out.append(run())
    return out


@pytest.mark.parametrize("dim,n,eq", [(3, 40, nls_amd.NLSE_CUBIC), (2, 96, nls_amd.NLSE_CUBIC),
                                      (3, 36, nls_amd.NLSE_CQ)])
def test_tail_queue_bitwise_nlse(dim, n, eq):
    cells = n ** dim
    u = _field(cells, 1)
    with nls_amd.Solver(dim, n, n, n if dim == 3 else 1, 0.2, 0.2, equation=eq, m=16) as s:
        def run():
            s.step(1e-3, 4)
            s.step(1e-3, 3)
            return s.get_field()
        res = _variants(s, lambda: s.set_field(u), run)
    assert all(np.isfinite(r).all() for r in res)
    for r in res[1:]:
        assert np.array_equal(res[0], r)


@pytest.mark.parametrize("sewi", [False, True])
def test_tail_queue_bitwise_g2(sewi):
    n = 30
    cells = n ** 3
    rng = np.random.default_rng(3)
    u = _field(cells, 2)
    mf = 1.0 + 0.5 * rng.random(cells)
    cf = 0.7 + 0.6 * rng.random(cells)
    with nls_amd.Solver(3, n, n, n, 0.25, 0.25, equation=nls_amd.NLSE_G2, m=20) as s:
        s.set_coefficients(mf, cf)

        def run():
            for i in range(4):
                if sewi:
                    s.step_sewi(1e-3, i + 1)
                else:
                    s.step(1e-3, 1)
                s.apply_bc()
            return s.get_field()
        res = _variants(s, lambda: s.set_field(u), run)
    for r in res[1:]:
        assert np.array_equal(res[0], r)


@pytest.mark.parametrize("eq,dim,n", [(nls_amd.SG_GAUTSCHI, 2, 96), (nls_amd.KG_GAUTSCHI, 3, 24)])
def test_tail_queue_bitwise_gautschi(eq, dim, n):
    cells = n ** dim
    u = _field(cells, 4, cplx=False)
    with nls_amd.Solver(dim, n, n, n if dim == 3 else 1, 0.2, 0.2, equation=eq, m=10) as s:
        if eq == nls_amd.KG_GAUTSCHI:
            rng = np.random.default_rng(5)
            s.set_coefficients(1.0 + 0.5 * rng.random(cells), 0.7 + 0.6 * rng.random(cells))

        def reset():
            if eq == nls_amd.KG_GAUTSCHI:
                s.set_sg_state(u, u.copy())
            else:
                s.set_sg_state(u, u.copy(), -np.ones(cells))

        def run():
            for _ in range(4):
                s.step(1e-3, 1)
                if eq == nls_amd.KG_GAUTSCHI:
                    s.apply_bc()
            return s.get_field()
        res = _variants(s, reset, run)
    for r in res[1:]:
        assert np.array_equal(res[0], r)
