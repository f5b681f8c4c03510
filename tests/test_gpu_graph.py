"""hipGraph replay of steady-state steps (NLS_GRAPH=1) against eager launches.

A replayed step runs the same kernels with the same arguments as an eager one,
so every trajectory must agree bit for bit; the handle's timing counters show
that replay actually happened.  Covers re-capture on a dt change, a field reset
(the first step after it is eager: it starts with k_nl_init), the G2 driver loop
(step + apply_bc), the sEWI steps (never replayed) interleaved, and KG / SG.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
nls_amd = pytest.importorskip("nls_amd")


def _field(n, seed=0, cplx=True):
    rng = np.random.default_rng(seed)
    x = np.linspace(-3, 3, n)
    base = np.exp(-x ** 2) + 0.1 * rng.standard_normal(n)
    return base * (1 + 0.3j) if cplx else base


def _run(monkeypatch, graph, body):
    monkeypatch.setenv("NLS_GRAPH", "1" if graph else "0")
    return body()


def _nlse(dim, n, eq):
    def body():
        cells = n ** dim
        nz = n if dim == 3 else 1
        u = _field(cells, 1)
        with nls_amd.Solver(dim, n, n, nz, 0.2, 0.2, equation=eq, m=12) as s:
            s.set_field(u)
            s.step(1e-3, 5)
            s.step(2e-3, 3)          # dt change: eager step (W_0 rebuilt), then a new graph
            s.step(1e-3, 4)
            a = s.get_field()
            s.set_field(u[::-1].copy())
            s.step(1e-3, 3)
            b = s.get_field()
            return a, b, s.timing()["graph_steps"], s.timing()["steps"]
    return body


@pytest.mark.parametrize("dim,n,eq", [(2, 64, nls_amd.NLSE_CUBIC), (3, 20, nls_amd.NLSE_CUBIC),
                                      (2, 70, nls_amd.NLSE_CQ)])
def test_graph_replay_bitwise_nlse(monkeypatch, dim, n, eq):
    a0, b0, g0, s0 = _run(monkeypatch, False, _nlse(dim, n, eq))
    a1, b1, g1, s1 = _run(monkeypatch, True, _nlse(dim, n, eq))
    assert np.array_equal(a0, a1) and np.array_equal(b0, b1)
    assert g0 == 0 and s0 == s1 == 15
    assert g1 == 15 - 4   # eager: the first step, both dt changes, the step after set_field


@pytest.mark.parametrize("dim,n", [(3, 14), (3, 16), (2, 40)])
def test_graph_replay_bitwise_g2(monkeypatch, dim, n):
    """n = 16 (3D): the anisotropic s-step passes; the sEWI steps then move the P2State
    to make room for their second basis (sewi_concurrent), which drops the step graph
    captured before them -- the steps after re-capture it."""
    def body():
        cells = n ** dim
        nz = n if dim == 3 else 1
        rng = np.random.default_rng(2)
        u = _field(cells, 3)
        mf, c = rng.uniform(0.5, 1.5, cells), rng.uniform(0.5, 1.5, cells)
        with nls_amd.Solver(dim, n, n, nz, 0.3, 0.3, equation=nls_amd.NLSE_G2, m=10) as s:
            s.set_coefficients(mf, c)
            s.set_field(u)
            for _ in range(6):
                s.step(1e-3, 1)
                s.apply_bc()
            a = s.get_field()
            for i in range(1, 4):
                s.step_sewi(1e-3, i)
                s.apply_bc()
            s.step(1e-3, 2)
            b = s.get_field()
            return a, b, s.timing()["graph_steps"]
    a0, b0, g0 = _run(monkeypatch, False, body)
    a1, b1, g1 = _run(monkeypatch, True, body)
    assert np.array_equal(a0, a1) and np.array_equal(b0, b1)
    assert g0 == 0 and g1 >= 5


@pytest.mark.parametrize("eq,dim,n", [(nls_amd.KG_GAUTSCHI, 3, 14), (nls_amd.KG_GAUTSCHI, 3, 16),
                                      (nls_amd.KG_GAUTSCHI, 2, 40), (nls_amd.SG_GAUTSCHI, 2, 48)])
def test_graph_replay_bitwise_real(monkeypatch, eq, dim, n):
    """KG 3D n = 14 (ny % 4 != 0): the one-vector passes; n = 16: the s-step cell-pair
    passes (run_lanczos2 on both bases, the TAIL_COMBINE_W0 -> TAIL_KG_END1 tails), whose
    first step after set_* is eager.  KG 2D keeps the one-vector passes; SG 2D runs the
    s-step passes (eager again after its second set_sg_state)."""
    def body():
        cells = n ** dim
        nz = n if dim == 3 else 1
        rng = np.random.default_rng(4)
        u = _field(cells, 5, cplx=False)
        up = u - 1e-3 * np.sin(np.arange(cells))
        mf, c = rng.uniform(0.5, 1.5, cells), rng.uniform(0.5, 1.5, cells)
        with nls_amd.Solver(dim, n, n, nz, 0.3, 0.3, equation=eq, m=10) as s:
            if eq == nls_amd.KG_GAUTSCHI:
                s.set_coefficients(mf, c)
                s.set_sg_state(u, up)
                for _ in range(5):
                    s.step(1e-2, 1)
                    s.apply_bc()
                v = s.get_sg_velocity(1e-2)
            else:
                s.set_sg_state(u, up, -mf)
                s.step(1e-2, 5)
                v = s.get_sg_velocity(1e-2)
                first = s.get_field()
                # the same state again: bitwise the same trajectory (the s-step bases
                # start cold after every nls_set_*, eager, not from the warm graph)
                s.set_sg_state(u, up, -mf)
                s.step(1e-2, 5)
                assert np.array_equal(s.get_field(), first)
            return s.get_field(), v, s.timing()["graph_steps"]
    a0, v0, g0 = _run(monkeypatch, False, body)
    a1, v1, g1 = _run(monkeypatch, True, body)
    assert np.array_equal(a0, a1) and np.array_equal(v0, v1)
    # s-step passes: the first step after each set_sg_state is eager (cold bases) --
    # SG 2D (two set_sg_state calls: 10 - 2) and KG 3D with ny % 4 == 0 and nx even
    # (5 - 1); the one-vector passes replay every step
    s_step_kg = eq == nls_amd.KG_GAUTSCHI and dim == 3 and n % 4 == 0
    want = 8 if eq == nls_amd.SG_GAUTSCHI else (4 if s_step_kg else 5)
    assert g0 == 0 and g1 == want
