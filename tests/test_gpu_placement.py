"""The basis placement probe (nls_placement; DESIGN.md section 4 "Placement").

Large single-rank handles allocate several candidate Krylov bases at nls_create, run the
same probe steps on each and keep the fastest.  Whatever was chosen, the handle must then
be in exactly the state a handle without the probe starts in, so every result is bitwise
the same as with NLS_PLACE=1 (one allocation, no probe).  NLS_LARGE_SLAB=1 gives small
grids the large-slab launch shapes, and with them the probe.
"""
import numpy as np
import pytest

from conftest import rel_l2

pytestmark = pytest.mark.gpu
nls_amd = pytest.importorskip("nls_amd")


def _field(n, seed=3):
    rng = np.random.default_rng(seed)
    x = np.linspace(-10, 10, n)
    g = np.exp(-(x[:, None, None] ** 2 + x[None, :, None] ** 2 + (x[None, None, :] - 1.0) ** 2) / 4.0)
    u = g * np.exp(0.7j * x[None, None, :]) + 1e-3 * (rng.standard_normal((n,) * 3)
                                                      + 1j * rng.standard_normal((n,) * 3))
    return u.ravel()


def _run(monkeypatch, place, n, m, steps, equation=nls_amd.NLSE_CUBIC):
    monkeypatch.setenv("NLS_LARGE_SLAB", "1")
    monkeypatch.setenv("NLS_PLACE", str(place))
    dx = 20.0 / (n - 1)
    u0 = _field(n)
    with nls_amd.Solver(3, n, n, n, dx, dx, equation=equation, m=m) as s:
        pl = s.placement()
        s.set_field(u0)
        s.step(1e-3, steps)
        a = s.get_field()
        s.step(1e-3, 1)          # a second call: blind start from the state the first left
        b = s.get_field()
        y = s.krylov_apply(u0, -1e-3j, nls_amd.F_EXP_ABS)
    return pl, a, b, y, u0


@pytest.mark.parametrize("n,m", [(48, 16), (40, 10)])
def test_placement_probe_changes_no_bit(monkeypatch, n, m):
    pl1, a1, b1, y1, u0 = _run(monkeypatch, 1, n, m, 3)
    pl4, a4, b4, y4, _ = _run(monkeypatch, 4, n, m, 3)
    assert pl1["candidates"] == 0 and pl1["chosen"] == -1
    assert 2 <= pl4["candidates"] <= 4, pl4
    assert 0 <= pl4["chosen"] < pl4["candidates"]
    assert all(t > 0 for t in pl4["probe_ms"])
    assert pl4["probe_ms"][pl4["chosen"]] == min(pl4["probe_ms"])
    assert np.array_equal(a1, a4)
    assert np.array_equal(b1, b4)
    assert np.array_equal(y1, y4)
    assert rel_l2(a1, u0) > 1e-6


def test_placement_cubic_quintic(monkeypatch):
    pl1, a1, b1, _, _ = _run(monkeypatch, 1, 32, 12, 2, nls_amd.NLSE_CQ)
    pl3, a3, b3, _, _ = _run(monkeypatch, 3, 32, 12, 2, nls_amd.NLSE_CQ)
    assert pl3["candidates"] == 3
    assert np.array_equal(a1, a3) and np.array_equal(b1, b3)


def test_no_probe_off_the_large_slab_class(monkeypatch):
    """Small 3D slabs, 2D grids and the real Gautschi handles keep their one allocation."""
    monkeypatch.delenv("NLS_LARGE_SLAB", raising=False)
    monkeypatch.setenv("NLS_PLACE", "4")
    with nls_amd.Solver(3, 32, 32, 32, 0.5, 0.5, m=10) as s:
        assert s.placement()["candidates"] == 0
    with nls_amd.Solver(2, 256, 256, 1, 0.1, 0.1, m=10) as s:
        assert s.placement()["candidates"] == 0
    monkeypatch.setenv("NLS_LARGE_SLAB", "1")
    with nls_amd.Solver(3, 32, 32, 32, 0.5, 0.5, equation=nls_amd.SG_GAUTSCHI, m=10) as s:
        assert s.placement()["candidates"] == 0


def test_placement_full_size_512_bitwise(monkeypatch):
    """The bench's own case: 512^3 m = 16 (large class, up to 8 candidates probed) against
    one allocation, two steps of one call, bit for bit."""
    n, m = 512, 16
    dx = 20.0 / (n - 1)
    x = np.linspace(-10, 10, n)
    g = np.exp(-(x ** 2) / 8.0)
    u0 = ((g[:, None, None] * g[None, :, None]) * (g * np.exp(0.5j * x))[None, None, :]).ravel()
    out = []
    for place in ("1", "8"):
        monkeypatch.setenv("NLS_PLACE", place)
        with nls_amd.Solver(3, n, n, n, dx, dx, m=m) as s:
            pl = s.placement()
            s.set_field(u0)
            s.step(1e-3, 2)
            out.append(s.get_field())
        if place == "1":
            assert pl["candidates"] == 0
        else:
            assert pl["candidates"] >= 2 and pl["probe_ms"][pl["chosen"]] == min(pl["probe_ms"])
    assert np.array_equal(out[0], out[1])
    assert rel_l2(out[0], u0) > 1e-8
