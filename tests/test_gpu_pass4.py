"""GPU parity of the four-vector first pass (k_p4d0, nls_pass4.hip; NLS_P4): 3D isotropic
NLSE trajectories against the CPU oracle with the same tolerances as
tests/test_gpu_pass2.py, one step against the two-vector schedule, and the launch
record (a pass at J = 0 and J = 4, none at J = 2).  The pass takes single-rank 3D
complex grids with nx % 64 == 0, ny % 4 == 0, ny >= 8 and m >= 6 (nls_api.cpp); the
numerics of the schedule: tests/test_sstep_model.py::test_four_vector_first_pass_matches_oracle."""
import numpy as np
import pytest

import oracle_py as O
from conftest import rel_l2
from test_gpu_parity import soliton_field, spacing

pytestmark = pytest.mark.gpu

nls_amd = pytest.importorskip("nls_amd")

TOL_TRAJ = 1e-10


def _ran_p4(s, m=16):
    """A pass at J = 0, none at J = 2 (and the next at J = 4 where m > 6)."""
    cnt = s.timing()["update_count"]
    return cnt[0] > 0 and cnt[2] == 0 and (m == 6 or cnt[4] > 0)


@pytest.mark.parametrize("nx,ny,nz,m,kz", [(64, 16, 12, 16, "8"), (64, 8, 9, 6, "4"), (128, 16, 10, 10, "64"),
                                           (64, 32, 20, 16, "5"), (64, 12, 7, 18, "64"), (192, 8, 6, 7, "3")])
@pytest.mark.parametrize("eq", [0, 1])
def test_p4_trajectory_matches_oracle(monkeypatch, nx, ny, nz, m, kz, eq):
    monkeypatch.setenv("NLS_P4", "1")
    monkeypatch.setenv("NLS_P4_KZ", kz)
    L = 10.0
    dx = spacing(nx, L)
    u0 = soliton_field(3, nx, ny, nz, L, seed=13)
    u0 = u0 / np.sqrt(np.sum(np.abs(u0) ** 2) * dx ** 3)
    g = O.grid(3, nx, ny, nz, dx, dx)
    dt, nsteps = 1e-3, 10
    ref = O.nlse_steps(g, u0, dt, nsteps, m, nonlin=eq)
    with nls_amd.Solver(3, nx, ny, nz, dx, dx, equation=eq, m=m) as s:
        s.set_field(u0)
        s.set_timing(True)
        s.step(dt, nsteps - 3)
        s.step(dt, 3)
        u = s.get_field()
        assert _ran_p4(s, m)
    assert np.all(np.isfinite(u))
    assert rel_l2(u, ref) <= TOL_TRAJ


@pytest.mark.parametrize("L,large", [(10.0, "0"), (0.6, "0"), (10.0, "1")])  # ||L|| ~ 1e2 and ~ 3e4
def test_p4_one_step_matches_two_vector_schedule(monkeypatch, L, large):
    nx, ny, nz, m = 64, 32, 16, 16
    dx = spacing(nx, L)
    u0 = soliton_field(3, nx, ny, nz, L, seed=5)
    monkeypatch.setenv("NLS_LARGE_SLAB", large)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("NLS_P4", mode)
        with nls_amd.Solver(3, nx, ny, nz, dx, dx, m=m) as s:
            s.set_field(u0)
            s.set_timing(True)
            s.step(1e-3, 1)
            out[mode] = s.get_field()
            assert _ran_p4(s) == (mode == "1")
    assert rel_l2(out["1"], out["0"]) <= 1e-12


def test_p4_not_taken_where_it_does_not_apply(monkeypatch):
    """ny < 8, nx % 64 != 0 and m < 6 keep the two-vector schedule."""
    monkeypatch.setenv("NLS_P4", "1")
    for nx, ny, nz, m in ((64, 4, 8, 16), (48, 16, 8, 16), (64, 16, 8, 5)):
        dx = spacing(nx, 10.0)
        with nls_amd.Solver(3, nx, ny, nz, dx, dx, m=m) as s:
            s.set_field(soliton_field(3, nx, ny, nz, 10.0, seed=1))
            s.set_timing(True)
            s.step(1e-3, 1)
            assert not _ran_p4(s, m)
