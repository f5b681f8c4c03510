"""GPU: z-slab (3D) / y-slab (2D) decomposition.  Ranks are handles of one
process driven by host threads (nls_group local transport): same kernels,
ghost-plane layout, halo planes (incl. the 3D y-wrap across slab boundaries)
and reduction decomposition as the RCCL path; only the byte mover differs.
The assembled field must match the single-rank oracle run."""
import threading

import numpy as np
import pytest

import oracle_py as O
from conftest import rel_l2

pytestmark = pytest.mark.gpu
nls_amd = pytest.importorskip("nls_amd")


def run_ranks(nranks, make_solver, body):
    grp = nls_amd.Group(nranks)
    out = [None] * nranks
    err = []

    def work(r):
        try:
            s = make_solver(r, grp)
            out[r] = body(s)
            s.close()
        except Exception as e:  # noqa: BLE001
            err.append((r, e))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    [t.start() for t in ts]
    [t.join(timeout=300) for t in ts]
    grp.close()
    assert not err, err
    return out


def field(n_cells, seed=0):
    rng = np.random.default_rng(seed)
    x = np.linspace(-3, 3, n_cells)
    return np.exp(-x * x) * np.exp(1j * x) + 1e-2 * (rng.standard_normal(n_cells) + 1j * rng.standard_normal(n_cells))


@pytest.mark.parametrize("dim,n,nranks,eq", [(3, 16, 2, 0), (3, 16, 3, 0), (3, 13, 4, 0), (3, 12, 2, 1),
                                             (2, 40, 3, 0), (2, 33, 4, 1)])
def test_nlse_slabs_match_single_rank(dim, n, nranks, eq):
    L, m, dt, steps = 10.0, 12, 1e-3, 5
    dx = 2 * L / (n - 1)
    N = n ** dim
    P = n * n if dim == 3 else n
    u0 = field(N, seed=n)
    ref = O.nlse_steps(O.grid(dim, n, n, n, dx, dx), u0, dt, steps, m, nonlin=eq)

    def mk(r, grp):
        return nls_amd.Solver(dim, n, n, n, dx, dx, equation=eq, m=m, device=0, nranks=nranks, rank=r, group=grp)

    def body(s):
        s.set_field(u0[s.z0 * P:(s.z0 + s.nzl) * P])
        s.step(dt, steps)
        return s.z0, s.get_field()

    res = sorted(run_ranks(nranks, mk, body), key=lambda t: t[0])
    got = np.concatenate([r[1] for r in res])
    assert got.size == N
    assert rel_l2(got, ref) <= 1e-10


@pytest.mark.parametrize("nranks", [2, 3])
def test_laplacian_and_krylov_slabs(nranks):
    n, L = 14, 5.0
    dx = 2 * L / (n - 1)
    N, P = n ** 3, n * n
    u = field(N, 3)
    g = O.grid(3, n, n, n, dx, dx)
    lap_ref = O.laplacian_c(g, u)
    kry_ref = O.krylov_c(g, u, -1e-2j, 16, 0)

    def mk(r, grp):
        return nls_amd.Solver(3, n, n, n, dx, dx, m=16, device=0, nranks=nranks, rank=r, group=grp)

    def body(s):
        sl = u[s.z0 * P:(s.z0 + s.nzl) * P]
        return s.z0, s.laplacian(sl), s.krylov_apply(sl, -1e-2j, nls_amd.F_EXP_ABS)

    res = sorted(run_ranks(nranks, mk, body), key=lambda t: t[0])
    assert rel_l2(np.concatenate([r[1] for r in res]), lap_ref) <= 1e-14
    assert rel_l2(np.concatenate([r[2] for r in res]), kry_ref) <= 1e-12


def test_sg_slabs_match_single_rank():
    n, L, nranks = 36, 3.0, 3
    dx = 2 * L / (n - 1)
    x = np.linspace(-L, L, n)
    Y, X = np.meshgrid(x, x, indexing="ij")
    u0 = (2.0 * np.arctan(np.exp(3.0 - 5.0 * np.sqrt(X * X + Y * Y)))).ravel()
    mf = -np.ones(n * n)
    dt = 0.01
    ref_u, _ = O.sg_steps(O.grid(2, n, n, 1, dx, dx), u0, u0, mf, dt, 6, 10)

    def mk(r, grp):
        return nls_amd.Solver(2, n, n, 1, dx, dx, equation=nls_amd.SG_GAUTSCHI, m=10, device=0,
                              nranks=nranks, rank=r, group=grp)

    def body(s):
        sl = slice(s.z0 * n, (s.z0 + s.nzl) * n)
        s.set_sg_state(u0[sl], u0[sl], mf[sl])
        s.step(dt, 6)
        return s.z0, s.get_field()

    res = sorted(run_ranks(nranks, mk, body), key=lambda t: t[0])
    assert rel_l2(np.concatenate([r[1] for r in res]), ref_u) <= 1e-10


@pytest.mark.parametrize("eq", [0, 2])
def test_rccl_collective_path_single_rank(monkeypatch, eq):
    """NLS_FORCE_RCCL=1 routes a 1-rank handle through the collective code path
    with a real RCCL communicator (split reductions + ncclAllReduce + grouped
    send/recv halo calls), the path the multi-GPU bench takes."""
    monkeypatch.setenv("NLS_FORCE_RCCL", "1")
    n, L = 14, 5.0
    dx = 2 * L / (n - 1)
    if eq == 0:
        u0 = field(n ** 3, 5)
        ref = O.nlse_steps(O.grid(3, n, n, n, dx, dx), u0, 1e-3, 4, 10)
        with nls_amd.Solver(3, n, n, n, dx, dx, m=10, device=0) as s:
            s.set_field(u0)
            s.step(1e-3, 4)
            got = s.get_field()
    else:
        u0 = np.real(field(n * n, 6))
        mf = -np.ones(n * n)
        ref, _ = O.sg_steps(O.grid(2, n, n, 1, dx, dx), u0, u0, mf, 0.01, 4, 8)
        with nls_amd.Solver(2, n, n, 1, dx, dx, equation=nls_amd.SG_GAUTSCHI, m=8, device=0) as s:
            s.set_sg_state(u0, u0, mf)
            s.step(0.01, 4)
            got = s.get_field()
    assert rel_l2(got, ref) <= 1e-10


def _ran_pass2(s, m):
    cnt = s.timing()["update_count"]
    return cnt[0] > 0 and cnt[1] == 0  # s-step passes start at J = 0, 2, (5,) ... never at 1


@pytest.mark.parametrize("split", ["1", "0", "peer"], ids=["split", "unsplit", "peer"])
@pytest.mark.parametrize("nranks,m", [(4, 16), (3, 15), (2, 10)])
def test_pass2_slabs_match_oracle(monkeypatch, nranks, m, split):
    """The two-vector passes (k_p2d, the default for the 3D NLSE) on z slabs: two
    ghost planes per stored vector, two-plane halos of every stencil vector (incl.
    the 3D y-wrap across slab boundaries at the radius-2 march), all-reduced pass
    sums; uneven slabs (40 planes over 3 ranks) and an odd m (X-only last pass).
    Spacing of the 512^3 bench (dx = 20/511): the stiff regime.  split: the slabs'
    boundary planes as their own k_p2d launch ahead of the interior (the default,
    slabs of >= 8 planes) or one launch per pass (NLS_P2_SPLIT=0); peer: NLS_PEER=1,
    each pass stores its next stencil vector's boundary planes straight into the
    neighbours' ghost planes (k_p2d<..., PEER>: no exchange step, no split)."""
    if split == "peer":
        monkeypatch.setenv("NLS_PEER", "1")
    else:
        monkeypatch.setenv("NLS_P2_SPLIT", split)
    nx, ny, nz = 64, 24, 40
    dx = 20.0 / 511
    P = nx * ny
    u0 = field(nx * ny * nz, seed=nranks)
    dt, steps = 1e-3, 5
    ref = O.nlse_steps(O.grid(3, nx, ny, nz, dx, dx), u0, dt, steps, m)

    def mk(r, grp):
        return nls_amd.Solver(3, nx, ny, nz, dx, dx, m=m, device=0, nranks=nranks, rank=r, group=grp)

    def body(s):
        s.set_field(u0[s.z0 * P:(s.z0 + s.nzl) * P])
        s.set_timing(True)
        s.step(dt, steps)
        return s.z0, s.get_field(), _ran_pass2(s, m)

    res = sorted(run_ranks(nranks, mk, body), key=lambda t: t[0])
    assert all(r[2] for r in res)
    got = np.concatenate([r[1] for r in res])
    assert rel_l2(got, ref) <= 1e-10
    with nls_amd.Solver(3, nx, ny, nz, dx, dx, m=m, device=0) as s:
        s.set_field(u0)
        s.step(dt, steps)
        one = s.get_field()
    assert rel_l2(got, one) <= 1e-12


def test_pass2_rccl_collective_path_single_rank(monkeypatch):
    """NLS_FORCE_RCCL=1: the two-vector passes through a real RCCL communicator
    (ncclAllReduce of the pass sums, grouped two-plane send/recv)."""
    monkeypatch.setenv("NLS_FORCE_RCCL", "1")
    n, m = 16, 10
    dx = 20.0 / (n - 1)
    u0 = field(n ** 3, 8)
    ref = O.nlse_steps(O.grid(3, n, n, n, dx, dx), u0, 1e-3, 4, m)
    with nls_amd.Solver(3, n, n, n, dx, dx, m=m, device=0) as s:
        s.set_field(u0)
        s.set_timing(True)
        s.step(1e-3, 4)
        got = s.get_field()
        assert _ran_pass2(s, m)
        assert s.comm_size() == (1, "rccl")  # ncclCommCount of the forced communicator
    assert rel_l2(got, ref) <= 1e-10


@pytest.mark.parametrize("nranks,nz,m", [(2, 24, 12), (4, 40, 12), (2, 24, 3), (2, 24, 4), (3, 24, 4)])
def test_peer_slabs_bitwise_equal_exchange(monkeypatch, nranks, nz, m):
    """The peer-store path moves the same bytes as the exchange: the unsplit two-vector
    passes (one k_p2d launch per pass, the send/recv after it) and NLS_PEER=1 (the same
    launch shape; k_p2d<..., PEER> stores the boundary planes into the neighbours' ghost
    planes itself) give bit-identical fields.  m = 3, 4: the blind J = 0 pass that opens
    each step writes the neighbours' ghost planes of S_{m-2}, which their previous tail
    read -- ordered by the per-step W_0 halo; several steps over two calls."""
    nx, ny = 64, 16
    dx = 20.0 / 511
    P = nx * ny
    u0 = field(nx * ny * nz, seed=11)

    def run(env):
        for k in ("NLS_PEER", "NLS_P2_SPLIT"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)

        def mk(r, grp):
            return nls_amd.Solver(3, nx, ny, nz, dx, dx, m=m, device=0, nranks=nranks, rank=r, group=grp)

        def body(s):
            s.set_field(u0[s.z0 * P:(s.z0 + s.nzl) * P])
            s.step(1e-3, 4)
            s.step(1e-3, 2)
            assert s.peer_state() == ("active" if env.get("NLS_PEER") == "1" else "off")
            return s.z0, s.get_field()
        res = sorted(run_ranks(nranks, mk, body), key=lambda t: t[0])
        return np.concatenate([r[1] for r in res])
    a = run({"NLS_P2_SPLIT": "0"})
    b = run({"NLS_PEER": "1"})
    assert np.array_equal(a, b)


def test_peer_loopback_single_rank_unchanged(monkeypatch):
    """NLS_PEER=1 on a 1-rank handle (the slab probe's cost measurement): the peer
    stores land in the slab's own out-of-grid ghost planes, which nothing reads --
    bit-identical to the plain handle."""
    n, m = 24, 16
    dx = 20.0 / 511
    u0 = field(n ** 3, 12)
    out = []
    for peer in ("0", "1"):
        monkeypatch.setenv("NLS_PEER", peer)
        with nls_amd.Solver(3, n, n, n, dx, dx, m=m, device=0) as s:
            s.set_field(u0)
            s.step(1e-3, 3)
            out.append(s.get_field())
    assert np.array_equal(out[0], out[1])
