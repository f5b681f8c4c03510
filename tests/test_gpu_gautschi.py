"""GPU parity of the G2 device Gautschi family through the C-ABI:
NLS_SG_G2 / NLS_SG_DOUBLE / NLS_SG_HYPERBOLIC / NLS_PHI4 against the oracle
(oracle_gautschi_g2_steps, a restatement of nlsolvers/device/include/
{sg_single,sg_double,sg_hyperbolic,phi4_single}.cuh + the drivers' apply_bc),
the golden fixture, the unfused kernels (NLS_FUSED_TAIL=0), the folded alpha,
z/y slabs of the in-process rank group, and the drop-in drivers
{sg_single,sg_double,sg_hyperbolic,phi4}_dev end to end.
Tolerance: 1e-10 relative L2 on the field (north_star)."""
import os
import subprocess
import threading

import numpy as np
import pytest

import oracle_py as O
from conftest import rel_l2

pytestmark = pytest.mark.gpu
nls_amd = pytest.importorskip("nls_amd")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "nonlinear-solvers_amd", "bin")
GOLD = os.path.join(ROOT, "tests", "golden")
EQ = {"sg": nls_amd.SG_G2, "sg_double": nls_amd.SG_DOUBLE, "sg_hyperbolic": nls_amd.SG_HYPERBOLIC,
      "phi4": nls_amd.PHI4}
PROG = {"sg": "sg_single_dev", "sg_double": "sg_double_dev", "sg_hyperbolic": "sg_hyperbolic_dev",
        "phi4": "phi4_dev"}


def _env(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _ic(dim, n, L, seed):
    rng = np.random.default_rng(seed)
    x = np.linspace(-L, L, n)
    if dim == 2:
        Y, X = np.meshgrid(x, x, indexing="ij")
        R2 = X ** 2 + Y ** 2
    else:
        Z, Y, X = np.meshgrid(x, x, x, indexing="ij")
        R2 = X ** 2 + Y ** 2 + Z ** 2
    u0 = (1.2 * np.exp(-R2 / 2) + 1e-3 * rng.standard_normal(R2.shape)).ravel()
    v0 = (0.2 * np.sin(X) * np.exp(-R2 / 4)).ravel()
    mf = (1.0 + 0.2 * np.cos(X + Y)).ravel()
    return u0, v0, mf


def _gpu(dim, nx, ny, nz, dx, eq, u0, up, mf, dt, steps, m, bc=True):
    with nls_amd.Solver(dim, nx, ny, nz, dx, dx, equation=eq, m=m) as s:
        s.set_sg_state(u0, up, mf)
        s.set_timing(True)
        for _ in range(steps):
            s.step(dt, 1)
            if bc:
                s.apply_bc()
        return s.get_field(), s.timing()


@pytest.mark.parametrize("kname", sorted(EQ))
@pytest.mark.parametrize("dim,n", [(2, 40), (3, 18)])
@pytest.mark.parametrize("fused", [True, False])
def test_gautschi_g2_matches_oracle(kname, dim, n, fused):
    L, m, dt, steps = 4.0, 10, 1e-2, 8
    dx = 2 * L / (n - 1)
    u0, v0, mf = _ic(dim, n, L, 5 + dim)
    up = u0 - dt * v0
    # unfused: the one-vector passes (the two-vector ones always end in the fused tail)
    a, tm = _env({"NLS_FUSED_TAIL": "1" if fused else "0", "NLS_PASS2": "1" if fused else "0"},
                 lambda: _gpu(dim, n, n, n, dx, EQ[kname], u0, up, mf, dt, steps, m))
    assert (tm["class_count"]["final"] > 0) == fused  # the fused tail k_tail<GG_MID> ran
    ref, _ = O.gautschi_g2_steps(O.grid(dim, n, n, n, dx, dx), O.GG_KINDS[kname], u0, up, mf, dt, steps, m)
    assert rel_l2(a, ref) <= 1e-10


def test_gautschi_g2_golden():
    d = np.load(os.path.join(GOLD, "gautschi_g2.npz"))
    n, dt = int(d["n"]), float(d["dt"])
    for kname, eq in EQ.items():
        a, _ = _gpu(2, n, n, 1, float(d["dx"]), eq, d["u0"], d["u0"] - dt * d["v0"], d["mfield"], dt,
                    int(d["steps"]), int(d["m"]))
        assert rel_l2(a, d[f"u_{kname}"]) <= 1e-10, kname


@pytest.mark.parametrize("kname", ["phi4", "sg_hyperbolic"])
def test_gautschi_g2_folded_alpha_and_m(kname):
    """Folded alpha on (forced) and Krylov dimensions 3 / 16 / 32."""
    n, L, dt = 36, 4.0, 1e-2
    dx = 2 * L / (n - 1)
    u0, v0, mf = _ic(2, n, L, 9)
    up = u0 - dt * v0
    for m in (3, 16, 32):
        a, tm = _env({"NLS_FUSED_ALPHA": "1"}, lambda: _gpu(2, n, n, 1, dx, EQ[kname], u0, up, mf, dt, 5, m))
        ref, _ = O.gautschi_g2_steps(O.grid(2, n, n, 1, dx, dx), O.GG_KINDS[kname], u0, up, mf, dt, 5, m)
        assert rel_l2(a, ref) <= 1e-10, m


@pytest.mark.parametrize("dim,n,nranks", [(2, 30, 3), (3, 14, 2)])
def test_gautschi_g2_slabs(dim, n, nranks):
    """y-/z-slab decomposition (nls_group) incl. the Neumann BC on the boundary slabs."""
    L, m, dt, steps = 4.0, 10, 1e-2, 5
    dx = 2 * L / (n - 1)
    u0, v0, mf = _ic(dim, n, L, 2)
    up = u0 - dt * v0
    P = n * n if dim == 3 else n
    ref, _ = O.gautschi_g2_steps(O.grid(dim, n, n, n, dx, dx), 3, u0, up, mf, dt, steps, m)
    grp = nls_amd.Group(nranks)
    out, err = [None] * nranks, []

    def work(r):
        try:
            with nls_amd.Solver(dim, n, n, n, dx, dx, equation=nls_amd.PHI4, m=m, device=0, nranks=nranks,
                                rank=r, group=grp) as s:
                sl = slice(s.z0 * P, (s.z0 + s.nzl) * P)
                s.set_sg_state(u0[sl], up[sl], mf[sl])
                for _ in range(steps):
                    s.step(dt, 1)
                    s.apply_bc()
                out[r] = (s.z0, s.get_field())
        except Exception as e:  # noqa: BLE001
            err.append((r, e))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    [t.start() for t in ts]
    [t.join(timeout=300) for t in ts]
    grp.close()
    assert not err, err
    got = np.concatenate([f for _, f in sorted(out, key=lambda t: t[0])])
    assert rel_l2(got, ref) <= 1e-10


@pytest.mark.parametrize("kname", sorted(PROG))
def test_gautschi_g2_driver_matches_oracle(tmp_path, kname):
    """`prog nx ny Lx Ly u0.npy v0.npy traj.npy T nt ns [m.npy]` as phi4_driver_dev.cpp:16-127."""
    nx = ny = 32
    L, T, nt, ns = 4.0, 0.2, 20, 4
    u0, v0, mf = _ic(2, nx, L, 13)
    for name, arr in (("u0", u0), ("v0", v0), ("m", mf)):
        np.save(tmp_path / f"{name}.npy", arr.reshape(ny, nx))
    out = tmp_path / "traj.npy"
    r = subprocess.run([os.path.join(BIN, PROG[kname]), str(nx), str(ny), str(L), str(L),
                        str(tmp_path / "u0.npy"), str(tmp_path / "v0.npy"), str(out), str(T), str(nt), str(ns),
                        str(tmp_path / "m.npy")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    traj = np.load(out)
    assert traj.shape == (ns, ny, nx) and traj.dtype == np.float64
    dx, dt, freq = 2 * L / (nx - 1), T / nt, nt // ns
    g = O.grid(2, nx, ny, 1, dx, dx)
    u, up = u0.copy(), u0 - dt * v0
    ref = [u0.copy()]
    for i in range(1, nt):
        u, up = O.gautschi_g2_steps(g, O.GG_KINDS[kname], u, up, mf, dt, 1, 10, bc=True)
        if i % freq == 0 and len(ref) < ns:
            ref.append(u.copy())
    for k in range(ns):
        assert rel_l2(traj[k].ravel(), ref[k]) <= 1e-10, k


def test_gautschi_g2_driver_default_m_on_bad_coupling(tmp_path):
    """A misshapen m file falls back to m = 1 with the reference's messages
    (phi4_driver_dev.cpp:68-74), the run continues."""
    nx = ny = 16
    u0, v0, _ = _ic(2, nx, 4.0, 1)
    np.save(tmp_path / "u0.npy", u0.reshape(ny, nx))
    np.save(tmp_path / "v0.npy", v0.reshape(ny, nx))
    np.save(tmp_path / "m.npy", np.ones((3, 3)))
    r = subprocess.run([os.path.join(BIN, "phi4_dev"), str(nx), str(ny), "4", "4", str(tmp_path / "u0.npy"),
                        str(tmp_path / "v0.npy"), str(tmp_path / "a.npy"), "0.05", "5", "5",
                        str(tmp_path / "m.npy")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "Using default m=1.0 everywhere" in r.stderr
    r2 = subprocess.run([os.path.join(BIN, "phi4_dev"), str(nx), str(ny), "4", "4", str(tmp_path / "u0.npy"),
                         str(tmp_path / "v0.npy"), str(tmp_path / "b.npy"), "0.05", "5", "5"],
                        capture_output=True, text=True, timeout=120)
    assert r2.returncode == 0
    assert np.array_equal(np.load(tmp_path / "a.npy"), np.load(tmp_path / "b.npy"))
