"""GPU: the drop-in CLI drivers end to end (argv + .npy in, .npy out), checked
against the oracle driven with the reference drivers' semantics
(device/nlse_call.cpp:35-82, device/sg_driver_dev.cpp:23-80)."""
import os
import re
import subprocess

import numpy as np
import pytest

import oracle_py as O
from conftest import rel_l2

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "nonlinear-solvers_amd", "bin")


def reference_trajectory(dim, n, L, u0, T, nt, ns, m=10, nonlin=0):
    dx = 2 * L / (n - 1)
    dt = T / nt
    freq = nt // ns
    u = u0.ravel() / np.sqrt(np.sum(np.abs(u0) ** 2) * dx ** dim)
    g = O.grid(dim, n, n, n, dx, dx)
    snaps = [u.copy()]
    for i in range(1, nt):
        u = O.nlse_steps(g, u, dt, 1, m, nonlin=nonlin)
        if i % freq == 0 and len(snaps) < ns:
            snaps.append(u.copy())
    return np.array(snaps)


def ic(dim, n, L):
    x = np.linspace(-L, L, n)
    if dim == 2:
        Y, X = np.meshgrid(x, x, indexing="ij")
        return np.exp(-((X - 3) ** 2 + (Y - 3) ** 2) / 0.16) * np.exp(-1j * (X + Y)) + \
            np.exp(-((X + 3) ** 2 + (Y + 3) ** 2) / 0.16) * np.exp(1j * (X + Y))   # nlse_driver.cpp:52-66
    Z, Y, X = np.meshgrid(x, x, x, indexing="ij")
    return np.exp(-(X ** 2 + Y ** 2 + Z ** 2) / 2) * np.exp(1j * X)


@pytest.mark.parametrize("prog,nonlin", [("nlse_call", 0), ("nlse_cq_call", 1), ("to_nlse_call", 0),
                                         ("to_nlse_cq_call", 1)])
def test_nlse_call_matches_oracle(tmp_path, prog, nonlin):
    n, L, T, nt, ns = 32, 10.0, 0.02, 20, 4
    u0 = ic(2, n, L)
    fi, fo = tmp_path / "u0.npy", tmp_path / "traj.npy"
    np.save(fi, u0)
    r = subprocess.run([os.path.join(BIN, prog), str(n), str(n), str(L), str(L), str(fi), str(fo),
                        str(T), str(nt), str(ns)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert re.match(r"^Trajectory took: \d\.\d{4}e[+-]\d\ds$", r.stdout.strip())
    out = np.load(fo)
    assert out.shape == (ns, n, n) and out.dtype == np.complex128
    ref = reference_trajectory(2, n, L, u0, T, nt, ns, nonlin=nonlin).reshape(ns, n, n)
    for k in range(ns):
        assert rel_l2(out[k], ref[k]) <= 1e-10


def twin_trajectory(n, L, u0, T, nt, ns, m=10):
    """The same trajectory from the numpy twin (np_ref: MGS + LAPACK eigh), the
    second independent CPU restatement (for the parity record only)."""
    import np_ref as R
    dx = 2 * L / (n - 1)
    dt = T / nt
    freq = nt // ns
    u = u0.ravel() / np.sqrt(np.sum(np.abs(u0) ** 2) * dx ** 2)
    snaps = [u.copy()]
    done = 0
    for i in range(freq, nt, freq):
        if len(snaps) >= ns:
            break
        u = R.nlse_steps(2, n, n, 1, dx, dx, u, dt, i - done, m)
        done = i
        snaps.append(u.copy())
    return np.array(snaps)


def test_c1_nlse_call_full_run_matches_oracle(tmp_path):
    """BASELINE C1 end to end: `nlse_call 256 256 10 10 u0 traj 0.5 500 100` -- the
    nlse_driver.cpp workload (2D 256^2, dt = T/nt = 1e-3, nt - 1 = 499 SS2 steps,
    m = 10, snapshot every nt/ns = 5 steps, nlse_driver.cpp:52-66 initial data;
    nlse_call.cpp:35-85, nlse_driver.cpp:27-106) -- against the oracle's 499-step
    trajectory, all 100 snapshots.  On this smooth initial field the reference
    algorithm amplifies its own rounding (~20x per step: the Lanczos basis blows
    high-mode rounding noise up by prod ||L|| / beta_j): the oracle started from
    u0 moved by one ulp per component drifts from the unperturbed oracle to ~1e-6
    after 5 steps and saturates near 1e-5 (conftest.self_floor).  The bound per
    snapshot is parity_bound(1e-10, that self-floor, "c1") = max(1e-10, 2 x floor)
    (observed GPU / floor <= 0.71, profiles/r03/parity_floor.txt); one step is checked
    at 1e-10 through the C-ABI directly, and the mechanism itself: the oracle continued
    from the GPU's field after that one step lands within PROPAGATED_FACTOR of the GPU
    at every later snapshot (the GPU's deviation is its first step's rounding, amplified
    by the reference algorithm at its own rate)."""
    from conftest import PROPAGATED_FACTOR, parity_bound, record_parity, self_floor
    n, L, T, nt, ns = 256, 10.0, 0.5, 500, 100
    u0 = ic(2, n, L)
    fi, fo = tmp_path / "u0.npy", tmp_path / "traj.npy"
    np.save(fi, u0)
    r = subprocess.run([os.path.join(BIN, "nlse_call"), str(n), str(n), str(L), str(L), str(fi), str(fo),
                        str(T), str(nt), str(ns)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert re.match(r"^Trajectory took: \d\.\d{4}e[+-]\d\ds$", r.stdout.strip())
    out = np.load(fo)
    assert out.shape == (ns, n, n) and out.dtype == np.complex128
    # the oracle from u0 and from two one-ulp perturbations of u0 (each normalised
    # as nlse_call.cpp:41-49 does)
    ref, floor = self_floor(lambda u: reference_trajectory(2, n, L, u, T, nt, ns), u0.ravel())
    ref = ref.reshape(ns, n, n)
    twin = twin_trajectory(n, L, u0, T, nt, ns).reshape(ns, n, n) if os.environ.get("NLS_PARITY_LOG") else None
    # one SS2 step of the same workload: below the floor's growth, 1e-10 holds
    import nls_amd
    dx = 2 * L / (n - 1)
    u = u0.ravel() / np.sqrt(np.sum(np.abs(u0) ** 2) * dx * dx)
    with nls_amd.Solver(2, n, n, 1, dx, dx, m=10) as s:
        s.set_field(u)
        s.step(T / nt, 1)
        one = s.get_field()
    g = O.grid(2, n, n, 1, dx, dx)
    assert rel_l2(one, O.nlse_steps(g, u, T / nt, 1, 10)) <= 1e-10
    # the oracle continued from the GPU's step-1 field, snapshot by snapshot
    prop, v, freq = {}, one, nt // ns
    for k in range(1, ns):  # snapshot k is step k * freq; v holds step 1, then (k-1) * freq
        v = O.nlse_steps(g, v, T / nt, freq - 1 if k == 1 else freq, 10)
        prop[k] = rel_l2(v, ref[k])
    rows = [(k, rel_l2(out[k], ref[k]), floor[k], rel_l2(twin[k], ref[k]) if twin is not None else None,
             prop.get(k)) for k in range(ns)]
    record_parity("C1 nlse_call 256^2 T=0.5 nt=500 ns=100 (snapshot = every 5 steps)", rows, "c1")
    bad = [(k, e, f, p) for k, e, f, _, p in rows
           if e > parity_bound(1e-10, f, "c1") or (p is not None and e > max(1e-10, PROPAGATED_FACTOR * p))]
    assert not bad, "snapshot, gpu err, self-floor, propagated: " + ", ".join(
        f"({k}, {e:.2e}, {f:.2e}, {p if p is None else f'{p:.2e}'})" for k, e, f, p in bad[:8])


def test_nlse_call_3d_matches_oracle(tmp_path):
    n, L, T, nt, ns = 12, 5.0, 0.01, 10, 2
    u0 = ic(3, n, L)
    fi, fo = tmp_path / "u0.npy", tmp_path / "traj.npy"
    np.save(fi, u0)
    r = subprocess.run([os.path.join(BIN, "nlse_call_3d"), str(n), str(n), str(n), str(L), str(L), str(L),
                        str(fi), str(fo), str(T), str(nt), str(ns), "--m=16"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = np.load(fo)
    assert out.shape == (ns, n, n, n)
    ref = reference_trajectory(3, n, L, u0, T, nt, ns, m=16).reshape(ns, n, n, n)
    for k in range(ns):
        assert rel_l2(out[k], ref[k]) <= 1e-10


def test_sg_driver_matches_oracle(tmp_path):
    n, L, T, nt, ns = 32, 3.0, 0.2, 20, 4
    r = subprocess.run([os.path.join(BIN, "sg_driver_dev"), f"--nx={n}", f"--T={T}", f"--nt={nt}",
                        f"--ns={ns}", f"--prefix={tmp_path}/sg"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    u = np.load(tmp_path / "sg_u_device.npy")
    v = np.load(tmp_path / "sg_v_device.npy")
    assert u.shape == (ns, n, n) and v.shape == (ns, n, n)
    dx = 2 * L / (n - 1)
    dt = T / nt
    x = np.linspace(-L, L, n)
    X, Y = np.meshgrid(x, x, indexing="ij")
    u0 = (2.0 * np.arctan(np.exp(3.0 - 5.0 * np.sqrt(X * X + Y * Y)))).ravel()
    g = O.grid(2, n, n, 1, dx, dx)
    cu, cp = u0.copy(), u0.copy()
    mf = -np.ones(n * n)
    ref_u, ref_v = [u0], [np.zeros(n * n)]
    for i in range(1, nt):
        cu, cp = O.sg_steps(g, cu, cp, mf, dt, 1, 10)
        if i % (nt // ns) == 0 and len(ref_u) < ns:
            ref_u.append(cu.copy())
            ref_v.append((cu - cp) / dt)
    for k in range(ns):
        assert rel_l2(u[k].ravel(), ref_u[k]) <= 1e-10
        if k:
            assert rel_l2(v[k].ravel(), ref_v[k]) <= 1e-8
