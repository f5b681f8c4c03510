"""Generate the committed golden fixtures (small .npz, no pickles).

Inputs are seeded synthetic fields; expected outputs come from the C oracle
(oracle/nls_oracle.cpp, a restatement of the reference G1 Eigen path) and are
cross-checked here against the independent numpy twin (oracle/np_ref.py)
before being written.  Parity status: the reference itself cannot be built
in this image (Eigen3 / libnpy absent), so these vectors are restatement
outputs, pinned by the reference's published scipy known-answer test
(tests/test_oracle.py::test_scipy_kat) -- see DESIGN.md "Oracle".

Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import np_ref  # noqa: E402
import oracle_py as O  # noqa: E402


def field(dim, n, L, seed):
    rng = np.random.default_rng(seed)
    x = np.linspace(-L, L, n)
    if dim == 2:
        Y, X = np.meshgrid(x, x, indexing="ij")
        u = np.exp(-((X - 1) ** 2 + Y ** 2)) * np.exp(1j * X) + 0.5 * np.exp(-((X + 2) ** 2 + (Y - 1) ** 2))
    else:
        Z, Y, X = np.meshgrid(x, x, x, indexing="ij")
        u = np.exp(-((X - 1) ** 2 + Y ** 2 + Z ** 2)) * np.exp(1j * (X + Z))
    u = u.ravel() + 1e-3 * (rng.standard_normal(u.size) + 1j * rng.standard_normal(u.size))
    return u


def main():
    cases = {}
    # --- cubic NLSE 2D 32^2, m=10, 20 steps (nlse_call defaults) --------------
    n, L, dt = 32, 10.0, 1e-3
    dx = 2 * L / (n - 1)
    u0 = field(2, n, L, 1)
    u0 /= np.sqrt(np.sum(np.abs(u0) ** 2) * dx * dx)
    g = O.grid(2, n, n, 1, dx, dx)
    out = O.nlse_steps(g, u0, dt, 20, 10)
    tw = np_ref.nlse_steps(2, n, n, 1, dx, dx, u0, dt, 20, 10)
    assert np.linalg.norm(out - tw) / np.linalg.norm(tw) < 1e-12
    cases["nlse2d"] = dict(dim=2, n=n, dx=dx, dt=dt, steps=20, m=10, nonlin=0, u0=u0, u=out)
    # --- cubic-quintic 2D 24^2, m=16, 10 steps ----------------------------------
    n = 24
    dx = 2 * L / (n - 1)
    u0 = field(2, n, L, 2)
    u0 /= np.sqrt(np.sum(np.abs(u0) ** 2) * dx * dx)
    g = O.grid(2, n, n, 1, dx, dx)
    out = O.nlse_steps(g, u0, dt, 10, 16, nonlin=1)
    tw = np_ref.nlse_steps(2, n, n, 1, dx, dx, u0, dt, 10, 16, nonlin=1)
    assert np.linalg.norm(out - tw) / np.linalg.norm(tw) < 1e-12
    cases["cq2d"] = dict(dim=2, n=n, dx=dx, dt=dt, steps=10, m=16, nonlin=1, u0=u0, u=out)
    # --- cubic NLSE 3D 12^3, m=16, 5 steps --------------------------------------
    n = 12
    dx = 2 * L / (n - 1)
    u0 = field(3, n, L, 3)
    u0 /= np.sqrt(np.sum(np.abs(u0) ** 2) * dx ** 3)
    g = O.grid(3, n, n, n, dx, dx)
    out = O.nlse_steps(g, u0, dt, 5, 16)
    tw = np_ref.nlse_steps(3, n, n, n, dx, dx, u0, dt, 5, 16)
    assert np.linalg.norm(out - tw) / np.linalg.norm(tw) < 1e-12
    cases["nlse3d"] = dict(dim=3, n=n, dx=dx, dt=dt, steps=5, m=16, nonlin=0, u0=u0, u=out)
    # --- sine-Gordon 2D 32^2, Gautschi m=10, 10 steps ---------------------------
    n, L = 32, 3.0
    dx = 2 * L / (n - 1)
    x = np.linspace(-L, L, n)
    Y, X = np.meshgrid(x, x, indexing="ij")
    su0 = (2.0 * np.arctan(np.exp(3.0 - 5.0 * np.sqrt(X * X + Y * Y)))).ravel()
    sdt = 5.0 / 500
    sup = su0.copy()
    mf = -np.ones(su0.size)
    g = O.grid(2, n, n, 1, dx, dx)
    su, sup1 = O.sg_steps(g, su0, sup, mf, sdt, 10, 10)
    tu, tup = np_ref.sg_steps(2, n, n, 1, dx, dx, su0, sup, mf, sdt, 10, 10)
    assert np.linalg.norm(su - tu) / np.linalg.norm(tu) < 1e-11
    cases["sg2d"] = dict(dim=2, n=n, dx=dx, dt=sdt, steps=10, m=10, u0=su0, u_past0=sup, mfield=mf,
                         u=su, u_past=sup1)
    # --- one Krylov action per matrix function, 3D 10^3 -------------------------
    n, L = 10, 5.0
    dx = 2 * L / (n - 1)
    g = O.grid(3, n, n, n, dx, dx)
    ur = np.real(field(3, n, L, 4))
    uc = field(3, n, L, 5)
    kr = {f"f{f}": O.krylov_r(g, ur, 1e-2, 12, f) for f in (2, 3, 4, 5, 6)}
    kc = {"f0": O.krylov_c(g, uc, -1e-2j, 12, 0), "f1": O.krylov_c(g, uc, 1e-2j, 12, 1)}
    lap = O.laplacian_c(g, uc)
    cases["krylov3d"] = dict(dim=3, n=n, dx=dx, m=12, ur=ur, uc=uc, lap=lap,
                             **{"r_" + k: v for k, v in kr.items()}, **{"c_" + k: v for k, v in kc.items()})
    # --- G2 cubic NLSE with m(x), c(x) and the Neumann copy BC -----------------
    #     (nlse_cubic_driver_3d.cpp: m=25; nlse_cubic_driver_2d.cpp: m=20)
    for name, dim, n, m, steps in (("g2_3d", 3, 12, 25, 5), ("g2_2d", 2, 24, 20, 10)):
        L = 4.0
        dx = 2 * L / (n - 1)
        rng = np.random.default_rng(7 + dim)
        u0 = field(dim, n, L, 10 + dim)
        N = u0.size
        cf = 1.0 + 0.5 * np.sin(np.arange(N) * 0.37) + 0.1 * rng.random(N)
        mf = 1.0 + 0.3 * rng.standard_normal(N)
        g = O.grid(dim, n, n, n, dx, dx)
        out = O.nlse_g2_steps(g, cf, mf, u0, dt, steps, m, bc=True)
        tw = np_ref.nlse_g2_steps(dim, n, n, n, dx, dx, cf, mf, u0, dt, steps, m, bc=True)
        assert np.linalg.norm(out - tw) / np.linalg.norm(tw) < 1e-12
        cases[name] = dict(dim=dim, n=n, dx=dx, dt=dt, steps=steps, m=m, u0=u0, c=cf, mfield=mf, u=out)
    # --- G2 sEWI (nlse_cubic_sewi_driver_3d.cpp: m=15), steps 1..6 with BC ----
    n, m, steps, L = 10, 15, 6, 4.0
    dx = 2 * L / (n - 1)
    rng = np.random.default_rng(21)
    u0 = field(3, n, L, 22)
    N = u0.size
    cf = 1.0 + 0.3 * np.cos(np.arange(N) * 0.21) + 0.1 * rng.random(N)
    mf = 1.0 + 0.2 * rng.standard_normal(N)
    g = O.grid(3, n, n, n, dx, dx)
    out, outp = O.nlse_sewi_steps(g, cf, mf, u0, None, dt, 1, steps, m, bc=True)
    tw, twp = np_ref.nlse_sewi_steps(3, n, n, n, dx, dx, cf, mf, u0, None, dt, 1, steps, m, bc=True)
    assert np.linalg.norm(out - tw) / np.linalg.norm(tw) < 1e-12
    cases["sewi_3d"] = dict(dim=3, n=n, dx=dx, dt=dt, steps=steps, m=m, u0=u0, c=cf, mfield=mf, u=out, u_prev=outp)
    # --- G2 Klein-Gordon Gautschi (kg_driver_dev_3d.cpp: m=10), BC after steps --
    n, m, steps, L, kdt = 10, 10, 8, 3.0, 5e-3
    dx = 2 * L / (n - 1)
    rng = np.random.default_rng(31)
    x = np.linspace(-L, L, n)
    Z, Y, X = np.meshgrid(x, x, x, indexing="ij")
    ku0 = (np.exp(-(X ** 2 + Y ** 2 + Z ** 2)) + 1e-3 * rng.standard_normal(X.shape)).ravel()
    kv0 = (0.1 * np.sin(X) * np.exp(-(Y ** 2 + Z ** 2))).ravel()
    cf = 1.0 + 0.3 * np.sin(0.5 * X + 0.2 * Z).ravel()
    mf = 1.0 + 0.2 * np.cos(Y).ravel()
    g = O.grid(3, n, n, n, dx, dx)
    ku, kup, kv = O.kg_steps(g, cf, mf, ku0, ku0 - kdt * kv0, kdt, steps, m, bc=True)
    tu, tup, tv = np_ref.kg_steps(3, n, n, n, dx, dx, cf, mf, ku0, ku0 - kdt * kv0, kdt, steps, m, bc=True)
    assert np.linalg.norm(ku - tu) / np.linalg.norm(tu) < 1e-12
    cases["kg_3d"] = dict(dim=3, n=n, dx=dx, dt=kdt, steps=steps, m=m, u0=ku0, v0=kv0, c=cf, mfield=mf,
                          u=ku, u_past=kup, v=kv)
    # --- G2 Gautschi family (phi4_dev / sg_{single,double,hyperbolic}_dev: m=10), BC per step
    n, m, steps, L, gdt = 24, 10, 8, 4.0, 1e-2
    dx = 2 * L / (n - 1)
    x = np.linspace(-L, L, n)
    Y, X = np.meshgrid(x, x, indexing="ij")
    rng = np.random.default_rng(41)
    gu0 = (1.5 * np.exp(-(X ** 2 + Y ** 2) / 2) + 1e-3 * rng.standard_normal(X.shape)).ravel()
    gv0 = (0.2 * np.sin(X) * np.exp(-Y ** 2)).ravel()
    gmf = (1.0 + 0.2 * np.cos(X + Y)).ravel()
    g = O.grid(2, n, n, 1, dx, dx)
    gg = dict(dim=2, n=n, dx=dx, dt=gdt, steps=steps, m=m, u0=gu0, v0=gv0, mfield=gmf)
    for kname, kind in O.GG_KINDS.items():
        ku, kup = O.gautschi_g2_steps(g, kind, gu0, gu0 - gdt * gv0, gmf, gdt, steps, m, bc=True)
        tu, _ = np_ref.gautschi_g2_steps(2, n, n, 1, dx, dx, kind, gu0, gu0 - gdt * gv0, gmf, gdt, steps, m)
        assert np.linalg.norm(ku - tu) / np.linalg.norm(tu) < 1e-12, kname
        gg[f"u_{kname}"], gg[f"u_past_{kname}"] = ku, kup
    cases["gautschi_g2"] = gg
    # --- G2 cubic-quintic (nlse_cubic_quintic_driver_dev.cpp: m=15), real sigmas,
    #     m(x), isotropic operator, BC per step ------------------------------------
    n, m, steps, L = 24, 15, 10, 4.0
    dx = 2 * L / (n - 1)
    rng = np.random.default_rng(51)
    u0 = field(2, n, L, 52)
    mf = 1.0 + 0.3 * rng.standard_normal(u0.size)
    s1, s2 = 1.0, -0.5
    g = O.grid(2, n, n, 1, dx, dx)
    out = O.nlse_cq_g2_steps(g, mf, u0, dt, steps, m, s1, s2, bc=True)
    tw = np_ref.nlse_cq_g2_steps(2, n, n, 1, dx, dx, mf, u0, dt, steps, m, s1, s2, bc=True)
    assert np.linalg.norm(out - tw) / np.linalg.norm(tw) < 1e-12
    cases["cq_g2_2d"] = dict(dim=2, n=n, dx=dx, dt=dt, steps=steps, m=m, s1=s1, s2=s2, u0=u0, mfield=mf, u=out)
    only = sys.argv[1:]  # optional: regenerate only the named fixtures
    for name, d in cases.items():
        if only and name not in only:
            continue
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **{k: np.asarray(v) for k, v in d.items()})
    total = sum(os.path.getsize(os.path.join(HERE, f"{k}.npz")) for k in cases
                if os.path.exists(os.path.join(HERE, f"{k}.npz")))
    print(f"wrote {len(cases)} fixtures, {total / 1024:.1f} KiB")


if __name__ == "__main__":
    main()
