#!/usr/bin/env python3
"""Headline benchmark: Mcells*steps/s of the Krylov/Lanczos exponential
time-stepper (BASELINE.json metric), one JSON line on rank 0.

Default workload = BASELINE.json configs[2]: 3D cubic NLSE 512^3, Krylov m=16,
complex128, dt=1e-3, L=10 (dx = 2L/(n-1), nlse_call.cpp:35).  A "step" is one
full Strang SS2 step (N(1/2) -> Krylov exp -> N(1/2)).  Inputs are resident in
HBM before the timed region.  With --gpus N (launched by torch.distributed.run)
the 512^3 grid is z-slab decomposed over N ranks (strong scaling) with RCCL halo
exchange + all-reduce of the Lanczos dot products.

roofline: for the NLSE the dominant kernel is the fused tail k_tail<NLSE, m>
(the last Lanczos vector + combination + both nonlinear half-steps; m-1 stored
vectors read, the next start vector written, u on a call's last step: the most
bytes per launch; the largest two-vector pass k_p2d<m-4> takes about as long at
512^3, m = 16), for the real Gautschi equations the largest
two-vector pass; timed with HIP events on the
solver's own stream in a separate pass of --prof-steps steps right after the
timed region (the timed region itself carries no per-launch events).
--gpus N without torch.distributed.run: bench.py starts the N ranks itself.
cpu_baseline: the oracle (single-threaded C++ restatement of the reference's
Eigen path, oracle/) on a bounded 128^3 sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nonlinear-solvers_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)

WORKLOADS = {
    # name: dim, n, L, m, equation, dt, description (BASELINE.json configs)
    "nlse3d_512": dict(dim=3, n=512, L=10.0, m=16, eq=0, dt=1e-3,
                       desc="3D cubic NLSE 512^3, Krylov m=16, fp64 complex"),
    "nlse2d_4096": dict(dim=2, n=4096, L=10.0, m=16, eq=0, dt=1e-3,
                        desc="2D cubic NLSE 4096x4096, Krylov m=16, fp64 complex"),
    "sg2d_8192": dict(dim=2, n=8192, L=3.0, m=10, eq=2, dt=5.0 / 500,
                      desc="2D sine-Gordon 8192x8192, Gautschi, Krylov m=10, fp64"),
    "cq3d_1024": dict(dim=3, n=1024, L=10.0, m=16, eq=1, dt=1e-3,
                      desc="3D cubic-quintic NLSE 1024^3, Krylov m=16, fp64 complex"),
    # G2 production driver (nlse_cubic_driver_3d.cpp: m=25, m(x), c(x), Neumann BC per step)
    "g2_3d_256": dict(dim=3, n=256, L=10.0, m=25, eq=3, dt=1e-3,
                      desc="G2 3D cubic NLSE 256^3 with m(x), div(c grad), Neumann BC, Krylov m=25, fp64 complex"),
    # G2 Klein-Gordon Gautschi driver (kg_driver_dev_3d.cpp: m=10, m(x), c(x), BC per step)
    "kg_3d_256": dict(dim=3, n=256, L=10.0, m=10, eq=4, dt=1e-3,
                      desc="G2 3D Klein-Gordon 256^3 (u_tt = div(c grad u) - m u^3), Gautschi, Neumann BC, "
                           "Krylov m=10, fp64"),
    # G2 sEWI driver (nlse_cubic_sewi_driver_3d.cpp: m=15, three Krylov actions per step)
    "sewi_3d_256": dict(dim=3, n=256, L=10.0, m=15, eq=3, dt=1e-3, sewi=True,
                        desc="G2 3D cubic NLSE 256^3, sEWI integrator, m(x), div(c grad), Neumann BC, "
                             "Krylov m=15, fp64 complex"),
}


def g2_coefficients(n, L, z0, nzl):
    """Smooth synthetic focusing field m(x) in [0.5, 1.5] and anisotropy c(x) in [0.7, 1.3]."""
    x = np.linspace(-L, L, n)
    Z = x[z0:z0 + nzl][:, None, None]
    Y = x[None, :, None]
    X = x[None, None, :]
    mf = 1.0 + 0.5 * np.cos(0.3 * X) * np.cos(0.2 * Y) * np.cos(0.25 * Z)
    cf = 1.0 + 0.3 * np.sin(0.4 * X + 0.1 * Y) * np.cos(0.3 * Z)
    return mf.ravel(), cf.ravel()


def algorithmic_bytes_per_cell_step(m: int, eq: int, sewi: bool = False) -> int:
    """E(m) = ((m-1)(m+2)/2 + m + 3) * 16 B (NLSE c128);
    E_SG(m) = ((m-1)(m+2) + 2m + 10) * 8 B (sine-Gordon f64).  sEWI: three
    Krylov actions per step, each (m-1)(m+2)/2 + m + 1 elements (start vector
    written, basis streamed, result combined), plus B(u), u_prev copy and the
    final update (read u, e, write u, u_prev)."""
    if eq in (2, 4):  # two real Krylov bases per step (SG: id+cos / sinc^2; KG: cos / sinc^2)
        return ((m - 1) * (m + 2) + 2 * m + 10) * 8
    if sewi:
        return (3 * ((m - 1) * (m + 2) // 2 + m + 1) + 8) * 16
    return ((m - 1) * (m + 2) // 2 + m + 3) * 16


def moved_bytes_per_cell_step(w, m, sched, pass2, u_frac, tm, steps):
    """Bytes per cell and step THIS implementation moves (DESIGN.md sections 3-4), by
    the launch sequence of the step; None where no model is written (KG, sEWI).
      two-vector NLSE: alpha_0 (blind start: first step only) + sum over passes
        (J+1 reads + ns writes) + the tail's alpha + tail (m-1 reads, W_0 and u on a
        call's last step);
      two-vector Gautschi (SG, two bases of f64, cell pairs): per basis the passes +
        alpha + tail; the mid tail reads S_0..S_{m-2}, m(x), u_past and writes u_past,
        g_0 (m+3), the end tail reads S_0..S_{m-2}, u_past, u and writes u, u_past (m+3);
      two-vector G2 NLSE: LDS-DMA form (k_p2d with c staged beside S_J): per pass
        S_0..S_J + c in, ns out; register form (nls_pass2g.hpp, two launches per
        pass -- told apart by the J = 0 launch count): the y = L S_J launch (S_J + c
        in, y out) and the pass (y + c + S_0..S_J in, ns out); then the tail's alpha
        (+ c), the tail (m-1 reads + c + m(x), u and W_0 written);
      one-vector G2 NLSE (div(c grad), m(x)): alpha passes j = 0..m-3 (W_j + c), the
        tail's alpha (W_{m-2} + c), updates J = 0..m-3 ((J+2) vectors + c), tail (m-1
        reads + c + m(x), u and W_0 written);
      two-vector Klein-Gordon (f64 cell pairs, div(c grad)): g = -m u^3 (u, m in, g out);
        per basis (g, then u) alpha_0 (W_0 + c; blind start: first step only), the passes
        (S_0..S_J + c in, ns out), the tail's alpha (S_{m-2} + c); the g basis's tail
        (m-1 reads + c, its W_0 written), the Gautschi tail (m-1 reads + c + that W_0 +
        u_past; u, u_past, v written);
      G2 sEWI (steps > 1, nls_step_sewi: three Krylov actions on one basis, each cold --
        alpha_0 (W_0 + c), the passes (LDS-DMA or register form, as the G2 NLSE), the
        tail's alpha (S_{m-2} + c)): B(u) (u, m in, W_0 out); the sinc action's tail into
        W_0 (m-1 reads + c, W_0 written); the exp action's tail into e (the same, e
        written); the W_0 <- u_prev copy (read + write); the exp(2 tau) action's tail
        (m-1 reads + c + e + u in; u and u_prev written).  (The driver's Neumann BC after
        each step touches the boundary shell only, ~6/n of a vector: not counted.)"""
    eq = w["eq"]
    if pass2 and w.get("sewi"):
        reg = tm["update_count"][0] > 4.5 * max(1, tm["steps"])  # two J = 0 launches per action
        if reg:
            passes = sum((j + 1 + ns) * 16 + (16 + 8 + 16) + (16 + 8) for j, ns in sched)
        else:
            passes = sum((j + 1 + ns) * 16 + 8 for j, ns in sched)
        action = (16 + 8) + passes + (16 + 8)
        tails = 2 * ((m - 1) * 16 + 8 + 16) + ((m - 1) * 16 + 8 + 16 + 16 + 16 + 16)
        return (16 + 8 + 16) + 3 * action + tails + 32
    if pass2 and eq == 4 and not w.get("sewi"):
        a0 = tm["class_count"].get("alpha", 0) - tm["class_count"].get("final", 0)  # alpha_0 launches
        a0 = max(0, a0) / max(1, tm["steps"])  # per step, both bases
        per_basis = sum((j + 1 + ns) * 8 + 8 for j, ns in sched) + 16
        return 24 + a0 * 16 + 2 * per_basis + ((m - 1) * 8 + 16) + ((m - 1) * 8 + 8 + 16 + 24)
    if w.get("sewi") or eq == 4:
        return None
    if pass2 and eq in (0, 1):
        a0 = tm["class_count"].get("alpha", 0) - tm["class_count"].get("final", 0)  # alpha_0 launches
        a0 = max(0, a0) / max(1, tm["steps"])
        return 16 * (a0 + sum(j + 1 + ns for j, ns in sched) + 1 + (m + u_frac))
    if pass2 and eq == 2:
        per_basis = sum(j + 1 + ns for j, ns in sched) + 1
        return 8 * (2 * per_basis + 2 * (m + 3))
    if pass2 and eq == 3:
        reg = tm["update_count"][0] > 1.5 * max(1, tm["steps"])  # two J = 0 launches per run
        if reg:
            # register two-vector passes (k_lap + k_p2m): per pass S_J + c read and y =
            # L S_J written, then y (stencil) + c + S_0..S_J read and ns vectors written
            passes = sum((j + 1 + ns) * 16 + (16 + 8 + 16) + (16 + 8) for j, ns in sched)
        else:
            passes = sum((j + 1 + ns) * 16 + 8 for j, ns in sched)
        return passes + (16 + 8) + ((m - 1) * 16 + 8 + 8 + 16 + 16)
    if not pass2 and eq == 3:
        alpha = (m - 1) * (16 + 8)
        upd = sum((J + 2) * 16 + 8 for J in range(m - 2))
        tail = (m - 1) * 16 + 16 + 8 + 8 + 16
        return alpha + upd + tail
    return None


def synthetic_ic(w, z0, nzl, seed=1234):
    """8 random Gaussian solitons with phases + 1e-3 complex white noise.
    Noise is drawn per global plane, so the field does not depend on the rank split."""
    n, L, dim = w["n"], w["L"], w["dim"]
    rng = np.random.default_rng(seed)
    cen = rng.uniform(-L / 2, L / 2, (8, 3))
    kv = rng.uniform(-2, 2, (8, 3))
    wid = rng.uniform(0.5, 1.5, 8)
    x = np.linspace(-L, L, n)
    plane = n * n if dim == 3 else n
    if w["eq"] in (2, 4):
        out = np.empty(nzl * plane, dtype=np.float64)
    else:
        out = np.empty(nzl * plane, dtype=np.complex128)
    if dim == 3:
        # separable Gaussian solitons: exp(-r^2/w^2) exp(i k.x) = prod over axes
        ax = lambda d: np.stack([np.exp(-((x - cen[s, d]) / wid[s]) ** 2 + 1j * kv[s, d] * x)
                                 for s in range(8)], axis=1)   # (n, 8)
        fx, fy, fz = ax(0), ax(1), ax(2)
        for q in range(nzl):
            k = z0 + q
            f = fy @ (fz[k][:, None] * fx.T)     # sum_s fz_s(k) fy_s(y) fx_s(x)
            nr = np.random.default_rng((seed, k))
            f += 1e-3 * (nr.standard_normal((n, n)) + 1j * nr.standard_normal((n, n)))
            out[q * plane:(q + 1) * plane] = (f.real if w["eq"] == 4 else f).ravel()
    else:
        for q in range(nzl):
            k = z0 + q
            y = x[k]
            nr = np.random.default_rng((seed, k))
            if w["eq"] == 2:  # sg_driver_dev.cpp:34-36 + noise
                r = np.sqrt(x * x + y * y)
                out[q * plane:(q + 1) * plane] = 2.0 * np.arctan(np.exp(3.0 - 5.0 * r)) + \
                    1e-3 * nr.standard_normal(n)
            else:
                f = np.zeros(n, dtype=np.complex128)
                for s in range(8):
                    r2 = ((x - cen[s, 0]) ** 2 + (y - cen[s, 1]) ** 2) / wid[s] ** 2
                    f += np.exp(-r2 + 1j * (kv[s, 0] * x + kv[s, 1] * y))
                f += 1e-3 * (nr.standard_normal(n) + 1j * nr.standard_normal(n))
                out[q * plane:(q + 1) * plane] = f
    return out


def global_mass(u, dv, dist=None):
    """sum |u|^2 dV over all ranks' slabs (the unit-mass normalisation of
    nlse_call.cpp:41-49 applied to the whole decomposed field)."""
    mass = float(np.sum(np.abs(u) ** 2) * dv)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        import torch
        t = torch.tensor([mass], dtype=torch.float64)
        dist.all_reduce(t)
        mass = float(t.item())
    return mass


def max_over_ranks(x, dist=None):
    """The bench contract's timing: the slowest rank's elapsed time."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    return x


def cpu_model():
    """The host CPU's model name (BASELINE.md section 3 asks for it)."""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(args, u_full=None, gpu_one=None):
    """The oracle (C++ restatement of nlse_driver.cpp -> NLSESolver::step ->
    expm_multiply) on a bounded sample of the workload, on the host: all cores
    (OpenMP build, SURVEY 8(d) "all cores" mode) and single-threaded (the
    reference's own Eigen path is single-threaded).  For the headline workload the
    reported `value` is ONE SS2 step of the full 512^3 grid (BASELINE.md section 3:
    "a few steps at GPU sizes"; a 34 GB basis in host RAM), all cores; the 128^3
    sub-grid rows stay beside it.  BASELINE C1 is timed in full as well."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py

    one = _cpu_sample(args, oracle_py)
    out = dict(one)
    out["cpu_model"] = cpu_model()
    try:
        oracle_py.use_openmp(True)
        nthr = oracle_py.threads()
        if nthr > 1:
            allc = _cpu_sample(args, oracle_py)
            out = dict(allc)
            out["cores"] = nthr
            out["cpu_model"] = cpu_model()
            out["sample"] = allc["sample"].replace("1 thread", f"OpenMP {nthr} threads")
            out["single_thread"] = {"value": one["value"], "seconds": one["seconds"], "sample": one["sample"]}
        if args.workload == "nlse3d_512":
            out["c1_full_run"] = _cpu_c1(oracle_py, nthr, T=0.5)
            out["c1_nlse_driver_defaults"] = _cpu_c1(oracle_py, nthr, T=1.5)
            if u_full is not None and nthr > 1 and not args.no_full_grid_cpu:
                full = _cpu_full_grid(args, oracle_py, u_full, nthr, gpu_one=gpu_one)
                sub = {k: out[k] for k in ("value", "seconds", "sample", "cores")}
                out.update(full)
                out["subgrid_128"] = sub
    except (OSError, FileNotFoundError):
        pass
    finally:
        oracle_py.use_openmp(False)
    return out


def _cpu_full_grid(args, oracle_py, u, nthr, steps=1, gpu_one=None):
    """One SS2 step of the headline workload at its full grid (512^3, m = 16) through
    the oracle on all cores: the CPU baseline at GPU size.  With gpu_one (the same step of
    the same field on the GPU, bench.py main) also the full-size parity of that step."""
    w = WORKLOADS[args.workload]
    n = w["n"]
    dx = 2 * w["L"] / (n - 1)
    g = oracle_py.grid(3, n, n, n, dx, dx)
    t0 = time.perf_counter()
    ref = oracle_py.nlse_steps(g, u, w["dt"], steps, w["m"], nonlin=w["eq"])
    el = time.perf_counter() - t0
    out = {"value": n ** 3 * steps / el / 1e6, "unit": "Mcells*steps/s", "cores": nthr, "kind": "port",
           "seconds": el,
           "sample": f"3D cubic NLSE {n}^3 m={w['m']} (the full workload grid), {steps} SS2 step, "
                     f"oracle/ C++ -O2 OpenMP {nthr} threads"}
    if gpu_one is not None and steps == 1:
        # north_star: "the final field matches the Eigen CPU path within 1e-10 relative L2"
        # -- here at the headline size itself, one SS2 step from the bench's own field
        out["parity_full_grid"] = {"check": f"GPU vs oracle, one SS2 step of the {n}^3 m={w['m']} bench field",
                                   "rel_l2": rel_l2(gpu_one, ref), "tolerance": 1e-10}
    return out


def _cpu_c1(oracle_py, nthr, T=0.5):
    """BASELINE C1 timed in full on the host through the oracle restatement, all
    cores: 256^2, L = 10, nt = 500 -> 499 SS2 steps, Krylov m = 10, the two-soliton
    collision IC of nlse_driver.cpp:52-66 normalised to unit mass.  T = 0.5 (dt =
    1e-3) is BASELINE.json C1 and the GPU C1 test; T = 1.5 (dt = 3e-3) is
    nlse_driver.cpp:35-40's own default."""
    n, L, nt, m = 256, 10.0, 500, 10
    dx = 2 * L / (n - 1)
    x = np.linspace(-L, L, n)
    Y, X = np.meshgrid(x, x, indexing="ij")
    sig = 0.2
    u = (np.exp(-((X - 3) ** 2 + (Y - 3) ** 2) / 4 / sig / sig) * np.exp(-1j * (X + Y))
         + np.exp(-((X + 3) ** 2 + (Y + 3) ** 2) / 4 / sig / sig) * np.exp(1j * (X + Y))).ravel()
    u = u / np.sqrt(np.sum(np.abs(u) ** 2) * dx * dx)
    g = oracle_py.grid(2, n, n, 1, dx, dx)
    t0 = time.perf_counter()
    oracle_py.nlse_steps(g, u, T / nt, nt - 1, m)
    el = time.perf_counter() - t0
    return {"workload": f"C1: 2D cubic NLSE 256^2, T = {T}, nt = 500 (dt = {T / nt:g}), 499 steps, m = 10"
                        + (" (BASELINE.json C1)" if T == 0.5 else " (nlse_driver.cpp:35-40 defaults)"),
            "seconds": el, "value": n * n * (nt - 1) / el / 1e6, "unit": "Mcells*steps/s",
            "cores": nthr}


def _cpu_sample(args, oracle_py):
    w = dict(WORKLOADS[args.workload])
    if w.get("sewi"):
        ns, steps = 48, 3
        w["n"] = ns
        dx = 2 * w["L"] / (ns - 1)
        u = synthetic_ic(w, 0, ns)
        mf, cf = g2_coefficients(ns, w["L"], 0, ns)
        g = oracle_py.grid(3, ns, ns, ns, dx, dx)
        u1, up1 = oracle_py.nlse_sewi_steps(g, cf, mf, u, None, w["dt"], 1, 1, w["m"])  # step 1 (SS2)
        t0 = time.perf_counter()
        oracle_py.nlse_sewi_steps(g, cf, mf, u1, up1, w["dt"], 2, steps, w["m"])
        el = time.perf_counter() - t0
        cells = ns ** 3
        sample = f"G2 3D sEWI {ns}^3 m={w['m']}, {steps} sEWI steps + BC (sub-grid of the workload, 1 thread)"
    elif w["eq"] == 4:
        ns, steps = 64, 3
        w["n"] = ns
        dx = 2 * w["L"] / (ns - 1)
        u = synthetic_ic(w, 0, ns)
        mf, cf = g2_coefficients(ns, w["L"], 0, ns)
        g = oracle_py.grid(3, ns, ns, ns, dx, dx)
        t0 = time.perf_counter()
        oracle_py.kg_steps(g, cf, mf, u, u.copy(), w["dt"], steps, w["m"])
        el = time.perf_counter() - t0
        cells = ns ** 3
        sample = f"G2 3D Klein-Gordon {ns}^3 m={w['m']}, {steps} Gautschi steps + BC (sub-grid, 1 thread)"
    elif w["eq"] == 3:
        ns, steps = 64, 3
        w["n"] = ns
        dx = 2 * w["L"] / (ns - 1)
        u = synthetic_ic(w, 0, ns)
        mf, cf = g2_coefficients(ns, w["L"], 0, ns)
        g = oracle_py.grid(3, ns, ns, ns, dx, dx)
        oracle_py.nlse_g2_steps(g, cf, mf, u, w["dt"], 1, w["m"])  # warm caches
        t0 = time.perf_counter()
        oracle_py.nlse_g2_steps(g, cf, mf, u, w["dt"], steps, w["m"])
        el = time.perf_counter() - t0
        cells = ns ** 3
        sample = f"G2 3D NLSE {ns}^3 m={w['m']}, {steps} steps + BC (sub-grid of the workload, 1 thread)"
    elif w["eq"] == 2:
        ns, steps = 256, 3
        w["n"] = ns
        dx = 2 * w["L"] / (ns - 1)
        u = synthetic_ic(w, 0, ns)
        g = oracle_py.grid(2, ns, ns, 1, dx, dx)
        up = u.copy()
        mf = -np.ones_like(u)
        t0 = time.perf_counter()
        oracle_py.sg_steps(g, u, up, mf, w["dt"], steps, w["m"])
        el = time.perf_counter() - t0
        cells = ns * ns
        sample = f"2D sine-Gordon {ns}^2 m={w['m']}, {steps} Gautschi steps (sub-grid of the workload, 1 thread)"
    else:
        ns = 128 if w["dim"] == 3 else 1024
        steps = args.cpu_steps
        w["n"] = ns
        dx = 2 * w["L"] / (ns - 1)
        u = synthetic_ic(w, 0, ns)
        g = oracle_py.grid(w["dim"], ns, ns, ns, dx, dx)
        oracle_py.nlse_steps(g, u, w["dt"], 1, w["m"], nonlin=w["eq"])  # warm caches
        t0 = time.perf_counter()
        oracle_py.nlse_steps(g, u, w["dt"], steps, w["m"], nonlin=w["eq"])
        el = time.perf_counter() - t0
        cells = ns ** w["dim"]
        sample = (f"{w['dim']}D {'cubic' if w['eq'] == 0 else 'cubic-quintic'} NLSE {ns}^{w['dim']} "
                  f"m={w['m']}, {steps} SS2 steps (sub-grid of the workload, oracle/ C++ -O2, 1 thread)")
    return {"value": cells * steps / el / 1e6, "unit": "Mcells*steps/s", "cores": 1,
            "kind": "port", "sample": sample, "seconds": el}


def load_traffic(workload, m, kernel_prefix):
    """HBM bytes per launch of the dominant kernel from the committed PMC summary
    (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, gfx950 read-side x2 correction): the
    summary's per-kernel entry whose name starts with kernel_prefix (a k_p2d<J, ...>
    pass or the k_tail), taken on the same workload and m; None otherwise."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("m") != m:
            return None
        for name, e in d.get("kernels", {}).items():
            if name.startswith(kernel_prefix):
                return e["read_bytes"] + e["write_bytes"]
        return None
    except Exception:
        return None


def _build_record(nls_amd):
    info = nls_amd.build_info()
    now = nls_amd.sources_sha256()
    return {"lib_src_sha256": info.get("src_sha256"), "sources_sha256": now,
            "lib_matches_sources": bool(now) and info.get("src_sha256") == now,
            "built": info.get("built"), "compiler": info.get("compiler")}


def _claim_stdout():
    """The contract's stdout is ONE JSON line, but native libraries print there too
    (RCCL's version banner at communicator init): route fd 1 to stderr for the run and
    return a writer on the original stdout for the result line."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(saved, "w")


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def rank_launch_cmd(n: int, argv, port: int):
    """The command `python bench.py --gpus N ...` runs when started without
    torch.distributed.run: the same launcher line the driver uses, one rank per GPU."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(n: int, argv):
    """Run the N ranks as children; return (exit code, rank 0's JSON line or None).
    Children's stderr passes through; their stdout (only rank 0 prints, one line)
    is scanned for the result line."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    p = subprocess.run(rank_launch_cmd(n, argv, free_port()), stdout=subprocess.PIPE, env=env, text=True)
    line = None
    for ln in p.stdout.splitlines():
        ln = ln.strip()
        if ln.startswith("{") and '"metric"' in ln:
            line = ln
        elif ln:
            print(ln, file=sys.stderr)
    return p.returncode, line


# ---- N > 1: the run validates its own multi-GPU path before timing ----
#
# Rank 0 starts, before any rank touches a GPU, a child job on the same N GPUs (the same
# launcher line, its own rendezvous port) that
#   * checks the N-rank field against a 1-rank run on rank 0's GPU (64^3 cubic NLSE, m = 16,
#     SELFCHECK_STEPS SS2 steps; rel-L2 <= SELFCHECK_TOL) and that the library's
#     communicator counts N ranks (ncclCommCount, nls_comm_size), once over the default
#     exchange (RCCL send/recv + all-reduce) and once with NLS_PEER=1 (IPC handshake,
#     peer stores, their ordering by the pass all-reduces and the W_0 halo);
#   * times both exchange paths on the bench workload (SELFCHECK_AB_STEPS steps each,
#     after a warm-up, max over ranks).
# The parent ranks then run the timed region on the exchange the child validated and
# measured faster (the default unless the peer path passed its check AND was faster); the
# child's report goes into the JSON line.  A child that faults, hangs (SELFCHECK_TIMEOUT)
# or fails a check leaves the default exchange in place and says so in the line.
SELFCHECK_N, SELFCHECK_M, SELFCHECK_STEPS, SELFCHECK_TOL = 64, 16, 5, 1e-12
SELFCHECK_AB_STEPS, SELFCHECK_TIMEOUT = 5, 420
_LAUNCHER_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                 "ROLE_RANK", "ROLE_NAME", "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def selfcheck_env(env):
    """The child job's environment: the parent's, without the launcher's per-rank
    variables (the child's own torch.distributed.run sets them) and without NLS_PEER."""
    out = {k: v for k, v in env.items()
           if k not in _LAUNCHER_ENV and not k.startswith("TORCHELASTIC_") and k != "NLS_PEER"}
    out.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return out


def selfcheck_cmd(n, args, json_path, port):
    argv = ["--gpus", str(n), "--workload", args.workload, "--selfcheck-json", json_path]
    if args.n:
        argv += ["--n", str(args.n)]
    if args.m:
        argv += ["--m", str(args.m)]
    return rank_launch_cmd(n, argv, port)


def run_selfcheck(n, args):
    """Rank 0 of the parent job: run the child job, return its report (or the failure)."""
    import subprocess
    import tempfile
    t0 = time.perf_counter()
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "selfcheck.json")
        # its own process group: on a timeout the launcher AND its rank processes go
        p = subprocess.Popen(selfcheck_cmd(n, args, path, free_port()), env=selfcheck_env(os.environ),
                             stdout=sys.stderr, stderr=sys.stderr, start_new_session=True)
        try:
            rc = p.wait(timeout=SELFCHECK_TIMEOUT)
        except subprocess.TimeoutExpired:
            import signal
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except OSError:
                pass
            p.wait()
            rc = "timeout"
        rep = None
        if os.path.exists(path):
            with open(path) as f:
                rep = json.load(f)
    if rep is None:
        rep = {"default": {"ok": False}, "peer": {"ok": False}, "error": f"self-check job ended with {rc}"}
    rep["child_rc"] = rc
    rep["seconds"] = time.perf_counter() - t0
    return rep


def choose_exchange(rep):
    """The exchange the timed run uses: the peer stores only when they passed the field
    check, actually ran (not the library's fallback) and were faster in the A/B leg."""
    ab = rep.get("ab") or {}
    peer_ok = bool(rep.get("peer", {}).get("ok")) and rep.get("peer", {}).get("state") == "active"
    if peer_ok and ab.get("peer_ms") and ab.get("default_ms") and ab["peer_ms"] < ab["default_ms"]:
        return "peer"
    return "default"


def gather_slabs(local, dist, world, rank):
    """Rank 0: the ranks' slabs concatenated in rank order (None elsewhere)."""
    parts = [None] * world
    dist.all_gather_object(parts, np.ascontiguousarray(local))
    return np.concatenate(parts) if rank == 0 else None


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def _bcast(obj, dist, rank):
    o = [obj if rank == 0 else None]
    dist.broadcast_object_list(o, src=0)
    return o[0]


def _selfcheck_field(nls_amd, dist, world, rank, local_rank, peer):
    """One leg of the field check (see above); the report (rank 0's, broadcast)."""
    n, m, dt = SELFCHECK_N, SELFCHECK_M, 1e-3
    w = dict(WORKLOADS["nlse3d_512"], n=n)
    dx = 2 * w["L"] / (n - 1)
    os.environ.pop("NLS_PEER", None)
    if peer:
        os.environ["NLS_PEER"] = "1"
    rep = {"grid": [n] * 3, "krylov_m": m, "steps": SELFCHECK_STEPS, "tol": SELFCHECK_TOL}
    try:
        rid = _bcast(nls_amd.rccl_unique_id() if rank == 0 else None, dist, rank)
        s = nls_amd.Solver(3, n, n, n, dx, dx, m=m, device=local_rank, nranks=world, rank=rank, rccl_id=rid)
        cnt, tr = s.comm_size()
        u = synthetic_ic(w, s.z0, s.nzl)
        s.set_field(u)
        s.step(dt, SELFCHECK_STEPS)
        f = s.get_field()
        state = s.peer_state()
        s.close()
    finally:
        os.environ.pop("NLS_PEER", None)
    full = gather_slabs(f, dist, world, rank)
    counts = [None] * world
    dist.all_gather_object(counts, (cnt, tr, state))
    if rank == 0:
        with nls_amd.Solver(3, n, n, n, dx, dx, m=m, device=local_rank) as s1:
            s1.set_field(synthetic_ic(w, 0, n))
            s1.step(dt, SELFCHECK_STEPS)
            ref = s1.get_field()
        err = rel_l2(full, ref)
        rep.update(comm_count=[c[0] for c in counts], transport=counts[0][1], state=counts[0][2],
                   states=[c[2] for c in counts], rel_l2_vs_1rank=err,
                   ok=bool(all(c[0] == world for c in counts) and err <= SELFCHECK_TOL))
    return _bcast(rep, dist, rank)


def _selfcheck_ab(nls_amd, dist, world, rank, local_rank, w, peer):
    """ms per step of the bench workload over one exchange path (max over ranks)."""
    n = w["n"]
    dx = 2 * w["L"] / (n - 1)
    os.environ.pop("NLS_PEER", None)
    if peer:
        os.environ["NLS_PEER"] = "1"
    try:
        rid = _bcast(nls_amd.rccl_unique_id() if rank == 0 else None, dist, rank)
        s = nls_amd.Solver(w["dim"], n, n, n if w["dim"] == 3 else 1, dx, dx, equation=w["eq"], m=w["m"],
                           device=local_rank, nranks=world, rank=rank, rccl_id=rid)
        s.set_field(synthetic_ic(w, s.z0, s.nzl))
        s.step(w["dt"], 2)
        s.sync()
        dist.barrier()
        t0 = time.perf_counter()
        s.step(w["dt"], SELFCHECK_AB_STEPS)
        s.sync()
        el = time.perf_counter() - t0
        state = s.peer_state()
        s.close()
    finally:
        os.environ.pop("NLS_PEER", None)
    return max_over_ranks(el, dist) * 1e3 / SELFCHECK_AB_STEPS, state


def selfcheck_main(args, dist, world, rank, local_rank):
    """The child job (--selfcheck-json): both field checks, the A/B leg, the report."""
    import nls_amd
    rep = {"n_ranks": world}
    if os.environ.get("NLS_BENCH_SELFCHECK_DRY"):
        # launcher-path test on CPU (tests/test_dist_cpu.py): the same gather / compare and
        # report plumbing on a synthetic field, no device
        w = dict(WORKLOADS["nlse3d_512"], n=20)
        z0, nzl = nls_amd.slab_planes(20, world, rank)
        full = gather_slabs(synthetic_ic(w, z0, nzl), dist, world, rank)
        for leg in ("default", "peer"):
            r = {"comm_count": [world] * world, "state": "active" if leg == "peer" else "off"}
            if rank == 0:
                r["rel_l2_vs_1rank"] = rel_l2(full, synthetic_ic(w, 0, 20))
                r["ok"] = r["rel_l2_vs_1rank"] <= SELFCHECK_TOL
            rep[leg] = _bcast(r, dist, rank)
        rep["ab"] = {"default_ms": 2.0, "peer_ms": 1.0, "peer_state": "active"}
    else:
        rep["default"] = _selfcheck_field(nls_amd, dist, world, rank, local_rank, False)
        try:
            rep["peer"] = _selfcheck_field(nls_amd, dist, world, rank, local_rank, True)
        except Exception as e:  # noqa: BLE001  (a failed peer leg leaves the default)
            rep["peer"] = {"ok": False, "error": repr(e)}
        w = dict(WORKLOADS[args.workload])
        if args.n:
            w["n"] = args.n
        if args.m:
            w["m"] = args.m
        ab = {"steps": SELFCHECK_AB_STEPS}
        ab["default_ms"], _ = _selfcheck_ab(nls_amd, dist, world, rank, local_rank, w, False)
        if rep["peer"].get("ok"):
            ab["peer_ms"], ab["peer_state"] = _selfcheck_ab(nls_amd, dist, world, rank, local_rank, w, True)
        rep["ab"] = ab
    if rank == 0:
        with open(args.selfcheck_json, "w") as f:
            json.dump(rep, f)
    dist.barrier()


def main():
    out = _claim_stdout()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="nlse3d_512", choices=sorted(WORKLOADS))
    ap.add_argument("--n", type=int, default=None, help="override grid side (testing only)")
    ap.add_argument("--m", type=int, default=None, help="override Krylov dim (testing only)")
    ap.add_argument("--cpu-steps", type=int, default=10)
    ap.add_argument("--prof-steps", type=int, default=5,
                    help="steps of the separate per-kernel timing pass (after the timed region)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-full-grid-cpu", action="store_true",
                    help="skip the one-step CPU oracle run at the full 512^3 grid")
    ap.add_argument("--no-selfcheck", action="store_true",
                    help="N > 1: skip the multi-GPU self-check job (default exchange)")
    ap.add_argument("--selfcheck-json", default=None, help=argparse.SUPPRESS)  # the child job
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # not started by torch.distributed.run: start the N ranks ourselves (before
        # anything touches the GPU) and forward rank 0's JSON line
        rc, line = launch_ranks(args.gpus, sys.argv[1:])
        if line:
            print(line, file=out, flush=True)
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        dist.init_process_group("gloo")
    if args.selfcheck_json:
        selfcheck_main(args, dist, world, rank, local_rank)
        dist.destroy_process_group()
        return
    check = None
    if world > 1 and not args.no_selfcheck:
        # before any rank touches a GPU: the child job on the same N GPUs (see run_selfcheck)
        check = _bcast(run_selfcheck(world, args) if rank == 0 else None, dist, rank)
        check["exchange"] = choose_exchange(check)
        if check["exchange"] == "peer":
            os.environ["NLS_PEER"] = "1"

    import nls_amd

    w = dict(WORKLOADS[args.workload])
    if args.n:
        w["n"] = args.n
    if args.m:
        w["m"] = args.m
    n, dim, m = w["n"], w["dim"], w["m"]
    dx = 2 * w["L"] / (n - 1)
    rid = None
    if world > 1:
        obj = [nls_amd.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        rid = obj[0]
    s = nls_amd.Solver(dim, n, n, n if dim == 3 else 1, dx, dx, equation=w["eq"], m=m,
                       device=local_rank, nranks=world, rank=rank, rccl_id=rid)
    comm_ranks, comm_transport = s.comm_size()  # what the library's transport reports
    if comm_ranks != world:
        raise SystemExit(f"library communicator has {comm_ranks} ranks, WORLD_SIZE={world}")
    placement = s.placement()  # basis placement probed at creation (nls_placement)
    u = synthetic_ic(w, s.z0, s.nzl)
    if w["eq"] == 2:
        s.set_sg_state(u, u.copy(), -np.ones(u.size))
    elif w["eq"] == 4:  # KG: u0 real part of the synthetic field, v0 = 0
        mf, cf = g2_coefficients(n, w["L"], s.z0, s.nzl)
        s.set_coefficients(mf, cf)
        s.set_sg_state(u, u.copy())
    elif w["eq"] == 3:  # G2 drivers do not normalise u0 (nlse_cubic_driver_3d.cpp:54-65)
        s.set_field(u)
        s.set_coefficients(*g2_coefficients(n, w["L"], s.z0, s.nzl))
    else:
        u /= np.sqrt(global_mass(u, dx ** dim, dist))  # nlse_call.cpp:41-49
        s.set_field(u)
    # the full-grid CPU baseline steps the same initial field (headline workload, 1 rank)
    keep_u = world == 1 and not args.no_cpu_baseline and args.workload == "nlse3d_512" and not args.n
    u_full = u if keep_u else None
    del u
    dt = w["dt"]

    step_no = [0]

    def run(k):
        if w.get("sewi"):  # nlse_cubic_sewi_driver_3d.cpp: step_sewi(i), apply_bc
            for _ in range(k):
                step_no[0] += 1
                s.step_sewi(dt, step_no[0])
                s.apply_bc()
        elif w["eq"] in (3, 4):  # the G2 driver loop: step, then apply_bc (nlse_cubic_driver_3d.cpp:116-119)
            for _ in range(k):
                s.step(dt, 1)
                s.apply_bc()
        else:
            s.step(dt, k)

    if args.warmup:
        run(args.warmup)
    s.sync()
    if dist is not None:
        dist.barrier()
    s.sync()
    t0 = time.perf_counter()
    run(args.steps)   # the timed region: no per-launch events
    s.sync()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    el = max_over_ranks(el, dist)
    # per-kernel times (roofline) from a separate, untimed pass with HIP events
    # around every launch on the solver's own streams
    s.reset_timing()
    s.set_timing(True)
    run(max(1, args.prof_steps))
    s.sync()
    tm = s.timing()
    s.set_timing(False)
    cells_total = n ** dim
    value = cells_total * args.steps / el / 1e6
    n_local = s.n_local

    # dominant kernel: the fused final pass k_final_fused<m> when the step uses it
    # (NLSE, m >= 3: W_0..W_{m-2} read, u and the next W_0 written, + m(x) on G2),
    # else the largest update pass k_update<J = m-2> (J+1 reads + 1 write); with
    # the two-vector passes (update launches at even J only) the longer of the
    # tail and the largest pass k_p2d<J> (J+1 reads + 2 writes)
    esz = 8 if w["eq"] in (2, 4) else 16
    fcnt = tm["class_count"].get("final", 0)
    ucnt = tm["update_count"]
    # s-step passes (k_p2d / k_p3d): update launches only at the schedule's pass
    # starts J (never at J = 1); pass J writes S_{J+1} .. S_{J+ns}, the last one S_{m-2}
    pass2 = m >= 4 and ucnt[0] > 0 and ucnt[1] == 0
    sched = []
    if pass2:
        Js = [j for j in range(m - 1) if ucnt[j]]
        sched = [(j, (Js[i + 1] if i + 1 < len(Js) else m - 2) - j) for i, j in enumerate(Js)]
    pass_ms = {j: tm["update_ms"][j] / ucnt[j] for j, _ in sched}
    p2J, p2ns = max(sched, key=lambda e: pass_ms[e[0]]) if sched else (0, 0)
    p2_ms = pass_ms.get(p2J, 0.0)
    tail_ms = tm["class_ms"]["final"] / fcnt if fcnt else 0.0
    own_bytes = None
    # the NLSE tail writes u = N(y) only on the last step of an nls_step call (the
    # others write just the next start vector): one call per run() for the G1 NLSE
    multi = w["eq"] in (0, 1) and not w.get("sewi")
    u_frac = (1.0 / args.steps) if multi else 1.0           # timed region
    u_frac_prof = (1.0 / max(1, args.prof_steps)) if multi else 1.0  # timing pass
    own_bytes = moved_bytes_per_cell_step(w, m, sched, pass2, u_frac, tm, args.steps)
    # the NLSE's dominant kernel is the fused tail (the most bytes per launch: m-1 reads,
    # the next start vector and u; the largest pass takes about as long, so a timing
    # rule would flip between runs), else the largest two-vector pass
    nlse_tail = bool(fcnt) and w["eq"] in (0, 1, 3) and not w.get("sewi")
    if pass2 and not nlse_tail:
        J = p2J
        cnt = ucnt[J]
        avg_ms = p2_ms
        bytes_launch = (J + 1 + p2ns) * esz * n_local
        kname = f"k_p{max(p2ns, 2)}d<J={J}> ({p2ns}-vector Lanczos pass: radius-{p2ns} stencil + CGS " \
                f"coefficients, {J + 1} reads + {p2ns} writes)"
        kprefix = f"k_p{max(p2ns, 2)}d<{J}, "
    elif fcnt and w["eq"] in (0, 1, 3) and not w.get("sewi"):
        J = m - 2
        cnt = fcnt
        avg_ms = tm["class_ms"]["final"] / fcnt
        bytes_launch = ((m + u_frac_prof) * esz + (8 if w["eq"] == 3 else 0)) * n_local
        kname = f"k_tail<NLSE, M={m}> (fused tail: stencil + last Lanczos vector + combination " \
                f"+ N(1/2) x2, {m - 1} reads + the next start vector + u on a call's last step)"
        kprefix = "k_tail<"
    else:  # the largest update pass that ran (m-3 where the basis ends in a fused tail)
        J = max([j for j, c in enumerate(tm["update_count"]) if c] or [0])
        cnt = tm["update_count"][J]
        avg_ms = tm["update_ms"][J] / cnt if cnt else float("nan")
        bytes_launch = (J + 2) * esz * n_local
        kname = f"k_update<J={J}> (stencil + CGS + write, {J + 1} reads + 1 write)"
        kprefix = None  # (no per-J PMC entry is matched for the one-vector passes)
    achieved = bytes_launch / (avg_ms * 1e-3) / 1e9 if cnt else None
    traffic = load_traffic(args.workload, m, kprefix) if world == 1 and kprefix else None
    step_bytes = algorithmic_bytes_per_cell_step(m, w["eq"], w.get("sewi", False)) * n_local
    step_ms = el * 1e3 / args.steps
    result = {
        "metric": "Mcells*steps/s and achieved HBM GB/s, 3D NLSE 512^3 at 1/2/4/8 MI355X"
        if args.workload == "nlse3d_512" else f"Mcells*steps/s ({w['desc']})",
        "value": value,
        "unit": "Mcells*steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": step_ms,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64" if w["eq"] in (2, 4) else "c128 (fp64 complex)",
        "data": "synthetic (8 random Gaussian solitons + 1e-3 complex white noise, seeded)",
        "config": {"workload": w["desc"], "grid": [n] * dim, "krylov_m": m, "dt": dt,
                   "equation": ["nlse_cubic", "nlse_cq", "sg_gautschi", "nlse_g2", "kg_gautschi"][w["eq"]]
                   + ("_sewi" if w.get("sewi") else ""),
                   "parallelism": f"z-slab x{world}" if world > 1 else "single GPU",
                   "ranks": {"world": world, "transport": comm_transport,
                             "library_comm_ranks": comm_ranks, "slab_planes_rank0": int(s.nzl)}},
        "roofline": {
            "bound": "hbm",
            "kernel": kname,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
            "traffic": traffic,
            "bytes_per_launch": bytes_launch,
            "avg_launch_ms": avg_ms,
            "timed_in": f"separate {max(1, args.prof_steps)}-step pass with HIP events (not the timed region)",
        },
        "step_roofline": {
            # bytes per cell and step that THIS implementation moves (model of its
            # passes), and the rate they move at over the step
            "moved_bytes_per_cell_step": own_bytes,
            "moved_GBs": own_bytes * n_local / (step_ms * 1e-3) / 1e9 if own_bytes else None,
            "frac": own_bytes * n_local / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if own_bytes else None,
            # the reference algorithm's bytes (one vector per Lanczos
            # iteration, MGS re-reads): an equivalent rate, above the HBM peak once the
            # passes move fewer bytes than that model -- not a bandwidth
            "reference_model_bytes_per_cell_step": algorithmic_bytes_per_cell_step(m, w["eq"],
                                                                                    w.get("sewi", False)),
            "reference_model_equiv_GBs": step_bytes / (step_ms * 1e-3) / 1e9,
            "gpu_kernel_ms_per_step": {k: v / max(tm["steps"], 1) for k, v in tm["class_ms"].items()},
            "lanczos": ("s-step passes " + " ".join(f"J{j}:{ns}" for j, ns in sched) + " + fused tail")
            if pass2 else "one-vector passes + fused tail",
            "bases_per_step": 2 if w["eq"] in (2, 4) else (3 if w.get("sewi") else 1),
        },
        # the basis allocation kept among the candidates probed at nls_create (DESIGN.md
        # section 4 "Placement"; candidates 0: no probe on this handle)
        "placement": placement,
        # build provenance: the library's compiled-in source hash against the sources shipped
        # beside it (a prebuilt libnls_amd.so that does not match them says so here)
        "build": _build_record(nls_amd),
    }
    if world > 1:
        # the self-check job's report and the exchange this timed run used (peer_state of
        # this handle: "active" = peer stores, "off" = RCCL send/recv exchange)
        result["multi_gpu_check"] = check
        result["config"]["exchange"] = {"used": s.peer_state(), "chosen": (check or {}).get("exchange", "default")}
    gpu_one = None
    if u_full is not None and not args.no_full_grid_cpu:
        # the full-size parity check of the CPU baseline's step (after the timed region)
        s.set_field(u_full)
        s.step(dt, 1)
        gpu_one = s.get_field()
    s.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, u_full, gpu_one)
    if rank == 0:
        print(json.dumps(result), file=out, flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
