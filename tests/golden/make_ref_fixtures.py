"""Golden fixtures computed by the REFERENCE'S OWN executable Python (build container only).

Two pieces of the hot path exist in the reference as runnable Python:

* ``LanczosStepTorch.forward`` (/root/reference/nlsolvers/fusing_kernels.py:8-45) --
  one complex128 Lanczos iteration of the G1 device recurrence
  (device/lanczos_complex.hpp:413-500): fresh dot T(j-1, j) = V[j-1]^H buf1, alpha,
  one classical Gram-Schmidt sweep over V[0..j], beta = ||.|| with the ``> 0`` guard,
  the T writes and the normalisation.  Driven on REAL-valued complex128 data (imaginary
  parts exactly 0, which every vdot / axpy / norm keeps exactly 0) it is the real
  recurrence of device/lanczos.hpp:126-194 and eigen_krylov_real.hpp:5-51 bit for bit
  in the real parts (asserted below: the imaginary parts stay exactly 0);
* ``neumann_bc`` (/root/reference/nlsolvers/device/include/bc_kernel_generation_test/
  bc_update_kernel_fusion.py:18-27) -- the 2D Neumann copy boundary condition,
  the same copy sequence as boundaries.cuh:10-19.

Trust boundary.  The reference tree is untrusted third-party code.  This script
imports exactly those two modules with importlib (module-level side effects included:
fusing_kernels.py imports triton and sets torch debug flags in THIS process only), in
the build container, never on the GPU box and never from a test; nothing the tests or
the product load executes reference code.  The sha256 of both source files is recorded
in ``ref_sources.json`` next to the fixtures, so a regenerated fixture set can be tied
to the exact reference text it came from.  Run it in a throwaway process (it is one).

Fixtures written (DATA only: inputs and the reference's outputs; no reference source is
kept anywhere in this repository):

* ``ref_lanczos_{2d,3d}_{smooth,noise}.npz`` (complex, G1 spacing dx = 20/(n-1) on the
  32^2 / 16^3 grids): u, the grid, and for m = 10 and 16: T (m x m), beta per
  iteration, beta0 = ||u||; the basis V of the m = 16 run (the m = 10 basis is its
  first 10 rows bit for bit, asserted below).  buf1 = L V[j] is formed as the
  reference's caller forms it, with the literal triplet-builder transcription
  ``np_ref.laplacian_triplets`` of laplacians.hpp:10-105;
* ``ref_lanczos_{2d,3d}_{smooth,noise}_real.npz``: the same on real fields (the real
  part of the complex IC), stored as float64;
* ``ref_lanczos_{2d,3d}_noise{,_real}_{hl,c2,c4}.npz``: the noise fields on the same
  grids at the spacings the BASELINE workloads run: hl = 20/511 (3D 512^3 headline,
  ||L|| dt ~ 7.8 at dt = 1e-3), c2 = 20/4095 (2D 4096^2, ||L|| dt ~ 335), c4 = 6/8191
  (sine-Gordon 8192^2, t sqrt||L|| ~ 39 at dt = 0.01);
* ``ref_bc2d.npz``: the BC applied to complex and real 2D fields, square and
  non-square.

tests/test_oracle.py pins the oracle's Lanczos, its Krylov actions (complex exp
conventions; real cos / sinc / sinc^2 / id / sinc^2-half of t sqrt|lambda|) and its BC
against them; tests/test_gpu_refpin.py pins the GPU (also on the bench's large-slab
launch shapes, NLS_LARGE_SLAB=1).

Run (build container, where /root/reference exists):
    python tests/golden/make_ref_fixtures.py
"""
import hashlib
import importlib.util
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import np_ref  # noqa: E402

REF = "/root/reference/nlsolvers"
SRC_LANCZOS = os.path.join(REF, "fusing_kernels.py")
SRC_BC = os.path.join(REF, "device/include/bc_kernel_generation_test/bc_update_kernel_fusion.py")

# spacings of the BASELINE workloads (nlse_call.cpp:35 dx = 2 Lx / (nx - 1); SG L = 3)
SPACINGS = {"hl": 20.0 / 511, "c2": 20.0 / 4095, "c4": 6.0 / 8191}


def load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def field(dim, n, kind, seed):
    """Smooth: two Gaussian solitons with a phase + 1e-3 noise (the bench's IC family);
    noise: complex white noise (every eigen-direction of L excited)."""
    rng = np.random.default_rng(seed)
    N = n ** dim
    if kind == "noise":
        return rng.standard_normal(N) + 1j * rng.standard_normal(N)
    x = np.linspace(-10.0, 10.0, n)
    g = np.meshgrid(*([x] * dim), indexing="ij")
    X = g[-1]
    r2a = sum(v * v for v in g[:-1]) + (X - 2.0) ** 2
    r2b = sum(v * v for v in g[:-1]) + (X + 3.0) ** 2
    u = np.exp(-r2a / 4) * np.exp(1j * X) + 0.6 / np.cosh(np.sqrt(r2b))
    return u.ravel() + 1e-3 * (rng.standard_normal(N) + 1j * rng.standard_normal(N))


def run_lanczos(step, torch, A, u, m):
    """The reference's iteration driven for j = 0 .. m-2 (m-1 iterations, T(m-1, m-1)
    never written: eigen_krylov_complex.hpp:19 / lanczos_complex.hpp:318-551)."""
    n = u.size
    ut = torch.from_numpy(u.astype(np.complex128))
    beta0 = float(torch.norm(ut))
    V = torch.zeros((m, n), dtype=torch.complex128)
    T = torch.zeros((m, m), dtype=torch.complex128)
    V[0] = ut / beta0
    betas = []
    for j in range(m - 1):
        buf1 = torch.from_numpy(A @ V[j].numpy())
        w, T, beta = step(buf1, V, T, j, m)
        V[j + 1] = w
        betas.append(beta)
    return V.numpy().copy(), T.numpy().copy(), np.array(betas), beta0


def record(step, torch, dim, n, dx, u, real):
    """m = 10 and 16 runs of the reference on u; real=True: u real, stored as f64."""
    A = np_ref.laplacian_triplets(dim, n, dx)
    out = dict(dim=dim, n=n, dx=dx, u=u.real.copy() if real else u)
    uc = u.real.astype(np.complex128) if real else u
    for m in (10, 16):
        V, T, betas, beta0 = run_lanczos(step, torch, A, uc, m)
        if real:  # the recurrence never leaves the real line
            assert not np.any(V.imag) and not np.any(T.imag)
            V, T = V.real.copy(), T.real.copy()
        out[f"T{m}"] = T
        out[f"beta{m}"] = betas
        out["beta0"] = beta0
        if m == 16:
            out["V16"] = V
        else:
            V10 = V
    assert np.array_equal(V10, out["V16"][:10])
    return out


def sha256(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def main():
    import torch

    fk = load("ref_fusing_kernels", SRC_LANCZOS)
    bcm = load("ref_bc_update_kernel_fusion", SRC_BC)
    step = fk.LanczosStepTorch().cpu()
    for dim, n in ((2, 32), (3, 16)):
        dx = 20.0 / (n - 1)  # nlse_call.cpp:35 with L = 10
        for kind, seed in (("smooth", 11), ("noise", 12)):
            u = field(dim, n, kind, seed + dim)
            for real in (False, True):
                name = f"ref_lanczos_{dim}d_{kind}" + ("_real" if real else "")
                out = record(step, torch, dim, n, dx, u, real)
                np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
                print(f"{name}: n={n}^{dim}, beta16[:3]={out['beta16'][:3]}")
            if kind != "noise":
                continue
            for tag, dxs in SPACINGS.items():
                for real in (False, True):
                    name = f"ref_lanczos_{dim}d_noise" + ("_real" if real else "") + f"_{tag}"
                    out = record(step, torch, dim, n, dxs, u, real)
                    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
                    print(f"{name}: dx={dxs:.3e}, beta16[:3]={out['beta16'][:3]}")
    rng = np.random.default_rng(7)
    bc = {}
    for a, b in ((24, 24), (9, 13)):
        uc = rng.standard_normal((a, b)) + 1j * rng.standard_normal((a, b))
        ur = rng.standard_normal((a, b))
        # neumann_bc(u, nx, ny) on a (nx, ny) tensor, in place; C order = our [ny][nx]
        # with the tensor's first axis as rows
        oc = bcm.neumann_bc(torch.from_numpy(uc.copy()), a, b).numpy().copy()
        orr = bcm.neumann_bc(torch.from_numpy(ur.copy()), a, b).numpy().copy()
        bc[f"uc_{a}x{b}"], bc[f"bc_c_{a}x{b}"] = uc, oc
        bc[f"ur_{a}x{b}"], bc[f"bc_r_{a}x{b}"] = ur, orr
    np.savez_compressed(os.path.join(HERE, "ref_bc2d.npz"), **bc)
    print("ref_bc2d: shapes", [k for k in bc if k.startswith("uc_")])
    srcs = {os.path.relpath(p, "/root/reference"): sha256(p) for p in (SRC_LANCZOS, SRC_BC)}
    srcs["torch"] = torch.__version__
    with open(os.path.join(HERE, "ref_sources.json"), "w") as f:
        json.dump(srcs, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
