"""Golden fixtures computed by the REFERENCE'S OWN executable Python (build container only).

Two pieces of the hot path exist in the reference as runnable Python:

* ``LanczosStepTorch.forward`` (/root/reference/nlsolvers/fusing_kernels.py:8-45) --
  one complex128 Lanczos iteration of the G1 device recurrence
  (device/lanczos_complex.hpp:413-500): fresh dot T(j-1, j) = V[j-1]^H buf1, alpha,
  one classical Gram-Schmidt sweep over V[0..j], beta = ||.|| with the ``> 0`` guard,
  the T writes and the normalisation;
* ``neumann_bc`` (/root/reference/nlsolvers/device/include/bc_kernel_generation_test/
  bc_update_kernel_fusion.py:18-27) -- the 2D Neumann copy boundary condition,
  the same copy sequence as boundaries.cuh:10-19.

This script loads both modules from the read-only reference tree with importlib (no
copy of their source is kept anywhere in this repository), drives them on CPU tensors
and writes their outputs as plain ``.npz`` data:

* ``ref_lanczos_{2d,3d}_{smooth,noise}.npz``: u, the operator's grid (G1 5-/7-point
  Laplacian, laplacians.hpp:10-105, applied as the literal triplet-builder
  transcription ``np_ref.laplacian_triplets`` -- buf1 = L V[j] as the reference's
  caller forms it), and for m = 10 and m = 16: T (m x m), beta per iteration and
  beta0 = ||u||; the basis V of the m = 16 run (the m = 10 basis is its first 10
  rows bit for bit, asserted below);
* ``ref_bc2d.npz``: the BC applied to complex and real 2D fields, square and
  non-square.

The fixtures are DATA (inputs and the reference's outputs); the reference's Python
never travels to the GPU box.  tests/test_oracle.py pins the oracle's Lanczos, its
Krylov action and its BC against them; tests/test_gpu_refpin.py pins the GPU.

Run (build container, where /root/reference exists):
    python tests/golden/make_ref_fixtures.py
"""
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import np_ref  # noqa: E402

REF = "/root/reference/nlsolvers"


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


def main():
    import torch

    fk = load("ref_fusing_kernels", os.path.join(REF, "fusing_kernels.py"))
    bcm = load("ref_bc_update_kernel_fusion",
               os.path.join(REF, "device/include/bc_kernel_generation_test/bc_update_kernel_fusion.py"))
    step = fk.LanczosStepTorch().cpu()
    for dim, n in ((2, 32), (3, 16)):
        dx = 20.0 / (n - 1)  # nlse_call.cpp:35 with L = 10
        A = np_ref.laplacian_triplets(dim, n, dx)
        for kind, seed in (("smooth", 11), ("noise", 12)):
            u = field(dim, n, kind, seed + dim)
            out = dict(dim=dim, n=n, dx=dx, u=u)
            for m in (10, 16):
                V, T, betas, beta0 = run_lanczos(step, torch, A, u, m)
                out[f"T{m}"] = T
                out[f"beta{m}"] = betas
                out["beta0"] = beta0
                if m == 16:
                    out["V16"] = V
                else:
                    V10 = V
            assert np.array_equal(V10, out["V16"][:10])
            np.savez_compressed(os.path.join(HERE, f"ref_lanczos_{dim}d_{kind}.npz"), **out)
            print(f"ref_lanczos_{dim}d_{kind}: n={n}^{dim}, beta16[:3]={out['beta16'][:3]}")
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


if __name__ == "__main__":
    main()
