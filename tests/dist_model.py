"""CPU model of the multi-GPU slab decomposition over torch.distributed (gloo).

TEST INFRASTRUCTURE.  It restates, per rank and in numpy, exactly the data
movement the library performs on N GPUs (nonlinear-solvers_amd/csrc/nls_api.cpp):

  * the slab of planes each rank owns comes from the library's own
    nls_slab_planes() (3D: z-planes, 2D: y-rows);
  * every vector is stored with one ghost plane below and above; after a new
    Krylov vector is produced, its first/last local planes are exchanged with
    the neighbouring ranks (the library's ncclSend/ncclRecv pair) -- one plane
    also carries the 3D flat-index "y-wrap" coupling (i, ny-1, k) <-> (i, 0, k+1)
    (laplacians.hpp:89-92), which crosses slab boundaries;
  * every inner product is a local partial sum followed by an all-reduce
    (the library's ncclAllReduce of the packed dot vector), after which all
    ranks do identical small-matrix work (eigensolve, f(T)) without a broadcast.

The Lanczos/SS2 arithmetic follows the oracle (eigen_krylov_complex.hpp:10-84,
nlse_solver.hpp:53-77); tests/test_dist_cpu.py runs it with world_size 2 and 3
on CPU and checks the gathered field against the single-process oracle.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "nonlinear-solvers_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


class Slab:
    def __init__(self, dim, nx, ny, nz, dx, dy, rank, world):
        import nls_amd
        self.dim, self.nx, self.ny, self.nz = dim, nx, ny, nz
        self.P = nx * ny if dim == 3 else nx
        self.npl = nz if dim == 3 else ny
        self.z0, self.nzl = nls_amd.slab_planes(self.npl, world, rank)
        self.rank, self.world = rank, world
        self.s = 1.0 / (dx * dx) if dim == 3 else 1.0 / (dx * dy)
        self.N = self.P * self.npl

    def ext(self, local):
        """local (nzl*P,) -> extended (nzl+2, P) with zero ghost planes + halo exchange."""
        v = np.zeros((self.nzl + 2, self.P), dtype=local.dtype)
        v[1:-1] = local.reshape(self.nzl, self.P)
        self.halo(v)
        return v

    def halo(self, v):
        import torch
        import torch.distributed as dist
        reqs = []
        cplx = np.iscomplexobj(v)
        def t(a):
            a = np.ascontiguousarray(a)
            return torch.from_numpy(a.view(np.float64) if cplx else a)
        bufs = {}
        if self.rank > 0:
            reqs.append(dist.isend(t(v[1]), self.rank - 1))
            bufs["below"] = torch.empty(self.P * (2 if cplx else 1), dtype=torch.float64)
            reqs.append(dist.irecv(bufs["below"], self.rank - 1))
        if self.rank < self.world - 1:
            reqs.append(dist.isend(t(v[-2]), self.rank + 1))
            bufs["above"] = torch.empty(self.P * (2 if cplx else 1), dtype=torch.float64)
            reqs.append(dist.irecv(bufs["above"], self.rank + 1))
        for r in reqs:
            r.wait()
        conv = (lambda b: b.numpy().view(np.complex128)) if cplx else (lambda b: b.numpy())
        if "below" in bufs:
            v[0] = conv(bufs["below"])
        if "above" in bufs:
            v[-1] = conv(bufs["above"])

    def lap(self, v):
        """Isotropic no-flux operator on the local planes of the extended slab v
        (flat-index neighbours with the global range tests of laplacians.hpp:10-105)."""
        P, nx, s = self.P, self.nx, self.s
        n = self.nzl * P
        flat = v.ravel()
        loc = np.arange(n) + P                 # positions of the local cells in flat
        g = np.arange(n) + self.z0 * P         # global flat index
        i = g % nx
        cur = flat[loc]
        if self.dim == 3:
            j = (g // nx) % self.ny
            k = g // P
            bd = (i == 0) | (i == nx - 1) | (j == 0) | (j == self.ny - 1) | (k == 0) | (k == self.nz - 1)
            d = np.where(bd, -5.0, -6.0)
        else:
            k = g // P
            bd = (i == 0) | (i == nx - 1) | (k == 0) | (k == self.npl - 1)
            d = np.where(bd, -3.0, -4.0)
        out = (d * s) * cur
        out = out + np.where(i > 0, s * flat[loc - 1], 0)
        out = out + np.where(i < nx - 1, s * flat[np.minimum(loc + 1, flat.size - 1)], 0)
        if self.dim == 3:
            out = out + np.where(g >= nx, s * flat[loc - nx], 0)
            out = out + np.where(g + nx < self.N, s * flat[np.minimum(loc + nx, flat.size - 1)], 0)
            out = out + np.where(g >= P, s * flat[loc - P], 0)
            out = out + np.where(g + P < self.N, s * flat[np.minimum(loc + P, flat.size - 1)], 0)
        else:
            out = out + np.where(g >= P, s * flat[loc - P], 0)
            out = out + np.where(g + P < self.N, s * flat[np.minimum(loc + P, flat.size - 1)], 0)
        return out

    def allsum(self, vals):
        import torch
        import torch.distributed as dist
        a = np.asarray(vals, dtype=np.complex128)
        t = torch.from_numpy(np.ascontiguousarray(a).view(np.float64).copy())
        dist.all_reduce(t)
        return t.numpy().view(np.complex128)


def krylov_dist(sl: Slab, u_loc, t, m, func_exp_abs=True):
    """Distributed restatement of expm_multiply (eigen_krylov_complex.hpp:55-84):
    MGS Lanczos with all-reduced dots, identical eigensolve on every rank."""
    n = u_loc.size
    V = np.zeros((m, n), dtype=np.complex128)
    T = np.zeros((m, m), dtype=np.complex128)
    beta = np.sqrt(sl.allsum([np.vdot(u_loc, u_loc)])[0].real)
    V[0] = u_loc / beta
    for j in range(m - 1):
        w = sl.lap(sl.ext(V[j]))
        if j > 0:
            w = w - T[j - 1, j] * V[j - 1]
        T[j, j] = sl.allsum([np.vdot(V[j], w)])[0]
        w = w - T[j, j] * V[j]
        for i in range(j + 1):
            c = sl.allsum([np.vdot(V[i], w)])[0]
            w = w - c * V[i]
        nb = np.sqrt(sl.allsum([np.vdot(w, w)])[0].real)
        T[j + 1, j] = T[j, j + 1] = nb
        V[j + 1] = w / nb
    A = np.tril(T.real)
    A = A + np.tril(A, -1).T
    lam, Q = np.linalg.eigh(A)
    f = np.exp(t * (np.abs(lam) if func_exp_abs else lam))
    c = Q @ (f * Q[0, :])
    return beta * (c @ V)


def nlse_steps_dist(sl: Slab, u_loc, dt, nsteps, m):
    """NLSESolver::step (nlse_solver.hpp:53-77) on the slab, tau = 1j*dt."""
    u = u_loc.astype(np.complex128).copy()
    half = lambda v: np.exp(-0.5j * dt * (v.real * v.real + v.imag * v.imag)) * v
    for _ in range(nsteps):
        u = half(krylov_dist(sl, half(u), -1j * dt, m))
    return u


def gather(sl: Slab, local):
    """All slabs to rank 0 (in rank order); None elsewhere."""
    import torch
    import torch.distributed as dist
    cplx = np.iscomplexobj(local)
    a = np.ascontiguousarray(local)
    t = torch.from_numpy(a.view(np.float64) if cplx else a)
    sizes = [None] * sl.world
    dist.all_gather_object(sizes, int(t.numel()))
    if sl.rank == 0:
        parts = [t]
        for r in range(1, sl.world):
            b = torch.empty(sizes[r], dtype=torch.float64)
            dist.recv(b, r)
            parts.append(b)
        out = torch.cat(parts).numpy()
        return out.view(np.complex128) if cplx else out
    dist.send(t, 0)
    return None
