"""numpy twin of the C oracle -- TEST INFRASTRUCTURE ONLY.

A second, independent restatement of the reference G1 CPU path (vectorised
numpy, ``numpy.linalg.eigh`` instead of the C oracle's Jacobi), used by the
CPU test-suite to pin the C oracle, plus a restatement of the triplet
builders (the operator as an explicit scipy CSR matrix) and of the G2
anisotropic builder used by the reference's scipy known-answer test.

Reference lines followed:
  laplacians.hpp:10-52 / :55-105          build_laplacian_noflux{,_3d}
  nlsolvers/common/include/laplacians.hpp:54-103, 158-218   anisotropic 2D/3D (c-field)
  nlsolvers/device/include/nlse_dev.hpp:187-203, boundaries.cuh:10-81   G2 step + BC
  eigen_krylov_complex.hpp:10-84          lanczos_L + expm_multiply (|lambda|)
  eigen_krylov_real.hpp:5-201             real Lanczos + cos/sinc^2/id filters
  nlse_solver.hpp:53-77                   Strang SS2 step
  sg_solver.hpp:53-74                     Gautschi step
  nlsolvers/device/include/{sg_single,sg_double,sg_hyperbolic,phi4_single}.cuh   G2 Gautschi family
  nlsolvers/common/include/util.hpp:95-125  create_centered_gaussian_3d
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

F_EXP_ABS, F_EXP, F_COS_SQRT, F_SINC_SQRT, F_SINC2_SQRT, F_ID_SQRT, F_SINC2_HALF, F_SINC = range(8)


def _shape(dim, nx, ny, nz):
    return (ny, nx) if dim == 2 else (nz, ny, nx)


def laplacian_triplets(dim: int, n: int, dx: float, dy: float | None = None) -> sp.csr_matrix:
    """Literal transcription of the triplet loops (laplacians.hpp:10-105).

    ``n`` is the full side length (the builders receive ``n - 2``)."""
    dy = dx if dy is None else dy
    if dim == 2:
        N = n * n
        rows, cols, vals = [], [], []
        for i in range(N):
            v = -4.0
            if i < n or i >= N - n or i % n == 0 or i % n == n - 1:
                v = -3.0
            rows.append(i); cols.append(i); vals.append(v)
        for i in range(N - 1):
            if (i + 1) % n != 0:
                rows += [i, i + 1]; cols += [i + 1, i]; vals += [1.0, 1.0]
        for i in range(N - n):
            rows += [i, i + n]; cols += [i + n, i]; vals += [1.0, 1.0]
        scale = 1.0 / (dx * dy)
    else:
        P = n * n
        N = P * n
        rows, cols, vals = [], [], []
        for k in range(n):
            for j in range(n):
                for i in range(n):
                    idx = k * P + j * n + i
                    bd = k in (0, n - 1) or j in (0, n - 1) or i in (0, n - 1)
                    rows.append(idx); cols.append(idx); vals.append(-5.0 if bd else -6.0)
        for i in range(N - 1):
            if (i + 1) % n != 0:
                rows += [i, i + 1]; cols += [i + 1, i]; vals += [1.0, 1.0]
        for i in range(N - n):
            rows += [i, i + n]; cols += [i + n, i]; vals += [1.0, 1.0]
        for i in range(N - P):
            rows += [i, i + P]; cols += [i + P, i]; vals += [1.0, 1.0]
        scale = 1.0 / (dx * dx)
    A = sp.coo_matrix((np.array(vals) * scale, (rows, cols)), shape=(N, N)).tocsr()
    A.sum_duplicates()
    return A


def aniso_laplacian_3d(n: int, dx: float, c: np.ndarray) -> sp.csr_matrix:
    """build_anisotropic_laplacian_noflux_3d (nlsolvers/common/include/laplacians.hpp:158-218)."""
    P = n * n
    N = P * n
    c = np.asarray(c, dtype=np.float64).ravel()
    diag = np.zeros(N)
    r, cc, v = [], [], []
    idx = np.arange(N - 1)
    m = (idx + 1) % n != 0
    i0 = idx[m]
    a = (c[i0] + c[i0 + 1]) / 2.0
    r += [i0, i0 + 1]; cc += [i0 + 1, i0]; v += [a, a]
    np.add.at(diag, i0, a); np.add.at(diag, i0 + 1, a)
    for off in (n, P):
        i0 = np.arange(N - off)
        a = (c[i0] + c[i0 + off]) / 2.0
        r += [i0, i0 + off]; cc += [i0 + off, i0]; v += [a, a]
        np.add.at(diag, i0, a); np.add.at(diag, i0 + off, a)
    r.append(np.arange(N)); cc.append(np.arange(N)); v.append(-diag)
    A = sp.coo_matrix((np.concatenate(v), (np.concatenate(r), np.concatenate(cc))), shape=(N, N)).tocsr()
    A.sum_duplicates()
    return A * (1.0 / (dx * dx))


def aniso_laplacian(dim: int, nx: int, ny: int, nz: int, dx: float, dy: float,
                    c: np.ndarray) -> sp.csr_matrix:
    """build_anisotropic_laplacian_noflux{,_3d} on a general grid
    (nlsolvers/common/include/laplacians.hpp:54-103 for 2D, :158-218 for 3D):
    fast-axis couplings (i, i+1) unless (i+1) % nx == 0, flat (i, i+nx) for
    i < N - nx, and (3D) (i, i+P); weight (c_a + c_b)/2, diagonal -sum."""
    P = nx * ny
    N = P * (nz if dim == 3 else 1)
    c = np.asarray(c, dtype=np.float64).ravel()
    assert c.size == N
    diag = np.zeros(N)
    r, cc, v = [], [], []
    idx = np.arange(N - 1)
    i0 = idx[(idx + 1) % nx != 0]
    a = (c[i0] + c[i0 + 1]) / 2.0
    r += [i0, i0 + 1]; cc += [i0 + 1, i0]; v += [a, a]
    np.add.at(diag, i0, a); np.add.at(diag, i0 + 1, a)
    for off in ((nx, P) if dim == 3 else (nx,)):
        i0 = np.arange(N - off)
        a = (c[i0] + c[i0 + off]) / 2.0
        r += [i0, i0 + off]; cc += [i0 + off, i0]; v += [a, a]
        np.add.at(diag, i0, a); np.add.at(diag, i0 + off, a)
    r.append(np.arange(N)); cc.append(np.arange(N)); v.append(-diag)
    A = sp.coo_matrix((np.concatenate(v), (np.concatenate(r), np.concatenate(cc))), shape=(N, N)).tocsr()
    A.sum_duplicates()
    return A * (1.0 / (dx * dy) if dim == 2 else 1.0 / (dx * dx))


def neumann_bc(dim, nx, ny, nz, u):
    """Neumann copy BC (nlsolvers/device/include/boundaries.cuh:10-81) as the
    clamp gather it amounts to: u[k, j, i] <- u[clamp(k), clamp(j), clamp(i)]
    with every index clamped into [1, n-2]."""
    u = np.asarray(u).reshape(_shape(dim, nx, ny, nz)).copy()
    idx = [np.clip(np.arange(n), 1, n - 2) for n in u.shape]
    return u[np.ix_(*idx)].ravel()


def nlse_g2_steps(dim, nx, ny, nz, dx, dy, c, mfield, u, dt, nsteps, m, bc=True):
    """G2 SS2 (nlsolvers/device/include/nlse_dev.hpp:187-203) + driver BC."""
    A = aniso_laplacian(dim, nx, ny, nz, dx, dy, c)
    mf = np.asarray(mfield, dtype=np.float64).ravel()
    u = np.asarray(u, dtype=np.complex128).ravel().copy()
    N = lambda v: v * np.exp(0.5 * 1j * dt * (mf * (v.real * v.real + v.imag * v.imag)))
    for _ in range(nsteps):
        b = krylov(lambda v: A @ v, N(u), 1j * dt, m, F_EXP)
        u = N(b)
        if bc:
            u = neumann_bc(dim, nx, ny, nz, u)
    return u


def nlse_cq_g2_steps(dim, nx, ny, nz, dx, dy, mfield, u, dt, nsteps, m, s1, s2, bc=True):
    """G2 cubic-quintic (nlsolvers/device/include/nlse_cubic_quintic{.cuh:9-40,_dev.hpp:79-95}):
    rho = m (s1 d + s2 d^2), N = exp(-tau/2 rho), linear exp(-tau lambda) on the
    isotropic operator (laplacians.hpp:10-52), driver BC after every step."""
    A = laplacian_triplets(dim, nx, dx, dy) if (dim == 2 and nx == ny) else None
    mf = np.asarray(mfield, dtype=np.float64).ravel()
    u = np.asarray(u, dtype=np.complex128).ravel().copy()

    def N(v):
        d = v.real * v.real + v.imag * v.imag
        return v * np.exp(-0.5 * 1j * dt * (mf * (s1 * d + s2 * d * d)))
    ap = (lambda v: A @ v) if A is not None else (lambda v: laplacian_apply(dim, nx, ny, nz, dx, dy, v))
    for _ in range(nsteps):
        b = krylov(ap, N(u), -1j * dt, m, F_EXP)
        u = N(b)
        if bc:
            u = neumann_bc(dim, nx, ny, nz, u)
    return u


def nlse_sewi_steps(dim, nx, ny, nz, dx, dy, c, mfield, u, u_prev, dt, first_step, nsteps, m, bc=True):
    """G2 sEWI (nlsolvers/device/include/nlse_dev.hpp:205-238) + driver BC."""
    A = aniso_laplacian(dim, nx, ny, nz, dx, dy, c)
    ap = lambda v: A @ v
    mf = np.asarray(mfield, dtype=np.float64).ravel()
    u = np.asarray(u, dtype=np.complex128).ravel().copy()
    up = u.copy() if u_prev is None else np.asarray(u_prev, dtype=np.complex128).ravel().copy()
    N = lambda v: v * np.exp(0.5 * 1j * dt * (mf * (v.real * v.real + v.imag * v.imag)))
    for s in range(nsteps):
        i = first_step + s
        if i == 1:
            up = u.copy()
            u = N(krylov(ap, N(u), 1j * dt, m, F_EXP))
        else:
            B = -mf * (u.real * u.real + u.imag * u.imag) * u
            e = krylov(ap, krylov(ap, B, dt, m, F_SINC), 1j * dt, m, F_EXP)
            new = krylov(ap, up, 2j * dt, m, F_EXP) - 2j * dt * e
            up = u
            u = new
        if bc:
            u = neumann_bc(dim, nx, ny, nz, u)
    return u, up


def kg_steps(dim, nx, ny, nz, dx, dy, c, mfield, u, u_past, dt, nsteps, m, bc=True):
    """G2 Klein-Gordon Gautschi (kg_single.cuh:49-86) on -div(c grad) + BC."""
    A = -aniso_laplacian(dim, nx, ny, nz, dx, dy, c)
    ap = lambda x: A @ x
    mf = np.asarray(mfield, dtype=np.float64).ravel()
    u = np.asarray(u, dtype=np.float64).ravel().copy()
    up = np.asarray(u_past, dtype=np.float64).ravel().copy()
    v = np.zeros_like(u)
    for _ in range(nsteps):
        c2 = 2.0 * krylov(ap, u, dt, m, F_COS_SQRT)
        s = krylov(ap, -mf * u * u * u, dt, m, F_SINC2_SQRT)
        new = (c2 - up) + s * (dt * dt)
        up = u
        u = new
        v = (u - up) / dt
        if bc:
            u = neumann_bc(dim, nx, ny, nz, u)
    return u, up, v


def laplacian_apply(dim, nx, ny, nz, dx, dy, x):
    """Vectorised matrix-free application (same operator, flat-index form)."""
    x = np.asarray(x).ravel()
    N = x.size
    P = nx * ny
    s = 1.0 / (dx * dy) if dim == 2 else 1.0 / (dx * dx)
    idx = np.arange(N)
    i = idx % nx
    j = (idx // nx) % ny
    bd = (i == 0) | (i == nx - 1) | (j == 0) | (j == ny - 1)
    if dim == 3:
        k = idx // P
        bd |= (k == 0) | (k == nz - 1)
        d = np.where(bd, -5.0, -6.0)
    else:
        d = np.where(bd, -3.0, -4.0)
    y = (d * s) * x
    xm = np.zeros_like(x); xm[1:] = x[:-1]; xm[i == 0] = 0
    xp = np.zeros_like(x); xp[:-1] = x[1:]; xp[i == nx - 1] = 0
    y = y + s * xm + s * xp
    y[nx:] += s * x[:-nx]
    y[:-nx] += s * x[nx:]
    if dim == 3:
        y[P:] += s * x[:-P]
        y[:-P] += s * x[P:]
    return y


def lanczos(apply, u, m):
    """lanczos_L (eigen_krylov_complex.hpp:10-53): MGS, m-1 iterations, T[m-1,m-1]=0."""
    u = np.asarray(u)
    n = u.size
    cplx = np.iscomplexobj(u)
    dt = np.complex128 if cplx else np.float64
    V = np.zeros((n, m), dtype=dt)
    T = np.zeros((m, m), dtype=dt)
    beta = np.linalg.norm(u)
    V[:, 0] = u / beta
    for j in range(m - 1):
        w = apply(V[:, j])
        if j > 0:
            w = w - T[j - 1, j] * V[:, j - 1]
        T[j, j] = np.vdot(V[:, j], w)
        w = w - T[j, j] * V[:, j]
        for i in range(j + 1):
            w = w - np.vdot(V[:, i], w) * V[:, i]
        nb = np.linalg.norm(w)
        T[j + 1, j] = nb
        T[j, j + 1] = nb
        V[:, j + 1] = w / nb
    return V, T, beta


def _f(func, lam, t):
    if func == F_EXP_ABS:
        return np.exp(t * np.abs(lam))
    if func == F_EXP:
        return np.exp(t * lam)
    if func == F_SINC:  # sinc(t*lambda), complex t (matfunc_complex.hpp:293-300)
        val = t * lam + 0j
        safe = np.where(np.abs(val) < 1e-8, 1.0, val)
        return np.where(np.abs(val) < 1e-8, 1.0, np.sin(safe) / safe)
    x = np.real(t) * np.sqrt(np.abs(lam))
    sinc = lambda z: np.where(np.abs(z) < 1e-8, 1.0, np.sin(z) / np.where(z == 0, 1, z))
    if func == F_COS_SQRT:
        return np.cos(x)
    if func == F_SINC_SQRT:
        return sinc(x)
    if func == F_SINC2_SQRT:
        return sinc(x) ** 2
    if func == F_ID_SQRT:
        return x
    if func == F_SINC2_HALF:
        return sinc(np.real(t) / 2.0 * np.sqrt(np.abs(lam))) ** 2
    raise ValueError(func)


def krylov(apply, u, t, m, func):
    V, T, beta = lanczos(apply, u, m)
    A = np.tril(np.real(T))
    A = A + np.tril(A, -1).T
    lam, Q = np.linalg.eigh(A)
    c = Q @ (_f(func, lam, t) * Q[0, :])
    if not np.iscomplexobj(u):
        c = np.real(c)
    return beta * (V @ c)


def nonlin_half(u, dt, nonlin=0, sigma=(0.0, 0.5, -0.5, 0.0)):
    tau = 1j * dt
    if nonlin == 0:
        x = u.real * u.real + u.imag * u.imag
        return np.exp(-0.5 * tau * x) * u
    s1 = sigma[0] + 1j * sigma[1]
    s2 = sigma[2] + 1j * sigma[3]
    d = np.abs(u) * np.abs(u)
    return np.exp(-0.5 * tau * (s1 * d + s2 * d * d)) * u


def nlse_steps(dim, nx, ny, nz, dx, dy, u, dt, nsteps, m, nonlin=0, sigma=(0.0, 0.5, -0.5, 0.0)):
    ap = lambda v: laplacian_apply(dim, nx, ny, nz, dx, dy, v)
    u = np.asarray(u, dtype=np.complex128).ravel().copy()
    for _ in range(nsteps):
        r = nonlin_half(u, dt, nonlin, sigma)
        b = krylov(ap, r, -1j * dt, m, F_EXP_ABS)
        u = nonlin_half(b, dt, nonlin, sigma)
    return u


def sg_steps(dim, nx, ny, nz, dx, dy, u, u_past, mfield, dt, nsteps, m):
    ap = lambda v: laplacian_apply(dim, nx, ny, nz, dx, dy, v)
    u = np.asarray(u, dtype=np.float64).ravel().copy()
    up = np.asarray(u_past, dtype=np.float64).ravel().copy()
    mf = np.asarray(mfield, dtype=np.float64).ravel()
    for _ in range(nsteps):
        filt = krylov(ap, u, dt, m, F_ID_SQRT)
        g = mf * (-np.sin(filt))
        s2 = krylov(ap, g, dt, m, F_SINC2_HALF)
        cs = krylov(ap, u, dt, m, F_COS_SQRT)
        u, up = 2 * cs - up + dt * dt * s2, u
    return u, up


def gg_force(y, kind):
    """F of the G2 Gautschi family: sg_single.cuh:18, sg_double.cuh:19, sg_hyperbolic.cuh:18,
    phi4_single.cuh:18 (g = -m F(y))."""
    if kind == 0:
        return np.sin(y)
    if kind == 1:
        return np.sin(y) + np.sin(0.5 * y)
    if kind == 2:
        return np.sinh(y)
    return y + y ** 3


def gautschi_g2_steps(dim, nx, ny, nz, dx, dy, kind, u, u_past, mfield, dt, nsteps, m, bc=True):
    """Phi4Solver / SGE{,Double,Hyperbolic}Solver::step (nlsolvers/device/include/phi4_single.cuh:33-47)
    on the isotropic operator, then the drivers' apply_bc on u."""
    ap = lambda v: laplacian_apply(dim, nx, ny, nz, dx, dy, v)
    u = np.asarray(u, dtype=np.float64).ravel().copy()
    up = np.asarray(u_past, dtype=np.float64).ravel().copy()
    mf = np.asarray(mfield, dtype=np.float64).ravel()
    for _ in range(nsteps):
        y = krylov(ap, u, dt, m, F_ID_SQRT)
        g = -(mf * gg_force(y, kind))
        s2 = krylov(ap, g, dt, m, F_SINC2_SQRT)
        cs = krylov(ap, u, dt, m, F_COS_SQRT)
        u, up = 2.0 * cs - up + dt * dt * s2, u
        if bc:
            u = neumann_bc(dim, nx, ny, nz, u)
    return u, up


def centered_gaussian_3d(n, L, width):
    """create_centered_gaussian_3d (nlsolvers/common/include/util.hpp:95-125), dx = 2L/n."""
    d = 2.0 * L / n
    x = -L + (np.arange(n) + 0.5) * d
    Z, Y, X = np.meshgrid(x, x, x, indexing="ij")
    u = np.exp(-(X * X + Y * Y + Z * Z) / (width * width)).ravel()
    return u / np.linalg.norm(u)
