"""ctypes binding of liboracle_nls.so -- TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class OracleGrid(C.Structure):
    _fields_ = [("dim", C.c_int), ("nx", C.c_uint32), ("ny", C.c_uint32), ("nz", C.c_uint32),
                ("dx", C.c_double), ("dy", C.c_double)]


def use_openmp(on: bool = True):
    """Switch to the OpenMP build (all-cores CPU baseline timing only)."""
    global _LIB, _NAME
    _NAME = "liboracle_nls_omp.so" if on else "liboracle_nls.so"
    _LIB = None


_NAME = "liboracle_nls.so"


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, _NAME)
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        _LIB = C.CDLL(path)
        dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
        g = C.POINTER(OracleGrid)
        L = _LIB
        L.oracle_threads.restype = C.c_int
        L.oracle_laplacian_apply_c.argtypes = [g, dp, dp]
        L.oracle_laplacian_apply_r.argtypes = [g, dp, dp]
        L.oracle_lanczos_c.argtypes = [g, dp, C.c_uint32, dp, dp, C.POINTER(C.c_double)]
        L.oracle_lanczos_r.argtypes = [g, dp, C.c_uint32, dp, dp, C.POINTER(C.c_double)]
        L.oracle_krylov_c.argtypes = [g, dp, C.c_double, C.c_double, C.c_uint32, C.c_int, dp]
        L.oracle_krylov_r.argtypes = [g, dp, C.c_double, C.c_uint32, C.c_int, dp]
        ip = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
        L.oracle_krylov_csr_c.argtypes = [C.c_uint64, ip, ip, dp, dp, C.c_double, C.c_double,
                                          C.c_uint32, C.c_int, dp]
        L.oracle_krylov_csr_r.argtypes = [C.c_uint64, ip, ip, dp, dp, C.c_double, C.c_uint32,
                                          C.c_int, dp]
        L.oracle_nlse_steps.argtypes = [g, dp, C.c_double, C.c_uint32, C.c_uint32, C.c_int,
                                        C.POINTER(C.c_double)]
        L.oracle_sg_steps.argtypes = [g, dp, dp, dp, C.c_double, C.c_uint32, C.c_uint32]
        L.oracle_laplacian_aniso_apply_c.argtypes = [g, dp, dp, dp]
        L.oracle_krylov_aniso_c.argtypes = [g, dp, dp, C.c_double, C.c_double, C.c_uint32, C.c_int,
                                            dp]
        L.oracle_neumann_bc_c.argtypes = [g, dp]
        L.oracle_nlse_g2_steps.argtypes = [g, dp, dp, dp, C.c_double, C.c_uint32, C.c_uint32,
                                           C.c_int]
        L.oracle_nlse_cq_g2_steps.argtypes = [g, dp, dp, C.c_double, C.c_uint32, C.c_uint32,
                                              C.c_double, C.c_double, C.c_int]
        L.oracle_kg_steps.argtypes = [g, dp, dp, dp, dp, dp, C.c_double, C.c_uint32, C.c_uint32, C.c_int]
        L.oracle_neumann_bc_r.argtypes = [g, dp]
        L.oracle_gautschi_g2_steps.argtypes = [g, C.c_int, dp, dp, dp, C.c_double, C.c_uint32, C.c_uint32,
                                               C.c_int]
        L.oracle_nlse_sewi_steps.argtypes = [g, dp, dp, dp, dp, C.c_double, C.c_uint32, C.c_uint32,
                                             C.c_uint32, C.c_int]
    return _LIB


def threads():
    return int(lib().oracle_threads())


def grid(dim, nx, ny, nz, dx, dy):
    return OracleGrid(dim, nx, ny, nz if dim == 3 else 1, dx, dy)


def _c(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.complex128)).view(np.float64).ravel()


def _check(rc):
    if rc != 0:
        raise RuntimeError(f"oracle returned {rc}")


def laplacian_c(g, x):
    xi = _c(x)
    out = np.zeros_like(xi)
    _check(lib().oracle_laplacian_apply_c(C.byref(g), xi, out))
    return out.view(np.complex128)


def laplacian_r(g, x):
    xi = np.ascontiguousarray(x, dtype=np.float64).ravel()
    out = np.zeros_like(xi)
    _check(lib().oracle_laplacian_apply_r(C.byref(g), xi, out))
    return out


def lanczos_c(g, u, m):
    """lanczos_L (eigen_krylov_complex.hpp:10-53): V as m rows of n, T (m x m, T[r, c]),
    beta0 = ||u||."""
    ui = _c(u)
    n = ui.size // 2
    V = np.zeros(2 * n * m)
    T = np.zeros(2 * m * m)
    b = C.c_double(0.0)
    _check(lib().oracle_lanczos_c(C.byref(g), ui, m, V, T, C.byref(b)))
    # column-major n x m -> rows; column-major m x m -> T[r, c]
    return V.view(np.complex128).reshape(m, n), T.view(np.complex128).reshape(m, m).T.copy(), b.value


def lanczos_r(g, u, m):
    """real lanczos_L (eigen_krylov_real.hpp:5-51): V as m rows of n, T[r, c], beta0."""
    ui = np.ascontiguousarray(u, dtype=np.float64).ravel()
    n = ui.size
    V = np.zeros(n * m)
    T = np.zeros(m * m)
    b = C.c_double(0.0)
    _check(lib().oracle_lanczos_r(C.byref(g), ui, m, V, T, C.byref(b)))
    return V.reshape(m, n), T.reshape(m, m).T.copy(), b.value


def krylov_c(g, u, t, m, func=0):
    ui = _c(u)
    out = np.zeros_like(ui)
    t = complex(t)
    _check(lib().oracle_krylov_c(C.byref(g), ui, t.real, t.imag, m, func, out))
    return out.view(np.complex128)


def krylov_r(g, u, t, m, func):
    ui = np.ascontiguousarray(u, dtype=np.float64).ravel()
    out = np.zeros_like(ui)
    _check(lib().oracle_krylov_r(C.byref(g), ui, float(t), m, func, out))
    return out


def krylov_csr(A, u, t, m, func):
    A = A.tocsr()
    rp = A.indptr.astype(np.int64)
    ci = A.indices.astype(np.int64)
    val = np.ascontiguousarray(A.data, dtype=np.float64)
    if np.iscomplexobj(u) or isinstance(t, complex):
        ui = _c(u)
        out = np.zeros_like(ui)
        t = complex(t)
        _check(lib().oracle_krylov_csr_c(A.shape[0], rp, ci, val, ui, t.real, t.imag, m, func, out))
        return out.view(np.complex128)
    ui = np.ascontiguousarray(u, dtype=np.float64).ravel()
    out = np.zeros_like(ui)
    _check(lib().oracle_krylov_csr_r(A.shape[0], rp, ci, val, ui, float(t), m, func, out))
    return out


def nlse_steps(g, u, dt, nsteps, m, nonlin=0, sigma=(0.0, 0.5, -0.5, 0.0)):
    ui = _c(u).copy()
    sg = (C.c_double * 4)(*sigma)
    _check(lib().oracle_nlse_steps(C.byref(g), ui, dt, nsteps, m, nonlin, sg))
    return ui.view(np.complex128)


def sg_steps(g, u, u_past, mfield, dt, nsteps, m):
    u = np.ascontiguousarray(u, dtype=np.float64).ravel().copy()
    up = np.ascontiguousarray(u_past, dtype=np.float64).ravel().copy()
    mf = np.ascontiguousarray(mfield, dtype=np.float64).ravel()
    _check(lib().oracle_sg_steps(C.byref(g), u, up, mf, dt, nsteps, m))
    return u, up


def _r(a):
    return np.ascontiguousarray(a, dtype=np.float64).ravel()


def laplacian_aniso_c(g, c, x):
    """G2 div(c grad) operator (nlsolvers/common/include/laplacians.hpp:54-218)."""
    xi = _c(x)
    out = np.zeros_like(xi)
    _check(lib().oracle_laplacian_aniso_apply_c(C.byref(g), _r(c), xi, out))
    return out.view(np.complex128)


def krylov_aniso_c(g, c, u, t, m, func=1):
    ui = _c(u)
    out = np.zeros_like(ui)
    t = complex(t)
    _check(lib().oracle_krylov_aniso_c(C.byref(g), _r(c), ui, t.real, t.imag, m, func, out))
    return out.view(np.complex128)


def neumann_bc(g, u):
    ui = _c(u).copy()
    _check(lib().oracle_neumann_bc_c(C.byref(g), ui))
    return ui.view(np.complex128)


def nlse_g2_steps(g, c, mfield, u, dt, nsteps, m, bc=True):
    ui = _c(u).copy()
    _check(lib().oracle_nlse_g2_steps(C.byref(g), _r(c), _r(mfield), ui, dt, nsteps, m, 1 if bc else 0))
    return ui.view(np.complex128)


def nlse_cq_g2_steps(g, mfield, u, dt, nsteps, m, s1, s2, bc=True):
    """G2 cubic-quintic (nlse_cubic_quintic_dev.hpp:79-95) + the driver's BC."""
    ui = _c(u).copy()
    _check(lib().oracle_nlse_cq_g2_steps(C.byref(g), _r(mfield), ui, dt, nsteps, m, s1, s2, 1 if bc else 0))
    return ui.view(np.complex128)


def nlse_sewi_steps(g, c, mfield, u, u_prev, dt, first_step, nsteps, m, bc=True):
    """G2 sEWI steps first_step .. first_step+nsteps-1; returns (u, u_prev)."""
    ui = _c(u).copy()
    pi = _c(u if u_prev is None else u_prev).copy()
    _check(lib().oracle_nlse_sewi_steps(C.byref(g), _r(c), _r(mfield), ui, pi, dt, first_step, nsteps, m,
                                        1 if bc else 0))
    return ui.view(np.complex128), pi.view(np.complex128)


def kg_steps(g, c, mfield, u, u_past, dt, nsteps, m, bc=True):
    """G2 Klein-Gordon Gautschi steps; returns (u, u_past, v)."""
    u = _r(u).copy()
    up = _r(u_past).copy()
    v = np.zeros_like(u)
    _check(lib().oracle_kg_steps(C.byref(g), _r(c), _r(mfield), u, up, v, dt, nsteps, m, 1 if bc else 0))
    return u, up, v


def neumann_bc_r(g, u):
    ui = _r(u).copy()
    _check(lib().oracle_neumann_bc_r(C.byref(g), ui))
    return ui


GG_KINDS = {"sg": 0, "sg_double": 1, "sg_hyperbolic": 2, "phi4": 3}


def gautschi_g2_steps(g, kind, u, u_past, mfield, dt, nsteps, m, bc=True):
    """G2 Gautschi family (phi4_single.cuh:33-47 & siblings); returns (u, u_past)."""
    u = _r(u).copy()
    up = _r(u_past).copy()
    _check(lib().oracle_gautschi_g2_steps(C.byref(g), int(kind), u, up, _r(mfield), dt, nsteps, m,
                                          1 if bc else 0))
    return u, up
