"""GPU parity at the BASELINE.json sizes through size-independent properties.

The oracle cannot run 512^3 or 8192^2 in seconds, so at the benchmark sizes
the tests check what must hold exactly or to rounding for ANY correct
implementation of the reference algorithm:

  * unitarity: the cubic SS2 step conserves the discrete L2 norm (exp of the
    Hermitian T is unitary, the nonlinear phase has unit modulus);
  * mirror symmetry: the operators are symmetric under x -> -x (3D; the 3D
    "y-wrap" breaks the y mirror) and under x, y mirrors and transposition (2D),
    so an exactly symmetric initial field stays exactly (bitwise) symmetric:
    every per-cell sum the kernels form pairs mirrored neighbours as a + b,
    and the reductions are scalars shared by all cells;
  * scale covariance of one Krylov action: f(L)(2u) == 2 f(L)u bit for bit
    (the Lanczos start vector u/||u|| is the same number);
  * bitwise run-to-run reproducibility (fixed-order reductions).
"""
import numpy as np
import pytest

from conftest import rel_l2

pytestmark = pytest.mark.gpu
nls_amd = pytest.importorskip("nls_amd")


def mirror_x_field(dim, n, L=10.0, seed=0):
    """Gaussian solitons placed in mirror pairs about x = 0 (+ x-symmetric noise);
    built from separable 1D factors so that 512^3 takes seconds."""
    rng = np.random.default_rng(seed)
    x = np.linspace(-L, L, n)
    u = np.zeros((n,) * dim, dtype=np.complex128)
    for _ in range(3):
        cx, cy, cz = rng.uniform(1.0, L / 2), rng.uniform(-L / 2, L / 2), rng.uniform(-L / 2, L / 2)
        ky = rng.uniform(-1, 1)
        fy = np.exp(-((x - cy) ** 2) / 2.0) * np.exp(1j * ky * x)
        fx = np.exp(-((x - cx) ** 2) / 2.0) + np.exp(-((x + cx) ** 2) / 2.0)   # mirror pair in x
        if dim == 3:
            fz = np.exp(-((x - cz) ** 2) / 2.0)
            u += fz[:, None, None] * (fy[:, None] * fx[None, :])[None, :, :]
        else:
            u += fy[:, None] * fx[None, :]
    u += 1e-3 * (rng.standard_normal(u.shape) + 1j * rng.standard_normal(u.shape))
    return 0.5 * (u + u[..., ::-1])   # exactly x-symmetric (a + b == b + a)


def symmetrize_2d(u):
    """Exactly symmetric under both mirrors and the transpose."""
    u = 0.5 * (u + u[:, ::-1])
    u = 0.5 * (u + u[::-1, :])
    return 0.5 * (u + u.T)


def test_3d_512_cubic_norm_symmetry_determinism():
    n, m, dt, steps = 512, 16, 1e-3, 2
    dx = 20.0 / (n - 1)
    u0 = mirror_x_field(3, n)
    with nls_amd.Solver(3, n, n, n, dx, dx, m=m) as s:
        s.set_field(u0.ravel())
        s.step(dt, steps)
        a = s.get_field().reshape(n, n, n)
        s.set_field(u0.ravel())
        s.step(dt, steps)
        b = s.get_field().reshape(n, n, n)
    assert np.array_equal(a, b)                                   # reproducible
    n0, n1 = np.linalg.norm(u0), np.linalg.norm(a)
    assert abs(n1 / n0 - 1.0) < 1e-12                             # unitary step
    assert np.array_equal(a, a[..., ::-1])                        # x mirror, bitwise
    assert rel_l2(a, u0) > 1e-6                                   # and it did evolve


def test_3d_512_krylov_scale_covariance():
    n, m = 512, 16
    dx = 20.0 / (n - 1)
    u0 = mirror_x_field(3, n, seed=1).ravel()
    with nls_amd.Solver(3, n, n, n, dx, dx, m=m) as s:
        y1 = s.krylov_apply(u0, -1e-3j, nls_amd.F_EXP_ABS)
        y2 = s.krylov_apply(2.0 * u0, -1e-3j, nls_amd.F_EXP_ABS)
    assert np.array_equal(y2, 2.0 * y1)


def test_2d_4096_cubic_norm_and_symmetries():
    n, m, dt, steps = 4096, 16, 1e-3, 3
    dx = 20.0 / (n - 1)
    x = np.linspace(-10, 10, n)
    Y, X = np.meshgrid(x, x, indexing="ij", sparse=True)
    u0 = np.zeros((n, n), np.complex128)
    for c in (2.0, 4.5):   # four-fold symmetric arrangement, real initial data
        for sx in (1, -1):
            for sy in (1, -1):
                u0 += np.exp(-((X - sx * c) ** 2 + (Y - sy * c) ** 2))
    u0 += 1e-3 * np.cos(3 * X) * np.cos(3 * Y)
    u0 = symmetrize_2d(u0)
    with nls_amd.Solver(2, n, n, 1, dx, dx, m=m) as s:
        s.set_field(u0.ravel())
        s.step(dt, steps)
        a = s.get_field().reshape(n, n)
    assert abs(np.linalg.norm(a) / np.linalg.norm(u0) - 1.0) < 1e-12
    for img in (a[:, ::-1], a[::-1, :], a.T):
        assert np.array_equal(a, img)


def test_sg_8192_symmetries_and_determinism():
    """C4 (sg_driver_dev.cpp:34-36 initial data, m(x) = -1): radially symmetric
    data stays symmetric under both mirrors and the transpose."""
    n, m, steps, L = 8192, 10, 2, 3.0
    dx = 2 * L / (n - 1)
    dt = 5.0 / 500
    x = np.linspace(-L, L, n)
    Y, X = np.meshgrid(x, x, indexing="ij", sparse=True)
    u0 = symmetrize_2d(2.0 * np.arctan(np.exp(3.0 - 5.0 * np.sqrt(X * X + Y * Y)))).ravel()
    mf = -np.ones(n * n)
    with nls_amd.Solver(2, n, n, 1, dx, dx, equation=nls_amd.SG_GAUTSCHI, m=m) as s:
        s.set_sg_state(u0, u0, mf)
        s.step(dt, steps)
        a = s.get_field().reshape(n, n)
        s.set_sg_state(u0, u0, mf)
        s.step(dt, steps)
        b = s.get_field().reshape(n, n)
    assert np.array_equal(a, b)
    for img in (a[:, ::-1], a[::-1, :], a.T):
        assert np.array_equal(a, img)
    assert rel_l2(a, u0.reshape(n, n)) > 1e-8
