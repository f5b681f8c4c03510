"""GPU against fixtures computed by the reference's own executable Python
(tests/golden/make_ref_fixtures.py): Krylov actions built from the V and T of
LanczosStepTorch (nlsolvers/fusing_kernels.py:8-45) -- complex, and on real-valued
data the real recurrence of device/lanczos.hpp:126-194 / eigen_krylov_real.hpp:5-51 --
and the 2D Neumann BC of neumann_bc (bc_update_kernel_fusion.py:18-27).  No oracle in
the loop: the reference's numbers directly.

Code paths: the GPU's default pass form (two new vectors per pass: k_p2d, also as real
cell pairs in 2D), the one-vector passes (NLS_PASS2=0), and the default pass form on
the LARGE-SLAB launch shapes the 512^3 bench runs (NLS_LARGE_SLAB=1: one tile per
workgroup grids, 4-plane alpha tiles, the fused tail's tile queue with 8-plane tiles,
plus NLS_P2_KZ=4 so every k_p2d column has several z tiles as at 512^3).

Fixtures: the 32^2 / 16^3 grids at the G1 drivers' spacing 20/(n-1) and, on white
noise, at the BASELINE workloads' spacings (hl = 20/511: 3D 512^3; c2 = 20/4095: 2D
4096^2; c4 = 6/8191: sine-Gordon 8192^2).

Tolerances: the action's error scales with the argument of f (the eigenvalues carry a
relative rounding error, multiplied by |t| rho(T), or |t| sqrt(rho(T)) for the
t sqrt|lambda| functions: tests/test_oracle.py ref_kappa), so the bound is
max(1e-12, TOL_GPU_K (1 + kappa)) with TOL_GPU_K = 1000 eps; at the mild spacings that
is the 1e-12 every GPU action test uses.  BC bit-exact.
"""
import os

import numpy as np
import pytest

from conftest import rel_l2
from test_oracle import (REF_COMPLEX, REF_REAL, REF_STIFF, ref_action, ref_action_err, ref_cases, ref_kappa,
                         ref_overflows)

pytestmark = pytest.mark.gpu
nls_amd = pytest.importorskip("nls_amd")

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TOL_GPU_K = 1000 * 2.22e-16
MODES = {"pass2": {"NLS_PASS2": "1"}, "one": {"NLS_PASS2": "0"},
         "large": {"NLS_PASS2": "1", "NLS_LARGE_SLAB": "1", "NLS_P2_KZ": "4"}}


def _bound(kap):
    return max(1e-12, TOL_GPU_K * (1 + kap))


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name", REF_COMPLEX + REF_REAL + REF_STIFF)
@pytest.mark.parametrize("m", [10, 16])
def test_gpu_action_matches_reference_lanczos(monkeypatch, mode, name, m):
    """Every Krylov convention on the GPU == beta0 V Q f(Lambda) Q^H e1 from the
    reference's own V, T: complex fields (NLSE handle) exp(t|lambda|), exp(t lambda),
    sinc(t lambda); real fields (sine-Gordon handle) cos, sinc, sinc^2, id and
    sinc^2-half of t sqrt|lambda|."""
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    d = np.load(os.path.join(GOLD, f"{name}.npz"))
    dim, n, dx = int(d["dim"]), int(d["n"]), float(d["dx"])
    real = "_real" in name
    eq = nls_amd.SG_GAUTSCHI if real else nls_amd.NLSE_CUBIC
    errs, overflow = [], []
    with nls_amd.Solver(dim, n, n, n, dx, dx, equation=eq, m=m) as s:
        for t, func in ref_cases(name):
            kap = ref_kappa(d, m, t, func)
            got = s.krylov_apply(d["u"], t, func)
            with np.errstate(all="ignore"):
                ref = ref_action(d, m, t, func)
            if ref_overflows(ref):
                # sinc(t lambda) of an imaginary argument past kappa ~ 710 (sinh growth): the
                # reference's own action is not finite; the device must overflow as well
                overflow.append((t, func, kap, bool(np.all(np.isfinite(got)))))
                continue
            err = ref_action_err(got, ref)
            errs.append((t, func, err, kap))
    assert all(f == 7 and not fin for _, f, _, fin in overflow), overflow
    assert len(errs) >= len(ref_cases(name)) - 2
    bad = [e for e in errs if not e[2] <= _bound(e[3])]
    assert not bad, "; ".join(f"t={t} f={f}: {e:.2e} (kappa {k:.1f}, bound {_bound(k):.1e})"
                              for t, f, e, k in bad)


def test_gpu_neumann_bc_matches_reference():
    """nls_apply_bc (k_neumann_bc) == the reference's neumann_bc, bit for bit, on a
    square and a non-square complex field (tensor axis 0 = our rows, ny)."""
    d = np.load(os.path.join(GOLD, "ref_bc2d.npz"))
    for a, b in ((24, 24), (9, 13)):
        with nls_amd.Solver(2, b, a, 1, 0.5, 0.5, equation=nls_amd.NLSE_G2, m=4) as s:
            s.set_coefficients(np.ones(a * b), np.ones(a * b))
            s.set_field(d[f"uc_{a}x{b}"].ravel())
            s.apply_bc()
            assert np.array_equal(s.get_field().reshape(a, b), d[f"bc_c_{a}x{b}"])


def test_gpu_neumann_bc_real_matches_reference():
    """The real-field BC of the Klein-Gordon drivers (k_neumann_bc_r) == neumann_bc on f64."""
    d = np.load(os.path.join(GOLD, "ref_bc2d.npz"))
    for a, b in ((24, 24), (9, 13)):
        with nls_amd.Solver(2, b, a, 1, 0.5, 0.5, equation=nls_amd.KG_GAUTSCHI, m=4) as s:
            s.set_coefficients(np.ones(a * b), np.ones(a * b))
            u = d[f"ur_{a}x{b}"].ravel()
            s.set_sg_state(u, u)
            s.apply_bc()
            assert np.array_equal(s.get_field().reshape(a, b), d[f"bc_r_{a}x{b}"])
