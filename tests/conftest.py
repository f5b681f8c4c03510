"""Shared test setup: markers, import paths, device detection."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "nonlinear-solvers_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running")


def rel_l2(a, b):
    import numpy as np
    a = np.asarray(a).ravel()
    b = np.asarray(b).ravel()
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (nb if nb > 0 else 1.0))


@pytest.fixture
def rel():
    return rel_l2


# The reference algorithm's own rounding sensitivity (DESIGN.md section 6,
# "parity floor"): on smooth data over fine grids, or at ||L|| dt >> m, the
# Lanczos basis amplifies rounding noise in the high modes by roughly
# prod_j ||L|| / beta_j per action, and the SS2 map carries that growth from
# step to step.  The floor is measured on the ORACLE ITSELF: the same oracle
# trajectory from an initial field perturbed by one ulp per component
# (perturb_ulp, two seeds; self_floor).  Where it exceeds the north_star
# tolerance the reference algorithm cannot resolve 1e-10 on that problem, and a
# GPU trajectory is held to a per-case factor x that floor instead.  The factor is
# the per-step rounding of a valid implementation in units of that one-ulp start: the
# GPU's first SS2 step differs from the oracle's by 8-14x the one-ulp floor
# (different but equally exact summation orders: CGS / s-step vs MGS, tiles,
# FMA), the numpy twin's by 25-140x, and the reference algorithm then amplifies
# either deviation at the same rate.  FLOOR_FACTORS are ~2x the largest GPU/floor
# ratio observed where the floor exceeds the tolerance (profiles/r03/parity_floor.txt):
# C1 0.71, 2D cubic at C2's spacing 7.8, 2D cubic-quintic 15.0, sine-Gordon at C4's
# spacing 5.8.  The floored tests also check the mechanism directly: the GPU within
# PROPAGATED_FACTOR x the oracle continued from the GPU's own early field (observed
# GPU/propagated 0.57-1.34).
# ("resolved": cases held to the tolerance at every checkpoint; the factor only labels
# the parity record)
FLOOR_FACTORS = {"c1": 2.0, "nlse2d_cubic": 16.0, "nlse2d_cq": 30.0, "sg": 12.0, "resolved": 1.0}
PROPAGATED_FACTOR = 3.0


def parity_bound(tol, floor, case):
    return max(tol, FLOOR_FACTORS[case] * floor)


def perturb_ulp(u, seed):
    """u with every real and imaginary component moved by about one ulp
    (relative 2^-52 Gaussian noise): the size of one rounding error."""
    import numpy as np
    rng = np.random.default_rng(seed)
    u = np.asarray(u)
    e = 2.0 ** -52
    if np.iscomplexobj(u):
        return (u.real * (1 + e * rng.standard_normal(u.shape))
                + 1j * u.imag * (1 + e * rng.standard_normal(u.shape)))
    return u * (1 + e * rng.standard_normal(u.shape))


def self_floor(run, u0, seeds=(101, 202)):
    """Per checkpoint, the largest distance between the oracle run `run(u0)` and
    the oracle runs from one-ulp perturbations of u0.  run returns a dict
    {checkpoint: field} (or a list of snapshots); so does self_floor."""
    # the runs are independent oracle calls (ctypes releases the GIL): in parallel
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=1 + len(seeds)) as ex:
        futs = [ex.submit(run, u0)] + [ex.submit(run, perturb_ulp(u0, sd)) for sd in seeds]
        base, others = futs[0].result(), [f.result() for f in futs[1:]]
    keys = list(base.keys()) if isinstance(base, dict) else list(range(len(base)))
    fl = {k: 0.0 for k in keys}
    for other in others:
        for k in keys:
            fl[k] = max(fl[k], rel_l2(other[k], base[k]))
    return base, fl


def record_parity(case, rows, kind):
    """Append one case's per-checkpoint parity record to $NLS_PARITY_LOG (JSON
    lines; tools/parity_floor.py formats profiles/<round>/parity_floor.txt).
    rows: [(checkpoint, gpu_err, self_floor, twin_floor or None[, propagated])];
    kind: the FLOOR_FACTORS key of the case."""
    path = os.environ.get("NLS_PARITY_LOG")
    if not path:
        return
    import json
    with open(path, "a") as f:
        f.write(json.dumps({"case": case, "rows": [
            {"checkpoint": r[0], "gpu_err": r[1], "self_floor": r[2], "twin_floor": r[3],
             "propagated": r[4] if len(r) > 4 else None,
             "bound": parity_bound(1e-10, r[2], kind), "ratio_gpu_self": (r[1] / r[2]) if r[2] > 0 else None}
            for r in rows]}) + "\n")
