"""Same-allocation A/B of launch-shape knobs (nls_debug_knob) on one live handle: the
per-allocation placement of the basis moves kernel times by up to ~5-10 % from handle
to handle on one box, more than the effects measured here, so every variant runs on
the SAME handle, rounds interleaved.  Prints per variant and round the per-pass times,
the tail and the step's kernel classes.
usage: python tools/knob_ab.py n m steps rounds "knob=v,knob=v" ...
knobs: tail_dyn (1), kz_fused (2), p2_order (3); "" = as created.  (Round 4: shorter k_p2d tiles at the
end of each launch, chunks of 128 / 64 / 32 planes after the first 256, measured no gain or a loss,
profiles/r04/knob_ab_512.txt; removed.)  (Tiles of k_p2d by
ticket of a global counter measured +1.8 % pass time, and the tail's queue on the full
tile grid +50 %: removed, profiles/r03/knob_ab_dyn.txt.)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nonlinear-solvers_amd"))
import nls_amd  # noqa: E402

KNOB = {"tail_dyn": 1, "kz_fused": 2, "p2_order": 3}
n, m, steps, rounds = (int(a) for a in sys.argv[1:5])
variants = sys.argv[5:] or [""]
dx = 20.0 / (n - 1)
rng = np.random.default_rng(0)
x = np.linspace(-10, 10, n)
u0 = (np.exp(-(x[:, None, None] ** 2 + x[None, :, None] ** 2 + x[None, None, :] ** 2) / 8)
      + 1e-3 * rng.standard_normal((n, n, n))).astype(np.complex128).ravel()
# KNOB_AB_G2=1: the G2 NLSE (m(x), div(c grad)) instead of the isotropic cubic NLSE
g2 = os.environ.get("KNOB_AB_G2") == "1"
kw = {"equation": nls_amd.NLSE_G2} if g2 else {}
with nls_amd.Solver(3, n, n, n, dx, dx, m=m, **kw) as s:
    if g2:
        N = n ** 3
        s.set_coefficients(1.0 + 0.5 * rng.random(N), 0.7 + 0.6 * rng.random(N))
    s.set_field(u0)
    s.step(1e-3, 2)
    for r in range(rounds):
        for v in variants:
            for kv in filter(None, v.split(",")):
                k, val = kv.split("=")
                s.debug_knob(KNOB[k], int(val))
            s.step(1e-3, 1)  # settle
            s.reset_timing()
            s.set_timing(True)
            s.step(1e-3, steps)
            t = s.timing()
            s.set_timing(False)
            uc = t["update_count"]
            per = " ".join(f"{t['update_ms'][J] / uc[J]:.3f}" for J in range(m - 1) if uc[J])
            cm = {k: round(val / steps, 3) for k, val in t["class_ms"].items() if val}
            print(f"round {r} [{v or 'as created'}] passes {per}; {cm}", flush=True)
