"""Per-pass and tail times of the 512^3 m=16 step under tile-order / tile-depth knobs,
every configuration in ONE process on one box, rounds interleaved (box drift cancels):
NLS_P2_ORDER (k_p2d tile order bits: 2 x-fastest, 4 no XCD bands), NLS_P2_KZ (k_p2d
tile depth), NLS_KZ_FUSED (fused tail tile depth), NLS_TILE_REMAP (tail XCD bands).
usage: python tools/order_sweep.py [n] [m] [steps] [rounds] "ENV=V,ENV=V" "..." ..."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nonlinear-solvers_amd"))
import nls_amd  # noqa: E402

n = int(sys.argv[1])
m = int(sys.argv[2])
steps = int(sys.argv[3])
rounds = int(sys.argv[4])
configs = sys.argv[5:] or [""]
KNOBS = ("NLS_P2_ORDER", "NLS_P2_KZ", "NLS_KZ_FUSED", "NLS_TILE_REMAP", "NLS_KZ_ALPHA2", "NLS_TAIL_DYN")
dx = 20.0 / (n - 1)
rng = np.random.default_rng(0)
x = np.linspace(-10, 10, n)
u0 = (np.exp(-(x[:, None, None] ** 2 + x[None, :, None] ** 2 + x[None, None, :] ** 2) / 8)
      + 1e-3 * rng.standard_normal((n, n, n))).astype(np.complex128).ravel()
ref = None
for r in range(rounds):
    for cfg in configs:
        for k in KNOBS:
            os.environ.pop(k, None)
        for kv in filter(None, cfg.split(",")):
            k, v = kv.split("=")
            os.environ[k] = v
        with nls_amd.Solver(3, n, n, n, dx, dx, m=m) as s:
            s.set_field(u0)
            s.step(1e-3, 2)
            s.set_timing(True)
            t0 = time.perf_counter()
            s.step(1e-3, steps)
            wall = (time.perf_counter() - t0) / steps * 1e3
            t = s.timing()
            s.set_timing(False)
            s.set_field(u0)
            s.step(1e-3, 1)
            u = s.get_field()
        if ref is None:
            ref = u
        dev = float(np.abs(u - ref).max())
        uc = t["update_count"]
        per = " ".join(f"{t['update_ms'][J] / uc[J]:.3f}" for J in range(m - 1) if uc[J])
        cm = {k: round(v / steps, 3) for k, v in t["class_ms"].items() if v}
        print(f"round {r} [{cfg or 'default'}] wall {wall:.2f} ms/step; passes {per}; {cm}; max|u-u_ref| {dev:.1e}",
              flush=True)
