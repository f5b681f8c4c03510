"""Per-pass times of the two-vector Lanczos at a BASELINE grid (HIP-event timing
of every launch): update_ms[J] / launches, algorithmic bytes (J+1 reads + 2 or 1
writes per cell) and the achieved GB/s.  Usage: python tools/p2_probe.py [n] [m] [steps]
(env NLS_PASS2 / NLS_P2_* select the variant)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nonlinear-solvers_amd"))
import nls_amd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
m = int(sys.argv[2]) if len(sys.argv) > 2 else 16
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
dx = 20.0 / (n - 1)
rng = np.random.default_rng(0)
x = np.linspace(-10, 10, n)
u0 = (np.exp(-(x[:, None, None] ** 2 + x[None, :, None] ** 2 + x[None, None, :] ** 2) / 8)
      + 1e-3 * rng.standard_normal((n, n, n))).astype(np.complex128).ravel()
cells = n ** 3
with nls_amd.Solver(3, n, n, n, dx, dx, m=m) as s:
    s.set_field(u0)
    s.step(1e-3, 2)
    s.set_timing(True)
    s.step(1e-3, steps)
    t = s.timing()
tot = 0.0
uc = t["update_count"]
p2 = os.environ.get("NLS_PASS2", "1") != "0" and uc[1] == 0
Js = [j for j in range(m - 1) if uc[j]]
for i, J in enumerate(Js):
    c = uc[J]
    ms = t["update_ms"][J] / c
    tot += t["update_ms"][J] / steps
    ns = ((Js[i + 1] if i + 1 < len(Js) else m - 2) - J) if p2 else 1
    vec = J + 1 + ns
    gbs = vec * 16 * cells / (ms * 1e-3) / 1e9
    print(f"J={J:2d} ns={ns} {ms:7.3f} ms  {vec:2d} vectors  {gbs:7.0f} GB/s")
print("update per step", round(tot, 3), "ms;", {k: round(v / steps, 3) for k, v in t["class_ms"].items()})
