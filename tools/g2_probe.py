"""Per-pass cost of the G2 anisotropic NLSE's two-vector passes (bench g2_3d_256:
256^3, m = 25, div(c grad), m(x), BC per step) for a list of environment variants,
e.g. the LDS-DMA form against the register form (NLS_P2_REG=1).  Prints ms per step,
per pass J the ms and the rate on the pass's bytes (S_0..S_J read, ns vectors
written, c once (DMA form) or y written + read and c twice (register form)).
usage: python tools/g2_probe.py [VAR=value,VAR=value ...] ..."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "nonlinear-solvers_amd"))
import nls_amd
n, m, steps = int(sys.argv[2]), int(sys.argv[3]), 10
dx = 20.0 / (n - 1)
rng = np.random.default_rng(0)
N = n ** 3
u = (rng.standard_normal(N) + 1j * rng.standard_normal(N)) * 1e-3 + 1.0
mf = 1.0 + 0.5 * rng.random(N)
cf = 0.7 + 0.6 * rng.random(N)
with nls_amd.Solver(3, n, n, n, dx, dx, equation=nls_amd.NLSE_G2, m=m) as s:
    s.set_coefficients(mf, cf)
    s.set_field(u)
    for _ in range(2):
        s.step(1e-3, 1); s.apply_bc()
    s.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        s.step(1e-3, 1); s.apply_bc()
    s.sync()
    el = (time.perf_counter() - t0) / steps
    s.set_timing(True)
    for _ in range(3):
        s.step(1e-3, 1); s.apply_bc()
    s.sync()
    tm = s.timing()
    s.set_timing(False)
reg = os.environ.get("NLS_P2_REG", "0") == "1"
cls = {k: round(v / 3, 3) for k, v in tm["class_ms"].items() if v}
nstore = m - 1
out = []
for j in range(0, 32):
    if not tm["update_count"][j]:
        continue
    ms = tm["update_ms"][j] / 3
    ns = min(2, nstore - 1 - j)
    b = (j + 1 + ns) * 16 + (64 if reg else 8)
    out.append(f"J{j}:{ms:.3f}ms/{b * N / ms / 1e9:.2f}TB/s")
print(f"{el * 1e3:8.3f} ms/step {N / el / 1e6:8.0f} Mcells*steps/s  {cls}", flush=True)
print("   " + " ".join(out), flush=True)
"""

n, m = 256, 25
# variants: one argument each, or several in one argument joined by '/' (gpu.sh py steps);
# '-' = no change
args = [v for a in sys.argv[1:] for v in a.split("/")] or ["", "NLS_P2_REG=1"]
variants = [dict(kv.split("=", 1) for kv in a.split(",")) if a and a != "-" else {} for a in args]
for extra in variants:
    env = dict(os.environ, **extra)
    print(f"# {extra}", flush=True)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, str(n), str(m)], env=env, timeout=300)
    if r.returncode:
        sys.exit(r.returncode)
