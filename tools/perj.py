"""Per-J update pass times (HIP events) for the bench workload, NLS_* env as given."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nonlinear-solvers_amd"), ROOT]
import nls_amd
import bench
w = dict(bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "nlse3d_512"])
n, dim, m = w["n"], w["dim"], w["m"]
dx = 2 * w["L"] / (n - 1)
s = nls_amd.Solver(dim, n, n, n if dim == 3 else 1, dx, dx, equation=w["eq"], m=m)
u = bench.synthetic_ic(w, s.z0, s.nzl)
if w["eq"] == 3:  # G2: m(x), c(x) as in bench.py
    s.set_field(u)
    s.set_coefficients(*bench.g2_coefficients(n, w["L"], s.z0, s.nzl))
else:
    u /= np.sqrt(bench.global_mass(u, dx ** dim))
    s.set_field(u)
s.step(w["dt"], 2)
s.sync()
s.reset_timing(); s.set_timing(True)
s.step(w["dt"], 4)
t = s.timing()
out = {"J": [round(t["update_ms"][j] / max(t["update_count"][j], 1), 4) for j in range(m)],
       "class": {k: round(v / 4, 3) for k, v in t["class_ms"].items()}}
print(json.dumps(out))
s.close()
