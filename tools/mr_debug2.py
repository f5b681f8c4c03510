import os, sys, threading, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nonlinear-solvers_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import nls_amd, oracle_py as O
n = 16; L = 5.0; dx = 2 * L / (n - 1); P = n * n
rng = np.random.default_rng(0)
u = rng.standard_normal(n**3) + 1j * rng.standard_normal(n**3)
print("total |u|^2", np.sum(abs(u)**2), "half", np.sum(abs(u[:n**3//2])**2))
grp = nls_amd.Group(2)
def work(r):
    s = nls_amd.Solver(3, n, n, n, dx, dx, m=1, device=0, nranks=2, rank=r, group=grp)
    y = s.krylov_apply(u[s.z0*P:(s.z0+s.nzl)*P], -1e-2j, 0)
    print("rank", r, "z0", s.z0, "nzl", s.nzl, "out norm", np.linalg.norm(y), flush=True)
ts = [threading.Thread(target=work, args=(r,)) for r in range(2)]
[t.start() for t in ts]; [t.join() for t in ts]
