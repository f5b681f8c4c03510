import os, sys, threading, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nonlinear-solvers_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import nls_amd, oracle_py as O

def run(nranks, fn, dim=3, n=16, m=4, eq=0):
    L = 5.0; dx = 2 * L / (n - 1)
    grp = nls_amd.Group(nranks); out = [None] * nranks; err = []
    def work(r):
        try:
            s = nls_amd.Solver(dim, n, n, n, dx, dx, equation=eq, m=m, device=0, nranks=nranks, rank=r, group=grp)
            out[r] = (s.z0, fn(s)); s.close()
        except Exception as e:
            err.append((r, repr(e)))
    ts = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    [t.start() for t in ts]; [t.join() for t in ts]
    if err: print("ERR", err)
    return np.concatenate([o[1] for o in sorted(out, key=lambda t: t[0])])

n = 16; L = 5.0; dx = 2 * L / (n - 1); P = n * n
rng = np.random.default_rng(0)
u = rng.standard_normal(n**3) + 1j * rng.standard_normal(n**3)
g = O.grid(3, n, n, n, dx, dx)
sl = lambda s: u[s.z0 * P:(s.z0 + s.nzl) * P]
got = run(2, lambda s: s.laplacian(sl(s)))
print("lap", np.linalg.norm(got - O.laplacian_c(g, u)) / np.linalg.norm(O.laplacian_c(g, u)))
for m in (1, 2, 3, 4):
    got = run(2, lambda s: s.krylov_apply(sl(s), -1e-2j, 0), m=m)
    ref = O.krylov_c(g, u, -1e-2j, m, 0)
    print("krylov m", m, np.linalg.norm(got - ref) / np.linalg.norm(ref), np.isnan(got).sum())
for m in (1, 4):
    def f(s):
        s.set_field(sl(s)); s.step(1e-3, 1); return s.get_field()
    got = run(2, f, m=m)
    ref = O.nlse_steps(g, u, 1e-3, 1, m)
    print("step m", m, np.linalg.norm(got - ref) / np.linalg.norm(ref), np.isnan(got).sum())
