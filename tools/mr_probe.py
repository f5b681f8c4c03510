"""2 ranks of the z-slab path on whatever GPUs exist (experiment)."""
import os, sys, numpy as np
import torch.multiprocessing as mp
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nonlinear-solvers_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))

def worker(rank, world, rid, q):
    import nls_amd
    n, L = 16, 5.0
    dx = 2 * L / (n - 1)
    rng = np.random.default_rng(0)
    u = rng.standard_normal(n**3) + 1j * rng.standard_normal(n**3)
    try:
        s = nls_amd.Solver(3, n, n, n, dx, dx, m=10, device=0, nranks=world, rank=rank, rccl_id=rid)
        P = n * n
        s.set_field(u[s.z0 * P:(s.z0 + s.nzl) * P])
        s.step(1e-3, 3)
        q.put((rank, s.z0, s.get_field()))
        s.close()
    except Exception as e:
        q.put((rank, -1, str(e)))

if __name__ == "__main__":
    import nls_amd, oracle_py as O
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    rid = nls_amd.rccl_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, rid, q)) for r in range(world)]
    [p.start() for p in ps]
    res = sorted([q.get(timeout=120) for _ in ps], key=lambda t: t[0])
    [p.join() for p in ps]
    if any(r[1] == -1 for r in res):
        print("FAILED", res); sys.exit(1)
    n, L = 16, 5.0; dx = 2 * L / (n - 1)
    rng = np.random.default_rng(0)
    u = rng.standard_normal(n**3) + 1j * rng.standard_normal(n**3)
    ref = O.nlse_steps(O.grid(3, n, n, n, dx, dx), u, 1e-3, 3, 10)
    got = np.concatenate([r[2] for r in res])
    print("rel err", np.linalg.norm(got - ref) / np.linalg.norm(ref))
