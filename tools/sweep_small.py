"""Tile-depth / graph-replay sweep over grid sizes (one process, GPU).

For each (dim, n, kz, graph): create a cubic-NLSE handle (m = 16) with
NLS_KZ / NLS_KZ_ALPHA / NLS_GRAPH set, warm up, time K steps with a host clock
around nls_sync.  Prints one JSON line per config.  Usage:
    python tools/sweep_small.py [--dims 2,3] [--kz 1,2,4,8,16,32] [--graph 0,1]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nonlinear-solvers_amd"))
import nls_amd  # noqa: E402

SIZES = {2: [128, 256, 512, 1024, 2048], 3: [32, 64, 96, 128, 192, 256]}


def run(dim, n, kz, graph, m, kz_alpha=None):
    os.environ["NLS_KZ"] = str(kz)
    os.environ["NLS_KZ_ALPHA"] = str(kz_alpha if kz_alpha else kz)
    os.environ["NLS_GRAPH"] = str(graph)
    cells = n ** dim
    dx = 20.0 / (n - 1)
    rng = np.random.default_rng(0)
    u = (rng.standard_normal(cells) + 1j * rng.standard_normal(cells)) * 0.1
    nz = n if dim == 3 else 1
    with nls_amd.Solver(dim, n, n, nz, dx, dx, m=m) as s:
        s.set_field(u)
        s.step(1e-4, 3)
        s.sync()
        est = max(1e-3, cells * 2700 / 5e12)
        k = int(min(400, max(20, 0.4 / est)))
        t0 = time.perf_counter()
        s.step(1e-4, k)
        s.sync()
        t = (time.perf_counter() - t0) / k
        out = s.get_field()
    assert np.all(np.isfinite(out))
    return dict(dim=dim, n=n, kz=kz, kz_alpha=kz_alpha or kz, graph=graph, m=m, steps=k, ms=t * 1e3,
                mcells=cells / t / 1e6)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dims", default="2,3")
    ap.add_argument("--kz", default="1,2,4,8,16,32")
    ap.add_argument("--graph", default="0,1")
    ap.add_argument("--kza", default="same", help="alpha tile depths, or 'same' (= kz)")
    ap.add_argument("--m", type=int, default=16)
    ap.add_argument("--sizes", default=None, help="override sizes, e.g. 2:256,512;3:128")
    a = ap.parse_args()
    sizes = dict(SIZES)
    if a.sizes:
        sizes = {}
        for part in a.sizes.split(";"):
            d, lst = part.split(":")
            sizes[int(d)] = [int(x) for x in lst.split(",")]
    for dim in [int(d) for d in a.dims.split(",")]:
        for n in sizes.get(dim, []):
            for kz in [int(k) for k in a.kz.split(",")]:
                if dim == 2 and kz > 16:
                    continue
                kzas = [None] if a.kza == "same" else [int(x) for x in a.kza.split(",")]
                for kza in kzas:
                    for g in [int(x) for x in a.graph.split(",")]:
                        print(json.dumps(run(dim, n, kz, g, a.m, kza)), flush=True)


if __name__ == "__main__":
    main()
