"""The decompositions of the driver's scaling bench (`bench.py --gpus N`, N = 2, 4, 8:
3D cubic NLSE 512^3, Krylov m=16, z-slabs of 256 / 128 / 64 planes) on one GPU.

The N ranks are handles of one process (nls_group local transport): the same slab
layout, two ghost planes, boundary/interior launch split of the two-vector passes
and per-rank fixed-order reductions as the RCCL path, only the byte mover differs.
The 512^3 oracle does not finish in seconds, so parity is through properties:

  * N slabs equal one rank to rounding (<= 1e-12 rel-L2; only the reduction order
    differs) after two SS2 steps at the bench's spacing dx = 20/511;
  * an exactly x-mirror-symmetric field stays bitwise x-symmetric on N slabs;
  * the cubic step is unitary on N slabs (<= 1e-12).

Reference: nlse_solver.hpp:53-77 (SS2), eigen_krylov_complex.hpp:10-84.
"""
import threading

import numpy as np
import pytest

from conftest import rel_l2

pytestmark = pytest.mark.gpu
nls_amd = pytest.importorskip("nls_amd")

N, M, DT, STEPS = 512, 16, 1e-3, 2
DX = 20.0 / (N - 1)


@pytest.fixture(scope="module")
def field_and_single():
    rng = np.random.default_rng(11)
    x = np.linspace(-10, 10, N)
    u = np.zeros((N, N, N), np.complex128)
    for _ in range(3):
        cx, cy, cz = rng.uniform(1, 5), rng.uniform(-5, 5), rng.uniform(-5, 5)
        ky = rng.uniform(-1, 1)
        fx = np.exp(-((x - cx) ** 2) / 2) + np.exp(-((x + cx) ** 2) / 2)
        fx = 0.5 * (fx + fx[::-1])
        fy = np.exp(-((x - cy) ** 2) / 2 + 1j * ky * x)
        fz = np.exp(-((x - cz) ** 2) / 2)
        u += fz[:, None, None] * np.outer(fy, fx)[None]
    half = N // 2
    noise = 1e-3 * (rng.standard_normal((N, N, half)) + 1j * rng.standard_normal((N, N, half)))
    u += np.concatenate([noise, noise[:, :, ::-1]], axis=2)
    del noise
    u /= np.sqrt(np.sum(np.abs(u) ** 2) * DX ** 3)
    u0 = u.reshape(-1)
    with nls_amd.Solver(3, N, N, N, DX, DX, m=M) as s:
        s.set_field(u0)
        s.step(DT, STEPS)
        single = s.get_field()
    return u0, single


@pytest.mark.parametrize("nr", [2, 4, 8])
def test_bench_slabs_match_single_rank(field_and_single, nr):
    u0, single = field_and_single
    grp = nls_amd.Group(nr)
    out = np.empty_like(u0)
    P = N * N
    err, planes, comm = [], [], []

    def work(r):
        try:
            with nls_amd.Solver(3, N, N, N, DX, DX, m=M, device=0, nranks=nr, rank=r, group=grp) as s:
                planes.append(s.nzl)
                comm.append(s.comm_size())
                sl = slice(s.z0 * P, (s.z0 + s.nzl) * P)
                s.set_field(u0[sl])
                s.step(DT, STEPS)
                out[sl] = s.get_field()
        except Exception as e:  # noqa: BLE001
            err.append((r, e))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(nr)]
    [t.start() for t in ts]
    [t.join(timeout=300) for t in ts]
    grp.close()
    assert not err, err
    assert sorted(planes) == [N // nr] * nr
    assert comm == [(nr, "group")] * nr  # the transport's own rank count (nls_comm_size)
    a3 = out.reshape(N, N, N)
    assert np.array_equal(a3, a3[:, :, ::-1]), f"{nr} slabs lost the exact x-mirror symmetry"
    assert abs(np.linalg.norm(out) / np.linalg.norm(u0) - 1.0) < 1e-12
    e = rel_l2(out, single)
    assert e <= 1e-12, f"{nr} slabs vs 1 rank rel-L2 {e:.3e}"
