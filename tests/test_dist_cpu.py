"""world_size 2 / 3 gloo tests of the N > 1 path, on CPU.

What runs on N GPUs is (a) bench.py's host orchestration -- RCCL id broadcast,
per-rank slab of the synthetic input, global mass normalisation, barrier and
max-over-ranks timing -- and (b) the library's slab decomposition with halo
exchange and all-reduced dots.  (a) is exercised here with the real bench.py
helpers over gloo; (b) with tests/dist_model.py, a numpy restatement of the same
data movement (ghost planes, one-plane halos incl. the 3D y-wrap, split
reductions) whose gathered result must equal the single-process oracle.  The
GPU implementation of (b) is tested against the oracle in
tests/test_gpu_multirank.py (in-process ranks, RCCL collective path).
"""
import json
import os
import socket
import tempfile

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, case, outdir):
    import dist_model as DM  # noqa: F401  (sets sys.path)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {}
        if case["kind"] == "nlse":
            import oracle_py as O
            dim, n, m, dt, steps = case["dim"], case["n"], case["m"], case["dt"], case["steps"]
            L = 10.0
            dx = 2 * L / (n - 1)
            sl = DM.Slab(dim, n, n, n, dx, dx, rank, world)
            N = n ** dim
            rng = np.random.default_rng(5)
            u = rng.standard_normal(N) + 1j * rng.standard_normal(N)
            u_loc = u[sl.z0 * sl.P:(sl.z0 + sl.nzl) * sl.P]
            # one stencil application with halos == the oracle operator
            lap = DM.gather(sl, sl.lap(sl.ext(u_loc)))
            out = DM.gather(sl, DM.nlse_steps_dist(sl, u_loc, dt, steps, m))
            if rank == 0:
                g = O.grid(dim, n, n, n, dx, dx)
                res["lap"] = float(np.linalg.norm(lap - O.laplacian_c(g, u)) / np.linalg.norm(O.laplacian_c(g, u)))
                ref = O.nlse_steps(g, u, dt, steps, m)
                res["traj"] = float(np.linalg.norm(out - ref) / np.linalg.norm(ref))
        else:  # bench.py orchestration helpers
            import bench
            w = dict(bench.WORKLOADS[case["workload"]])
            w["n"] = case["n"]
            import nls_amd
            npl = w["n"]
            z0, nzl = nls_amd.slab_planes(npl, world, rank)
            u = bench.synthetic_ic(w, z0, nzl)
            dx = 2 * w["L"] / (w["n"] - 1)
            mass = bench.global_mass(u, dx ** w["dim"], dist)
            full = DM.gather(DM.Slab(w["dim"], w["n"], w["n"], w["n"], dx, dx, rank, world), u)
            el = bench.max_over_ranks(0.1 * (rank + 1), dist)
            if rank == 0:
                ref = bench.synthetic_ic(w, 0, npl)
                res["ic_equal"] = bool(np.array_equal(full, ref))
                res["mass"] = float(abs(mass - np.sum(np.abs(ref) ** 2) * dx ** w["dim"]) / mass)
                res["max"] = el
        if rank == 0:
            with open(os.path.join(outdir, "res.json"), "w") as f:
                json.dump(res, f)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run(world, case):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), case, d), nprocs=world, join=True,
                           start_method="spawn")
        with open(os.path.join(d, "res.json")) as f:
            return json.load(f)


@pytest.mark.parametrize("world,dim,n", [(2, 3, 10), (3, 3, 11), (2, 2, 24), (3, 2, 17)])
def test_slab_decomposition_matches_single_process_oracle(world, dim, n):
    """Halo planes (incl. the 3D y-wrap across slab boundaries) and all-reduced
    dots reproduce the single-process operator and a 3-step SS2 trajectory."""
    r = _run(world, dict(kind="nlse", dim=dim, n=n, m=10, dt=1e-3, steps=3))
    assert r["lap"] <= 1e-15
    assert r["traj"] <= 1e-12


@pytest.mark.parametrize("world", [2, 3])
def test_bench_orchestration_over_gloo(world):
    """bench.py N>1 host logic: slab ICs concatenate to the single-rank IC, the
    mass normalisation is global, the timing is the max over ranks."""
    r = _run(world, dict(kind="bench", workload="nlse3d_512", n=20))
    assert r["ic_equal"]
    assert r["mass"] < 1e-14
    assert abs(r["max"] - 0.1 * world) < 1e-12


def test_bench_launcher_command_line():
    """`python bench.py --gpus N` without torch.distributed.run re-launches itself
    as N ranks with the driver's own launcher line (127.0.0.1 rendezvous)."""
    import bench
    cmd = bench.rank_launch_cmd(4, ["--gpus", "4", "--steps", "3"], 29555)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert "--master-port=29555" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_bench_launcher_forwards_rank0_line(tmp_path, monkeypatch):
    """launch_ranks runs a real torch.distributed.run with 2 gloo ranks (a stand-in
    script for bench.py: no GPU here) and forwards only rank 0's JSON line; the
    children see WORLD_SIZE / RANK / MASTER_ADDR from the launcher."""
    import sys
    import bench
    script = tmp_path / "fake_bench.py"
    script.write_text(
        "import json, os\n"
        "import torch.distributed as dist\n"
        "dist.init_process_group('gloo')\n"
        "r, w = dist.get_rank(), dist.get_world_size()\n"
        "assert os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
        "dist.barrier()\n"
        "if r == 0:\n"
        "    print('banner line on stdout')\n"
        "    print(json.dumps({'metric': 'x', 'value': 1.0, 'n_gpus': w}))\n"
        "dist.destroy_process_group()\n")
    real = bench.rank_launch_cmd

    def fake_cmd(n, argv, port):
        cmd = real(n, argv, port)
        i = cmd.index(os.path.abspath(bench.__file__))
        return cmd[:i] + [str(script)]
    monkeypatch.setattr(bench, "rank_launch_cmd", fake_cmd)
    rc, line = bench.launch_ranks(2, [])
    assert rc == 0
    assert json.loads(line) == {"metric": "x", "value": 1.0, "n_gpus": 2}


def test_bench_selfcheck_env_and_command():
    """The N > 1 self-check job: its launcher line and an environment without the
    parent launcher's per-rank variables (the child's own launcher sets them)."""
    import argparse
    import bench
    env = {"RANK": "1", "LOCAL_RANK": "1", "WORLD_SIZE": "8", "MASTER_PORT": "1", "MASTER_ADDR": "x",
           "TORCHELASTIC_RUN_ID": "r", "NLS_PEER": "1", "PATH": "/bin", "OMP_NUM_THREADS": "16"}
    e = bench.selfcheck_env(env)
    assert e["PATH"] == "/bin" and e["OMP_NUM_THREADS"] == "16" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert not any(k in e for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT", "MASTER_ADDR",
                                    "TORCHELASTIC_RUN_ID", "NLS_PEER"))
    a = argparse.Namespace(workload="nlse3d_512", n=None, m=None)
    cmd = bench.selfcheck_cmd(8, a, "/tmp/x.json", 29600)
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29600" in cmd
    i = cmd.index("--selfcheck-json")
    assert cmd[i + 1] == "/tmp/x.json" and cmd[cmd.index("--gpus") + 1] == "8"


def test_bench_choose_exchange():
    """Peer stores only when their field check passed, they actually ran and were faster."""
    import bench
    ok = {"default": {"ok": True}, "peer": {"ok": True, "state": "active"}}
    assert bench.choose_exchange(dict(ok, ab={"default_ms": 4.4, "peer_ms": 4.1})) == "peer"
    assert bench.choose_exchange(dict(ok, ab={"default_ms": 4.0, "peer_ms": 4.1})) == "default"
    assert bench.choose_exchange(dict(ok, ab={"default_ms": 4.4})) == "default"
    bad = {"default": {"ok": True}, "peer": {"ok": False, "state": "active"}, "ab": {"default_ms": 4.4, "peer_ms": 1}}
    assert bench.choose_exchange(bad) == "default"
    fb = {"default": {"ok": True}, "peer": {"ok": True, "state": "fell_back"}, "ab": {"default_ms": 4.4, "peer_ms": 1}}
    assert bench.choose_exchange(fb) == "default"
    assert bench.choose_exchange({"default": {"ok": False}, "peer": {"ok": False}, "error": "x"}) == "default"


def test_bench_selfcheck_job_over_gloo(monkeypatch):
    """run_selfcheck starts the real child job (torch.distributed.run, 2 gloo ranks,
    bench.py --selfcheck-json) and reads its report; NLS_BENCH_SELFCHECK_DRY=1 swaps the
    device legs for the same gather / compare plumbing on a synthetic field (no GPU here)."""
    import argparse
    import bench
    monkeypatch.setenv("NLS_BENCH_SELFCHECK_DRY", "1")
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    a = argparse.Namespace(workload="nlse3d_512", n=None, m=None)
    rep = bench.run_selfcheck(2, a)
    assert rep["child_rc"] == 0, rep
    assert rep["n_ranks"] == 2
    for leg in ("default", "peer"):
        assert rep[leg]["ok"] and rep[leg]["rel_l2_vs_1rank"] == 0.0 and rep[leg]["comm_count"] == [2, 2]
    assert bench.choose_exchange(rep) == "peer"


def test_bench_selfcheck_job_failure_reported(monkeypatch):
    """A child job that dies leaves the default exchange and a report saying so."""
    import argparse
    import bench
    monkeypatch.setattr(bench, "selfcheck_cmd", lambda n, args, path, port: ["false"])
    rep = bench.run_selfcheck(2, argparse.Namespace(workload="nlse3d_512", n=None, m=None))
    assert rep["child_rc"] == 1 and "error" in rep
    assert bench.choose_exchange(rep) == "default"


def test_bench_selfcheck_timeout_kills_the_job(monkeypatch, tmp_path):
    """A hung self-check job is killed with its whole process group at the timeout."""
    import argparse
    import bench
    marker = tmp_path / "child_pid"
    script = f"import os, time; open({str(marker)!r}, 'w').write(str(os.getpid())); time.sleep(60)"
    import sys
    monkeypatch.setattr(bench, "selfcheck_cmd",
                        lambda n, args, path, port: ["bash", "-c", f"{sys.executable} -c \"{script}\" & wait"])
    monkeypatch.setattr(bench, "SELFCHECK_TIMEOUT", 3)
    rep = bench.run_selfcheck(2, argparse.Namespace(workload="nlse3d_512", n=None, m=None))
    assert rep["child_rc"] == "timeout" and bench.choose_exchange(rep) == "default"
    pid = int(marker.read_text())
    import time
    time.sleep(0.5)
    assert not os.path.exists(f"/proc/{pid}") or open(f"/proc/{pid}/stat").read().split()[2] == "Z"
