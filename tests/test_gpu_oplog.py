"""GPU: the issue order of the transport operations of collective handles
(NLS_OPLOG=1, nls_debug_oplog) -- one communicator is never used from two HIP
streams at once, and every rank issues the matching sequence (tests/oplog_check.py).

Runs the slab decomposition through the in-process group (2-4 ranks; the same
issue points as the RCCL path: halo_planes / allreduce_sums in nls_api.cpp) and a
1-rank handle through a real RCCL communicator (NLS_FORCE_RCCL=1)."""
import numpy as np
import pytest

from oplog_check import ALLREDUCE, RECV, SEND, WAIT_HALO, rank_sequence_mismatches, stream_order_violations
from test_gpu_multirank import field, run_ranks

pytestmark = pytest.mark.gpu
nls_amd = pytest.importorskip("nls_amd")


@pytest.mark.parametrize("pass2", ["1", "0", "peer"], ids=["two_vector", "one_vector", "peer"])
@pytest.mark.parametrize("nranks", [2, 3, 4])
def test_slab_oplog_is_stream_ordered_and_rank_matched(monkeypatch, nranks, pass2):
    """peer: NLS_PEER=1, the passes' boundary planes go by peer stores; the only
    exchanges left are the start vectors' (one per step), all on the compute stream."""
    monkeypatch.setenv("NLS_OPLOG", "1")
    monkeypatch.setenv("NLS_PASS2", "1" if pass2 == "peer" else pass2)
    if pass2 == "peer":
        monkeypatch.setenv("NLS_PEER", "1")
    nx, ny, nz, m = 64, 16, 40, 12
    dx = 20.0 / 511
    P = nx * ny
    u0 = field(nx * ny * nz, seed=4)

    def mk(r, grp):
        return nls_amd.Solver(3, nx, ny, nz, dx, dx, m=m, device=0, nranks=nranks, rank=r, group=grp)

    def body(s):
        s.set_field(u0[s.z0 * P:(s.z0 + s.nzl) * P])
        s.step(1e-3, 3)
        s.sync()
        return s.z0, s.oplog()

    res = sorted(run_ranks(nranks, mk, body), key=lambda t: t[0])
    logs = [r[1] for r in res]
    for r, lg in enumerate(logs):
        kinds = [e[0] for e in lg]
        assert kinds.count(ALLREDUCE) >= 3 * (m // 2), f"rank {r}: too few all-reduces"
        assert SEND in kinds and RECV in kinds
        if pass2 == "peer":  # no halo stream: every transport op on the compute stream
            assert WAIT_HALO not in kinds and all(e[1] == 0 for e in lg)
            assert kinds.count(SEND) <= 2 * (3 + 1)  # set_field + one start vector per step
        else:
            assert WAIT_HALO in kinds
        bad = stream_order_violations(lg)
        assert not bad, f"rank {r}: unordered cross-stream ops at {bad[:5]}: {[lg[i] for i in bad[:5]]}"
    mism = rank_sequence_mismatches(logs)
    assert not mism, mism


def test_rccl_oplog_single_rank(monkeypatch):
    """A real RCCL communicator (1 rank): the all-reduces stay on the compute
    stream, ordered after the halo stream's work."""
    monkeypatch.setenv("NLS_OPLOG", "1")
    monkeypatch.setenv("NLS_FORCE_RCCL", "1")
    n, m = 16, 10
    dx = 20.0 / (n - 1)
    with nls_amd.Solver(3, n, n, n, dx, dx, m=m, device=0) as s:
        s.set_field(field(n ** 3, 9))
        s.step(1e-3, 2)
        s.sync()
        lg = s.oplog()
        assert s.comm_size() == (1, "rccl")
    assert any(e[0] == ALLREDUCE for e in lg)
    assert all(e[1] == 0 for e in lg if e[0] == ALLREDUCE)
    assert not stream_order_violations(lg)
    assert np.all([e[3] == -1 for e in lg if e[0] not in (SEND, RECV)])


def test_oplog_off_by_default():
    n = 16
    dx = 20.0 / (n - 1)
    with nls_amd.Solver(3, n, n, n, dx, dx, m=8, device=0) as s:
        s.set_field(field(n ** 3, 2))
        s.step(1e-3, 1)
        assert s.oplog() == []


def test_oplog_partial_drain(monkeypatch):
    """nls_debug_oplog with cap < n copies the oldest cap entries and keeps the rest:
    the two reads of one step's log concatenate to the log of an identical step."""
    import ctypes as C
    monkeypatch.setenv("NLS_OPLOG", "1")
    monkeypatch.setenv("NLS_FORCE_RCCL", "1")
    n = 16
    dx = 20.0 / (n - 1)
    u = field(n ** 3, 5)
    with nls_amd.Solver(3, n, n, n, dx, dx, m=8, device=0) as s:
        s.set_field(u)
        s.step(1e-3, 1)
        s.sync()
        full = s.oplog()
        assert len(full) >= 4
        s.set_field(u)
        s.step(1e-3, 1)
        s.sync()
        L = nls_amd.lib()
        cnt = C.c_uint64()
        buf = (C.c_int32 * 8)()
        assert L.nls_debug_oplog(s._h, buf, 2, C.byref(cnt)) == 0 and cnt.value == len(full)
        first = [tuple(buf[4 * i:4 * i + 4]) for i in range(2)]
        rest = s.oplog()
        assert first + rest == full


def test_oplog_truncation_is_marked(monkeypatch):
    """A log that outgrows NLS_OPLOG_MAX keeps the newest entries behind one leading
    NLS_OP_DROPPED entry that counts the dropped ones (a truncated log must
    not read as an ordering violation, nor as a complete log)."""
    import ctypes as C
    from oplog_check import DROPPED, truncated
    monkeypatch.setenv("NLS_OPLOG", "1")
    monkeypatch.setenv("NLS_FORCE_RCCL", "1")
    n = 8
    dx = 20.0 / (n - 1)
    L = nls_amd.lib()
    cnt = C.c_uint64()
    with nls_amd.Solver(3, n, n, n, dx, dx, m=4, device=0) as s:
        s.set_field(field(n ** 3, 6))
        total = 0
        for _ in range(200):
            s.step(1e-3, 500)
            s.sync()
            assert L.nls_debug_oplog(s._h, None, 0, C.byref(cnt)) == 0
            if cnt.value >= 65536:
                break
        s.step(1e-3, 50)
        s.sync()
        lg = s.oplog()
    assert len(lg) == 65536
    assert lg[0][0] == DROPPED and truncated(lg) > 0
    assert all(e[0] != DROPPED for e in lg[1:])
    assert not stream_order_violations(lg)
