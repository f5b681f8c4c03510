"""CPU: the op-log checks of tests/oplog_check.py on hand-written issue orders --
the two-vector pass of a split slab (boundary launch + exchange on the halo
stream, interior + all-reduce on the compute stream) with and without the wait
that orders the all-reduce after the exchange (the ADVICE r02 finding)."""
from oplog_check import (ALLREDUCE, DROPPED, RECV, SEND, WAIT_COMPUTE, WAIT_HALO, rank_sequence_mismatches,
                         stream_order_violations)


def _pass(rank, nranks, wait_before_allreduce=True, cnt=8192):
    """One split pass as nls_api.cpp run_lanczos2 issues it."""
    log = [(WAIT_COMPUTE, 1, 0, -1)]
    if rank > 0:
        log += [(SEND, 1, cnt, rank - 1), (RECV, 1, cnt, rank - 1)]
    if rank < nranks - 1:
        log += [(SEND, 1, cnt, rank + 1), (RECV, 1, cnt, rank + 1)]
    if wait_before_allreduce:
        log.append((WAIT_HALO, 0, 0, -1))
    log.append((ALLREDUCE, 0, 14, -1))
    return log


def test_ordered_split_pass_is_clean():
    for nranks in (2, 3, 8):
        logs = [_pass(r, nranks) * 3 for r in range(nranks)]
        assert all(not stream_order_violations(lg) for lg in logs)
        assert not rank_sequence_mismatches(logs)


def test_missing_wait_is_flagged():
    lg = _pass(1, 3, wait_before_allreduce=False)
    bad = stream_order_violations(lg)
    assert bad == [len(lg) - 1]  # the all-reduce while the exchange may be in flight


def test_unmatched_sends_are_flagged():
    logs = [_pass(r, 3) for r in range(3)]
    logs[2] = [e for e in logs[2] if not (e[0] == RECV and e[3] == 1)]
    assert rank_sequence_mismatches(logs)
    logs = [_pass(r, 2) for r in range(2)]
    logs[1] = logs[1] + [(ALLREDUCE, 0, 6, -1)]
    assert rank_sequence_mismatches(logs)


def test_next_pass_without_wait_compute_is_flagged():
    """The halo stream must wait for the compute stream (the all-reduce) before
    the next exchange."""
    lg = _pass(0, 2) + [e for e in _pass(0, 2) if e[0] != WAIT_COMPUTE]
    assert stream_order_violations(lg)


def test_truncated_log_is_reported_not_compared():
    """A log whose first entry is DROPPED (NLS_OPLOG_MAX exceeded) is reported as
    truncated instead of being compared entry by entry with the other ranks'."""
    full = [(ALLREDUCE, 0, 4, -1)] * 3
    cut = [(DROPPED, 0, 7, -1), (ALLREDUCE, 0, 4, -1)]
    assert rank_sequence_mismatches([full, full]) == []
    mism = rank_sequence_mismatches([full, cut])
    assert len(mism) == 1 and "truncated" in mism[0] and "7" in mism[0]
    assert stream_order_violations(cut) == []
