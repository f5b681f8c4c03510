"""Checks on the transport op log of a collective handle (nls_debug_oplog,
include/nls.h): the issue order the RCCL communicator sees.

Entries are (kind, stream, count, peer) with kind 1 all-reduce, 2 send, 3 recv,
4 the compute stream waits for the halo stream, 5 the halo stream waits for the
compute stream, 6 all-gather (the peer-store handshake), 7 the log was truncated
before this entry (NLS_OPLOG_MAX); stream 0 = compute, 1 = halo.

Two properties make one communicator safe without relying on RCCL to order its
operations across HIP streams:

* stream_order_violations: an operation on one stream is issued only after every
  earlier operation on the other stream is covered by a wait of this stream (so
  at no time are operations of both streams in flight on the communicator);
* rank_sequence_mismatches: every rank issues the same all-reduce sequence (kind,
  count), and every send a -> b is matched, in order and size, by a recv of b
  from a (the pairing ncclGroupStart/End needs to complete).
"""
from __future__ import annotations

ALLREDUCE, SEND, RECV, WAIT_HALO, WAIT_COMPUTE, ALLGATHER, DROPPED = 1, 2, 3, 4, 5, 6, 7
COMM_OPS = (ALLREDUCE, SEND, RECV, ALLGATHER)


def stream_order_violations(log):
    """Indices of communicator operations issued while an operation of the other
    stream was not yet ordered before them."""
    pending = [False, False]  # pending[s]: the other stream has unordered ops for s
    bad = []
    for i, (kind, stream, _count, _peer) in enumerate(log):
        if kind == DROPPED:  # nothing is known about what came before
            pending = [False, False]
        elif kind == WAIT_HALO:
            pending[0] = False
        elif kind == WAIT_COMPUTE:
            pending[1] = False
        elif kind in COMM_OPS:
            if pending[stream]:
                bad.append(i)
            pending[1 - stream] = True
    return bad


def truncated(log):
    """Entries dropped before the log's first one (its leading DROPPED entry), else 0."""
    return log[0][2] if log and log[0][0] == DROPPED else 0


def rank_sequence_mismatches(logs):
    """logs[r] = op log of rank r.  Returns a list of human-readable mismatches (a
    truncated log cannot be matched and is reported as such)."""
    out = [f"rank {r}: log truncated ({truncated(lg)} entries dropped)" for r, lg in enumerate(logs) if truncated(lg)]
    if out:
        return out
    ar = [[(k, c) for k, _s, c, _p in lg if k in (ALLREDUCE, ALLGATHER)] for lg in logs]
    for r in range(1, len(logs)):
        if ar[r] != ar[0]:
            out.append(f"rank {r} all-reduce sequence differs from rank 0 ({len(ar[r])} vs {len(ar[0])})")
    for a, lg in enumerate(logs):
        for b in range(len(logs)):
            if a == b:
                continue
            sends = [c for k, _s, c, p in lg if k == SEND and p == b]
            recvs = [c for k, _s, c, p in logs[b] if k == RECV and p == a]
            if sends != recvs:
                out.append(f"sends {a}->{b} {sends[:4]}... do not match recvs of {b} from {a} {recvs[:4]}...")
    return out
