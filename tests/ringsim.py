"""Test helper: the reference's ring collectives, simulated in one process.

Restates /root/reference/src/core/reduce_scatter_ring.cpp:73-101 and
/root/reference/src/core/all_gather_ring.cpp:44-64 (with their rank maps) plus the API-level
compositions of /root/reference/src/core/all_reduce_ring.cpp:59-72 and dccl.cpp
(ncclReduceScatter :619-654, ncclReduce :787-840, ncclAllGather :849-862).  All ranks run step
s "at the same time": every send of step s reads the sender's buffer as it was after step s-1.
``combine(send, recv)`` is injected: the tests pass the oracle (CPU) or the HIP combine (GPU).
"""
from __future__ import annotations


def _clone(x):
    return x.clone() if hasattr(x, "clone") else x.copy()


def _chunk(buf, W, i):
    slot = buf.shape[0] // W
    i %= W
    return buf[i * slot:(i + 1) * slot]


def reduce_scatter_ring(bufs, combine, to_new=lambda r, W: r, to_old=lambda n, W: n):
    W = len(bufs)
    assert bufs[0].shape[0] % W == 0 and bufs[0].shape[0] >= W
    # rank (old) o has new rank to_new(o); it sends DATA(new - s) to to_old(new+1)
    for s in range(W - 1):
        inflight = {}
        for o in range(W):
            nr = to_new(o, W)
            inflight[to_old((nr + 1) % W, W)] = _clone(_chunk(bufs[o], W, nr - s))
        for o in range(W):
            nr = to_new(o, W)
            combine(inflight[o], _chunk(bufs[o], W, nr - s - 1))
    return bufs


def all_gather_ring(bufs, copy, to_new=lambda r, W: r, to_old=lambda n, W: n):
    W = len(bufs)
    for s in range(W - 1):
        inflight = {}
        for o in range(W):
            nr = to_new(o, W)
            inflight[to_old((nr + 1) % W, W)] = _clone(_chunk(bufs[o], W, nr - s))
        for o in range(W):
            nr = to_new(o, W)
            copy(_chunk(bufs[o], W, nr - s - 1), inflight[o])
    return bufs


def ring_allreduce(bufs, combine, copy):
    """all_reduce_ring: RS with identity maps, then AG with new rank = r + 1."""
    reduce_scatter_ring(bufs, combine)
    all_gather_ring(bufs, copy, to_new=lambda r, W: (r + 1) % W, to_old=lambda n, W: (n - 1) % W)
    return bufs


def rs_maps():
    """Rank maps ncclReduceScatter / ncclReduce pass (dccl.cpp:626-630): rank r ends with slot r."""
    return (lambda o, W: (o + W - 1) % W), (lambda n, W: (n + 1) % W)
