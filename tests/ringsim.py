"""Test helper: the reference's ring all-reduce choreography, simulated in one process.

Restates /root/reference/src/core/reduce_scatter_ring.cpp:73-101 (identity rank maps, as
all_reduce_ring passes them, all_reduce_ring.cpp:59-61) and
/root/reference/src/core/all_gather_ring.cpp:44-64 with the +1 rank shift of
all_reduce_ring.cpp:70-72.  All ranks run step s "at the same time": every send of step s
reads the sender's buffer as it was after step s-1.  ``combine(send, recv)`` is injected:
the tests pass the oracle (CPU) or the HIP combine (GPU).
"""
from __future__ import annotations


def ring_allreduce(bufs, combine, copy):
    """bufs: list of W per-rank 1-D buffers (numpy arrays or tensors), reduced in place.

    combine(send_view, recv_view): recv_view = op(recv_view, send_view) in place.
    copy(dst_view, src_view): dst_view[:] = src_view.
    """
    W = len(bufs)
    n = bufs[0].shape[0]
    assert n % W == 0 and n >= W, "count must divide evenly (reduce_scatter_ring.cpp:53-58)"
    slot = n // W

    def chunk(r, i):
        i %= W
        return bufs[r][i * slot:(i + 1) * slot]

    # reduce-scatter: rank r sends DATA(r-s) to r+1, receives DATA_{r-1}(r-1-s) into its
    # scratchpad and combines it into DATA(r-s-1)
    for s in range(W - 1):
        inflight = [chunk(r, r - s).clone() if hasattr(chunk(r, r - s), "clone") else chunk(r, r - s).copy()
                    for r in range(W)]
        for r in range(W):
            scratch = inflight[(r - 1) % W]
            combine(scratch, chunk(r, r - s - 1))
    # all-gather with new rank r' = r+1: rank r receives DATA(r'-s-1) from r-1, sends DATA(r'-s)
    for s in range(W - 1):
        inflight = [chunk(r, (r + 1) - s).clone() if hasattr(bufs[r], "clone") else chunk(r, (r + 1) - s).copy()
                    for r in range(W)]
        for r in range(W):
            copy(chunk(r, (r + 1) - s - 1), inflight[(r - 1) % W])
    return bufs
