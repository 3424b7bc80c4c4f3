"""Test helper: the reference's Rabenseifner all-reduce, simulated in one process.

Restates /root/reference/src/core/all_reduce_recursive_halving_and_doubling.cpp:8-201 (fold of a
non-power-of-two world onto 2^k ranks, :37-67 rank maps, :72-151 pre-combine, :182-196 post),
/root/reference/src/core/reduce_scatter_recursive_halving.cpp:66-111 and
/root/reference/src/core/all_gather_recursive_doubling.cpp:48-76.  Every message of a step is taken
from the sender's buffer as it was before the step.  ``faithful=True`` keeps the reference's
all-gather step size fixed at one slice (its doubling is commented out, :85), which leaves blocks
undelivered once the subworld has 4 or more ranks; ``faithful=False`` moves 2^s slices at step s.
``combine(send, recv)`` applies recv = op(recv, send) in place.
"""
from __future__ import annotations


def _floor_log2(n: int) -> int:
    return n.bit_length() - 1


def _rev(x: int, nbits: int) -> int:
    r = 0
    for _ in range(nbits):
        r = (r << 1) | (x & 1)
        x >>= 1
    return r


def rabenseifner_allreduce(bufs, combine, faithful: bool = False):
    W = len(bufs)
    k = _floor_log2(W)
    sub = 1 << k
    rem = W - sub
    n = bufs[0].shape[0]
    assert n % sub == 0
    half = n // 2
    to_new = (lambda o: o // 2 if o < 2 * rem else o - rem)
    to_old = (lambda q: 2 * q if q < rem else q + rem)
    # pre-combine: leader 2i keeps op(L.first, F.first); follower 2i+1 computes op(F.second, L.second)
    for i in range(rem):
        L, F = bufs[2 * i], bufs[2 * i + 1]
        l_second, f_first = L[half:].copy(), F[:half].copy()
        combine(f_first, L[:half])
        combine(l_second, F[half:])
        L[half:] = F[half:]
    active = [o for o in range(W) if not (o < 2 * rem and o % 2 == 1)]
    # recursive halving reduce-scatter on the subworld
    region = {o: (0, n) for o in active}
    for s in range(k):
        msgs = {}
        for o in active:
            my = to_new(o)
            lo, hi = region[o]
            mid = (lo + hi) // 2
            keep, give = ((mid, hi), (lo, mid)) if (my >> s) & 1 else ((lo, mid), (mid, hi))
            msgs[to_old(my ^ (1 << s))] = bufs[o][give[0]:give[1]].copy()
            region[o] = keep
        for o in active:
            lo, hi = region[o]
            combine(msgs[o], bufs[o][lo:hi])
    # recursive doubling all-gather
    slice_ = n // sub
    block = {o: _rev(to_new(o), k) for o in active}
    for s in range(k):
        msgs = {}
        length = slice_ if faithful else slice_ << s
        for o in active:
            my = to_new(o)
            peer = to_old(my ^ (1 << (k - s - 1)))
            b = block[o] & ~((1 << s) - 1)
            block[o] = b
            msgs[peer] = (b * slice_, bufs[o][b * slice_:b * slice_ + length].copy())
        for o in active:
            start, data = msgs[o]
            bufs[o][start:start + data.shape[0]] = data
    # post: the leader hands the whole result to its follower
    for i in range(rem):
        bufs[2 * i + 1][:] = bufs[2 * i]
    return bufs
