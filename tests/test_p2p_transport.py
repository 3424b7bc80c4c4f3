"""The collectives over a plugged-in point-to-point transport (dccl_comm_init_p2p, include/dccl/dccl_comm.h):
the branch RCCL takes, with the exchange written in Python here, so it runs at any W on one GPU (RCCL
itself needs one process per GPU, and this pool hands out one GPU per box).

The fake transport is a mailbox per (source, destination) shared by W thread-ranks.  Device buffers:
the exchange drains the caller's stream, copies the outgoing bytes into a fresh device tensor
(dccl_copy_multi) and lands incoming ones with the same copy, so the ring's next combine sees them.
Host buffers: plain memmove.

CPU: all_gather / broadcast on host buffers (no combine), the init argument checks and an exchange failure
reported by every collective.  GPU: all_reduce (ring and Rabenseifner), reduce_scatter, reduce, on device
and host buffers, bit-exact against tests/ringsim.py / tests/rabsim.py + the oracle: the API glue of
dccl_api.cpp (in-place copy, scratchpads, rank maps, gather to the root) around the gfx950 combine.
"""
import ctypes
import queue
import threading

import numpy as np
import pytest

import oracle
from tests import rabsim, ringsim


class Mailbox:
    def __init__(self, W, timeout=60.0):
        self.timeout = timeout
        self.q = {(a, b): queue.Queue() for a in range(W) for b in range(W)}
        self.calls = [[] for _ in range(W)]


def make_exchange(box, rank, device, fail_at=None):
    """`device`: this run's buffers (and so the library's scratchpads) live in device memory."""
    import dccl_amd

    def exchange(sbuf, sn, to, rbuf, rn, frm, stream):
        box.calls[rank].append((to if sbuf else None, frm if rbuf else None, sn, rn))
        if fail_at is not None and len(box.calls[rank]) == fail_at:
            return 2  # ncclSystemError from the transport
        if device:
            import torch
            if stream:
                torch.cuda.ExternalStream(stream).synchronize()
            if sbuf:
                t = torch.empty(sn, dtype=torch.uint8, device="cuda")
                assert dccl_amd.copy_multi([sbuf], [t.data_ptr()], sn, 0) == 0
                torch.cuda.synchronize()
                box.q[(rank, to)].put(t)
            if rbuf:
                t = box.q[(frm, rank)].get(timeout=box.timeout)
                if t.numel() != rn:
                    return 5
                assert dccl_amd.copy_multi([t.data_ptr()], [rbuf], rn, 0) == 0
                torch.cuda.synchronize()
        else:
            if sbuf:
                box.q[(rank, to)].put(ctypes.string_at(sbuf, sn))
            if rbuf:
                data = box.q[(frm, rank)].get(timeout=box.timeout)
                if len(data) != rn:
                    return 5
                ctypes.memmove(rbuf, data, rn)
        return 0
    return exchange


def run_p2p(W, body, memory=3, fail_at=None, timeout=60.0, device=False):
    import dccl_amd
    box = Mailbox(W, timeout)
    out, errs = [None] * W, []

    def worker(r):
        try:
            comm = dccl_amd.Comm.p2p(W, r, make_exchange(box, r, device, fail_at if r == 0 else None), memory)
            try:
                out[r] = body(comm, r)
            finally:
                comm.finalize()
        except Exception as e:  # reported below
            errs.append((r, repr(e)))

    ts = [threading.Thread(target=worker, args=(r,)) for r in range(W)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "a rank hung"
    assert not errs, errs
    return out, box


# ------------------------------------------------------------------------------------------- CPU
def test_p2p_init_argument_checks_cpu():
    import dccl_amd
    h = ctypes.c_void_p()
    fn = dccl_amd.P2P_EXCHANGE_FN(lambda *a: 0)
    assert dccl_amd.lib.dccl_comm_init_p2p(ctypes.byref(h), 2, 2, fn, None, 3) == 4   # rank >= world
    assert dccl_amd.lib.dccl_comm_init_p2p(ctypes.byref(h), 0, 0, fn, None, 3) == 4   # world 0
    assert dccl_amd.lib.dccl_comm_init_p2p(ctypes.byref(h), 2, 0, fn, None, 0) == 4   # no memory kind
    assert dccl_amd.lib.dccl_comm_init_p2p(ctypes.byref(h), 2, 0, fn, None, 4) == 4
    assert dccl_amd.lib.dccl_comm_init_p2p(ctypes.byref(h), 2, 0, dccl_amd.P2P_EXCHANGE_FN(), None, 3) == 4
    assert dccl_amd.lib.dccl_comm_init_p2p(None, 2, 0, fn, None, 3) == 4


@pytest.mark.parametrize("W", [2, 3, 5, 8])
def test_p2p_all_gather_and_broadcast_host_cpu(W):
    n = 1001

    def body(comm, r):
        send = (np.arange(n, dtype=np.int64) * (r + 7)).copy()
        recv = np.zeros(n * W, np.int64)
        assert comm.all_gather(send.ctypes.data, recv.ctypes.data, n, 4) == 0
        b = np.full(n, r, np.float32) if r != 1 % W else np.linspace(0, 1, n).astype(np.float32)
        assert comm.broadcast(b.ctypes.data, b.ctypes.data, n, 7, 1 % W) == 0
        return recv, b

    out, box = run_p2p(W, body)
    want = np.concatenate([np.arange(n, dtype=np.int64) * (r + 7) for r in range(W)])
    for r in range(W):
        assert np.array_equal(out[r][0], want)
        assert np.array_equal(out[r][1], np.linspace(0, 1, n).astype(np.float32))
    # the ring all-gather is W-1 exchanges per rank, then the broadcast one per peer (root) or one (others)
    for r in range(W):
        assert len(box.calls[r]) == (W - 1) + ((W - 1) if r == 1 % W else 1)


def test_p2p_device_memory_only_rejects_host_cpu():
    def body(comm, r):
        x = np.zeros(8, np.float32)
        return comm.all_gather(x.ctypes.data, np.zeros(16, np.float32).ctypes.data, 8, 7)

    out, _ = run_p2p(2, body, memory=2)
    assert out == [5, 5]  # ncclInvalidUsage: the transport moves device memory only


def test_p2p_transport_error_is_returned_cpu():
    """The exchange fails on rank 0's first call: rank 0 gets the transport's code back; its peer, whose
    receive then never arrives, fails its own exchange by timeout instead of hanging."""
    def body(comm, r):
        send = np.arange(8, dtype=np.int32)
        recv = np.zeros(16, np.int32)
        return comm.all_gather(send.ctypes.data, recv.ctypes.data, 8, 2)

    out, _ = run_p2p(2, body, fail_at=1, timeout=2.0)
    assert out[0] == 2 and out[1] == 2


# ------------------------------------------------------------------------------------------- GPU
def _inputs(W, n, dt, op, seed):
    return [oracle.synth(n, dt, op, seed, r) for r in range(W)]


def _combine(dt, op):
    def c(send, recv):
        assert oracle.expected_reduce(np.ascontiguousarray(send), recv, dt, op) == 0
    return c


def _copy(dst, src):
    dst[:] = src


@pytest.mark.gpu
@pytest.mark.parametrize("device", [True, False])
@pytest.mark.parametrize("algo", ["ring", "rabenseifner"])
@pytest.mark.parametrize("W,dt,op", [(2, 7, 0), (3, 7, 2), (4, 2, 0), (6, 9, 1), (8, 7, 0)])
def test_p2p_all_reduce(gpu, W, dt, op, algo, device, monkeypatch):
    import torch
    monkeypatch.setenv("DCCL_ALLREDUCE_ALGORITHM", algo)
    n = 840 * 37
    inputs = _inputs(W, n, dt, op, 11)
    want = [x.copy() for x in inputs]
    if algo == "ring":
        ringsim.ring_allreduce(want, _combine(dt, op), _copy)
    else:
        rabsim.rabenseifner_allreduce(want, _combine(dt, op))

    def body(comm, r):
        if device:
            st = torch.cuda.Stream()
            buf = torch.from_numpy(inputs[r].view(np.uint8).copy()).cuda()
            torch.cuda.synchronize()
            rc = comm.all_reduce(buf.data_ptr(), buf.data_ptr(), n, dt, op, st.cuda_stream)
            st.synchronize()
            return rc, buf.cpu().numpy().view(inputs[r].dtype)
        buf = inputs[r].copy()
        return comm.all_reduce(buf.ctypes.data, buf.ctypes.data, n, dt, op), buf

    out, _ = run_p2p(W, body, device=device)
    for r in range(W):
        assert out[r][0] == 0
        assert out[r][1].tobytes() == want[r].tobytes(), (r, algo, device)


@pytest.mark.gpu
@pytest.mark.parametrize("device", [True, False])
@pytest.mark.parametrize("W", [2, 3, 5])
def test_p2p_reduce_scatter_and_reduce(gpu, W, device):
    import torch
    dt, op, slot = 7, 0, 4099
    n = slot * W
    inputs = _inputs(W, n, dt, op, 12)
    work = [x.copy() for x in inputs]
    ringsim.reduce_scatter_ring(work, _combine(dt, op), *ringsim.rs_maps())
    want_slots = [work[r][r * slot:(r + 1) * slot] for r in range(W)]
    root = W - 1

    def body(comm, r):
        if device:
            st = torch.cuda.Stream()
            send = torch.from_numpy(inputs[r].copy()).cuda()
            recv = torch.zeros(slot, device="cuda")
            full = torch.zeros(n, device="cuda")
            torch.cuda.synchronize()
            rc1 = comm.reduce_scatter(send.data_ptr(), recv.data_ptr(), slot, dt, op, st.cuda_stream)
            rc2 = comm.reduce(send.data_ptr(), full.data_ptr(), n, dt, op, root, st.cuda_stream)
            st.synchronize()
            return rc1, rc2, recv.cpu().numpy(), full.cpu().numpy()
        send = inputs[r].copy()
        recv = np.zeros(slot, np.float32)
        full = np.zeros(n, np.float32)
        rc1 = comm.reduce_scatter(send.ctypes.data, recv.ctypes.data, slot, dt, op)
        rc2 = comm.reduce(send.ctypes.data, full.ctypes.data, n, dt, op, root)
        return rc1, rc2, recv, full

    out, _ = run_p2p(W, body, device=device)
    for r in range(W):
        rc1, rc2, recv, full = out[r]
        assert rc1 == 0 and rc2 == 0
        assert recv.tobytes() == want_slots[r].tobytes(), r
    assert out[root][3].tobytes() == np.concatenate(want_slots).tobytes()
