"""The collectives C-ABI (include/dccl/dccl_comm.h) driven from Python threads (ctypes drops the
GIL, so W threads really run W ranks concurrently).

CPU: transport + ring choreography on host buffers for the paths without a combine, and the
null-communicator contract.  GPU: all_reduce / reduce_scatter through the HIP combine on device
and host buffers, bit-exact against the ring simulation + oracle; the RCCL transport's
bootstrap / init / finalize at world size 1 (multi-rank RCCL needs one process per GPU: it runs in
bench.py on multi-GPU nodes).
"""
import threading

import numpy as np
import pytest

import oracle
from tests import ringsim


def run_ranks(W, body):
    import dccl_amd
    errs, out = [], [None] * W

    def worker(r):
        try:
            comm = dccl_amd.Comm.in_process(W, r)
            try:
                out[r] = body(comm, r)
            finally:
                comm.finalize()
        except Exception as e:  # pragma: no cover - reported below
            errs.append((r, repr(e)))

    ts = [threading.Thread(target=worker, args=(r,)) for r in range(W)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not errs, errs
    return out


def test_all_gather_host_threads_cpu():
    W, n = 3, 3 * 1001
    data = [np.arange(n, dtype=np.int64) * (r + 1) for r in range(W)]

    def body(comm, r):
        recv = np.zeros(n, np.int64)
        slot = n // W
        send = data[r][r * slot:(r + 1) * slot].copy()
        assert comm.all_gather(send.ctypes.data, recv.ctypes.data, slot, 4) == 0
        return recv

    out = run_ranks(W, body)
    slot = n // W
    want = np.concatenate([data[r][r * slot:(r + 1) * slot] for r in range(W)])
    for r in range(W):
        assert np.array_equal(out[r], want)


def test_null_comm_is_invalid_argument_cpu():
    import dccl_amd
    assert dccl_amd.lib.dccl_all_reduce(None, None, 4, 7, 0, None, None) == 4
    assert dccl_amd.lib.dccl_comm_finalize(None) == 4
    assert dccl_amd.lib.dccl_comm_init_rank(None, 2, 0) == 4


def _expected_allreduce(inputs, dt, op):
    bufs = [x.copy() for x in inputs]

    def combine(s, r):
        assert oracle.expected_reduce(np.ascontiguousarray(s), r, dt, op) == 0

    def copy(d, s):
        d[:] = s

    ringsim.ring_allreduce(bufs, combine, copy)
    return bufs


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["", "ring"])
@pytest.mark.parametrize("device", [True, False])
@pytest.mark.parametrize("W,dt,op", [(4, 7, 0), (3, 9, 1), (2, 2, 3), (5, 8, 2)])
def test_all_reduce_threads(W, dt, op, device, algo, monkeypatch):
    """Thread ranks, bit-exact against the ring simulation + oracle.  algo "" is the default (the direct
    collectives: peer reads on device buffers, one staged chain combine per rank on host buffers);
    "ring" forces the ring."""
    import torch
    monkeypatch.setenv("DCCL_ALLREDUCE_ALGORITHM", algo)
    rng = np.random.default_rng(W * 10 + dt)
    n = W * 40961
    npd = oracle.NP_DTYPES[dt]
    if dt == 9:
        inputs = [torch.randn(n).bfloat16().view(torch.int16).numpy().view(np.uint16) for _ in range(W)]
    elif np.issubdtype(npd, np.integer):
        inputs = [rng.integers(-1000, 1000, n).astype(npd) for _ in range(W)]
    else:
        inputs = [rng.standard_normal(n).astype(npd) for _ in range(W)]
    want = _expected_allreduce(inputs, dt, op)

    def body(comm, r):
        if device:
            st = torch.cuda.Stream()
            buf = torch.from_numpy(inputs[r].view(np.uint8).copy()).cuda()
            torch.cuda.synchronize()
            assert comm.all_reduce(buf.data_ptr(), buf.data_ptr(), n, dt, op, st.cuda_stream) == 0
            st.synchronize()
            return buf.cpu().numpy().view(npd)
        buf = inputs[r].copy()
        assert comm.all_reduce(buf.ctypes.data, buf.ctypes.data, n, dt, op) == 0
        return buf

    out = run_ranks(W, body)
    for r in range(W):
        assert out[r].tobytes() == want[r].tobytes(), r


@pytest.mark.gpu
@pytest.mark.slow
def test_all_reduce_threads_host_large():
    """Host buffers beyond one staging area: the direct all_reduce stages each rank's chain in pieces
    (W = 4, 18 MiB chunks, W copies > 64 MiB); bit-exact against the ring simulation + oracle."""
    W, dt, op = 4, 7, 0
    n = W * ((18 << 20) // 4 + 37)
    rng = np.random.default_rng(77)
    inputs = [rng.standard_normal(n).astype(np.float32) for _ in range(W)]
    want = _expected_allreduce(inputs, dt, op)

    def body(comm, r):
        buf = inputs[r].copy()
        assert comm.all_reduce(buf.ctypes.data, buf.ctypes.data, n, dt, op) == 0
        return buf

    out = run_ranks(W, body)
    for r in range(W):
        assert out[r].tobytes() == want[r].tobytes(), r


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["", "ring"])
def test_reduce_scatter_threads_device(algo, monkeypatch):
    import torch
    monkeypatch.setenv("DCCL_ALLREDUCE_ALGORITHM", algo)
    W, slot, dt, op = 4, 65537, 7, 0
    rng = np.random.default_rng(3)
    inputs = [rng.standard_normal(W * slot).astype(np.float32) for _ in range(W)]
    work = [x.copy() for x in inputs]

    def combine(s, r):
        assert oracle.expected_reduce(np.ascontiguousarray(s), r, dt, op) == 0

    ringsim.reduce_scatter_ring(work, combine, *ringsim.rs_maps())

    def body(comm, r):
        st = torch.cuda.Stream()
        send = torch.from_numpy(inputs[r]).cuda()
        recv = torch.zeros(slot, device="cuda")
        torch.cuda.synchronize()
        assert comm.reduce_scatter(send.data_ptr(), recv.data_ptr(), slot, dt, op, st.cuda_stream) == 0
        st.synchronize()
        return recv.cpu().numpy()

    out = run_ranks(W, body)
    for r in range(W):
        assert out[r].tobytes() == work[r][r * slot:(r + 1) * slot].tobytes(), r


@pytest.mark.gpu
def test_rccl_transport_world1():
    import torch
    import dccl_amd
    if not dccl_amd.lib.dccl_rccl_available():
        pytest.skip("librccl not loadable")
    uid = dccl_amd.Comm.unique_id()
    comm = dccl_amd.Comm.rccl(1, 0, uid)
    try:
        x = torch.arange(1024, dtype=torch.float32, device="cuda")
        y = torch.zeros_like(x)
        assert comm.all_reduce(x.data_ptr(), y.data_ptr(), 1024, 7, 0) == 0
        g = torch.zeros_like(x)
        assert comm.all_gather(x.data_ptr(), g.data_ptr(), 1024, 7) == 0
        torch.cuda.synchronize()
        assert torch.equal(y, x) and torch.equal(g, x)
        h = np.zeros(4, np.float32)  # the RCCL transport moves device memory only
        assert comm.all_reduce(h.ctypes.data, h.ctypes.data, 4, 7, 0) == 5
    finally:
        assert comm.finalize() == 0
