"""Direct (peer-read) collectives, DESIGN.md §7.3.

GPU: the chain combine (dccl_local_reduce_chain) against the oracle applied in the ring's order,
the multi-source copy, the direct collectives of in-process ranks (threads on one GPU) against the
ring simulation + oracle (bit-exact), and the cross-process IPC transport with 2-4 processes
sharing the box's GPU.  CPU: argument checks of the new entry points.
"""
import multiprocessing as mp
import os
import sys
import threading
import uuid

import numpy as np
import pytest

import oracle
from tests import ringsim

SEED = 0xDCC1


def chain_expected(sends, own, dt, op):
    acc = np.array(sends[0], copy=True)
    for s in sends[1:]:
        acc = oracle.combine(acc, s, dt, op)  # op(recv = s, send = acc)
    return oracle.combine(acc, own, dt, op)   # op(recv = own, send = acc)


def test_chain_and_copy_argument_checks_cpu():
    import dccl_amd
    assert dccl_amd.local_reduce_chain([], 0, 0, 7, 16, 0) == 4           # nsend 0
    assert dccl_amd.local_reduce_chain([0] * 9, 0, 0, 7, 16, 0) == 4      # nsend 9
    assert dccl_amd.local_reduce_chain([8], 8, 8, 7, 16, 4) == 5          # Avg
    assert dccl_amd.local_reduce_chain([8], 8, 8, 11, 16, 0) == 4         # dtype
    assert dccl_amd.local_reduce_chain([8], 8, 8, 7, 0, 0) == 0           # count 0
    assert dccl_amd.local_reduce_chain([0], 8, 8, 7, 16, 0) == 4          # NULL send
    assert dccl_amd.copy_multi([0] * 9, [0] * 9, 16) == 4
    assert dccl_amd.copy_multi([], [], 16) == 0
    assert dccl_amd.copy_multi([0], [8], 16) == 4


def test_ipc_comm_rejects_bad_rank_cpu():
    import ctypes
    import dccl_amd
    h = ctypes.c_void_p()
    assert dccl_amd.lib.dccl_comm_init_ipc(ctypes.byref(h), 2, 2) == 4
    assert dccl_amd.lib.dccl_comm_init_ipc(ctypes.byref(h), 0, 0) == 4
    assert dccl_amd.lib.dccl_comm_init_ipc(None, 2, 0) == 4


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("dt", [0, 2, 6, 7, 8, 9])
def test_chain_host_against_oracle(gpu, dt):
    """dccl_local_reduce_chain_host: pageable and registered operands, own == dst and own != dst, odd
    sizes, and operands larger than one staging half (several double-buffered pieces)."""
    import dccl_amd
    from tests.test_gpu_parity import rand_inputs
    from tests.test_oracle import fp_equal
    rng = np.random.default_rng(50 + dt)
    for op in (0, 1, 2, 3):
        for k, n, pinned, same in ((1, 1, False, True), (3, 4099, False, True), (7, 65537, False, False),
                                   (2, 1000, True, True), (4, 30001, True, False)):
            arrs = [rand_inputs(rng, dt, n)[0] for _ in range(k + 1)]
            sends, own = arrs[:k], arrs[k].copy()
            want = chain_expected(sends, arrs[k], dt, op)
            dst = own if same else np.zeros_like(own)
            regs = (sends + [own] + ([] if same else [dst])) if pinned else []
            for x in regs:
                assert dccl_amd.register_host_memory(x.ctypes.data, x.nbytes) == 0
            try:
                assert dccl_amd.local_reduce_chain_host([s.ctypes.data for s in sends], own.ctypes.data,
                                                        dst.ctypes.data, dt, n, op) == 0
            finally:
                for x in regs:
                    dccl_amd.deregister_host_memory(x.ctypes.data)
            assert fp_equal(dst, want, dt), (op, k, n, pinned, same)
            if not same:
                assert own.tobytes() == arrs[k].tobytes()
    # 3 sends + own of 21 MiB + 5 elements: 8 MiB staging slots per half, 3 pieces; one send registered
    n = (21 << 20) // 4 + 5
    arrs = [rng.standard_normal(n).astype(np.float32) for _ in range(4)]
    want = chain_expected(arrs[:3], arrs[3], 7, 0)
    own = arrs[3].copy()
    assert dccl_amd.register_host_memory(arrs[1].ctypes.data, arrs[1].nbytes) == 0
    try:
        assert dccl_amd.local_reduce_chain_host([a.ctypes.data for a in arrs[:3]], own.ctypes.data, own.ctypes.data,
                                                7, n, 0) == 0
    finally:
        dccl_amd.deregister_host_memory(arrs[1].ctypes.data)
    assert own.tobytes() == want.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("dt", list(range(10)))
def test_chain_against_oracle(gpu, dt):
    import torch
    import dccl_amd
    from tests.test_gpu_parity import rand_inputs
    rng = np.random.default_rng(dt)
    esz = dccl_amd.size_of_type(dt)
    for op in (0, 1, 2, 3):
        for k, n, off in ((1, 1, 0), (2, 17, 0), (3, 4099, 0), (7, 65537, 0), (8, 1000, 0), (4, 3001, 4),
                          (5, 777, 2 * esz)):
            arrs = [rand_inputs(rng, dt, n)[0] for _ in range(k + 1)]
            sends, own = arrs[:k], arrs[k]
            want = chain_expected(sends, own, dt, op)
            dev = [torch.from_numpy(a.view(np.uint8).copy()).cuda() for a in sends]
            # own and dst in one buffer at `off` bytes; sends at the same 16-B phase only when off % 16 == 0
            t_own = torch.zeros(n * esz + off + 64, dtype=torch.uint8, device="cuda")
            t_own[off:off + n * esz].copy_(torch.from_numpy(own.view(np.uint8).copy()))
            p_own = t_own.data_ptr() + off
            assert dccl_amd.local_reduce_chain([d.data_ptr() for d in dev], p_own, p_own, dt, n, op) == 0
            got = t_own[off:off + n * esz].cpu().numpy().view(own.dtype)
            torch.cuda.synchronize()
            ok = got.tobytes() == want.tobytes()
            if not ok and dt in (6, 7, 8, 9):  # NaN payloads are not pinned
                from tests.test_oracle import fp_equal
                ok = fp_equal(got, want, dt)
            assert ok, (op, k, n, off)
            # separate dst: own untouched
            t_dst = torch.zeros(n * esz + off + 64, dtype=torch.uint8, device="cuda")
            t_own[off:off + n * esz].copy_(torch.from_numpy(own.view(np.uint8).copy()))
            assert dccl_amd.local_reduce_chain([d.data_ptr() for d in dev], p_own, t_dst.data_ptr() + off, dt, n,
                                               op) == 0
            torch.cuda.synchronize()
            assert t_own[off:off + n * esz].cpu().numpy().tobytes() == own.tobytes()
            assert (t_dst[off:off + n * esz].cpu().numpy().view(own.dtype).tobytes() == got.tobytes())


@pytest.mark.gpu
@pytest.mark.parametrize("dt", list(range(10)))
def test_chain_mixed_phases(gpu, dt):
    """Sends, own and dst each at their own element-aligned 16-B / 128-B phase (the phased chain kernel)."""
    import dccl_amd
    from tests.test_gpu_parity import rand_inputs, dev_bytes, host_of
    from tests.test_oracle import fp_equal
    rng = np.random.default_rng(500 + dt)
    esz = dccl_amd.size_of_type(dt)
    for k, n in ((1, 3), (2, 63), (3, 4099), (5, 65539), (7, 1000), (8, 20001)):
        op = int(rng.integers(0, 4))
        arrs = [rand_inputs(rng, dt, n)[0] for _ in range(k + 1)]
        sends, own = arrs[:k], arrs[k]
        want = chain_expected(sends, own, dt, op)
        offs = [int(rng.integers(0, 256 // esz)) * esz for _ in range(k + 2)]
        offs[0] = (offs[0] // 16) * 16 + (esz if esz < 16 else 0)
        dev = [dev_bytes(a, o) for a, o in zip(sends, offs)]
        t_own, p_own = dev_bytes(own, offs[k])
        t_dst, p_dst = dev_bytes(np.zeros_like(own), offs[k + 1])
        assert dccl_amd.local_reduce_chain([d[1] for d in dev], p_own, p_dst, dt, n, op) == 0
        import torch
        torch.cuda.synchronize()
        got = host_of(t_dst, offs[k + 1], own)
        assert fp_equal(got, want, dt), (op, k, n, offs)
        assert host_of(t_own, offs[k], own).tobytes() == own.tobytes()
        # in place: own == dst at its own phase, the sends at theirs
        assert dccl_amd.local_reduce_chain([d[1] for d in dev], p_own, p_own, dt, n, op) == 0
        torch.cuda.synchronize()
        assert fp_equal(host_of(t_own, offs[k], own), want, dt), (op, k, n, offs, "in place")


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [2, 4, 6, 7, 8, 9])
def test_chain_byte_offsets(gpu, dt):
    """Sends and own at any byte address (phased chain kernel with byte phases) into a dst that is
    element-aligned or not (reduce_windows_kernel), separate and in place (own == dst at a byte
    offset), against the ring-order oracle; nothing outside dst written."""
    import dccl_amd
    from tests.test_gpu_parity import rand_inputs, dev_bytes, host_of
    from tests.test_oracle import fp_equal
    import torch
    rng = np.random.default_rng(1500 + dt)
    esz = dccl_amd.size_of_type(dt)
    per_tile = 64 * (16 // esz)
    for k, n in ((1, 3), (2, per_tile - 1), (3, per_tile + 5), (4, 4099), (6, 2 * per_tile + 1), (8, 20001)):
        for dst_mis in (False, True):
            op = int(rng.integers(0, 4))
            arrs = [rand_inputs(rng, dt, n)[0] for _ in range(k + 1)]
            sends, own = arrs[:k], arrs[k]
            want = chain_expected(sends, own, dt, op)
            offs = [int(rng.integers(0, 64)) for _ in range(k + 1)]
            offs[0] = offs[0] // esz * esz + 1
            doff = int(rng.integers(0, 64 // esz)) * esz + (int(rng.integers(1, esz)) if dst_mis else 0)
            dev = [dev_bytes(a, o) for a, o in zip(sends, offs)]
            t_own, p_own = dev_bytes(own, offs[k])
            t_dst, p_dst = dev_bytes(np.zeros_like(own), doff)
            assert dccl_amd.local_reduce_chain([d[1] for d in dev], p_own, p_dst, dt, n, op) == 0
            torch.cuda.synchronize()
            assert fp_equal(host_of(t_dst, doff, own), want, dt), (op, k, n, offs, doff)
            nb = n * esz
            assert not t_dst[:doff].any() and not t_dst[doff + nb:].any(), (k, n, offs, doff)
            assert host_of(t_own, offs[k], own).tobytes() == own.tobytes()
            # in place: own == dst at a byte offset of its own
            t_in, p_in = dev_bytes(own, doff)
            assert dccl_amd.local_reduce_chain([d[1] for d in dev], p_in, p_in, dt, n, op) == 0
            torch.cuda.synchronize()
            assert fp_equal(host_of(t_in, doff, own), want, dt), (op, k, n, offs, doff, "in place")


@pytest.mark.gpu
def test_copy_multi(gpu):
    import torch
    import dccl_amd
    for nbytes, soff, doff in ((1, 0, 0), (15, 3, 3), (4096, 0, 0), ((1 << 20) + 7, 5, 5), (1000, 1, 2),
                               (1023, 4, 0), (1024 * 64 + 17, 0, 12), ((1 << 20) + 3, 13, 6), (17, 15, 1),
                               (64 * 16 + 5, 8, 9), (999999, 7, 3)):
        srcs = [torch.randint(0, 255, (nbytes + 64,), dtype=torch.uint8, device="cuda") for _ in range(8)]
        dsts = [torch.zeros(nbytes + 64, dtype=torch.uint8, device="cuda") for _ in range(8)]
        assert dccl_amd.copy_multi([s.data_ptr() + soff for s in srcs], [d.data_ptr() + doff for d in dsts],
                                   nbytes) == 0
        torch.cuda.synchronize()
        for s, d in zip(srcs, dsts):
            assert torch.equal(d[doff:doff + nbytes], s[soff:soff + nbytes])
            assert int(d[:doff].sum()) == 0 and int(d[doff + nbytes:].sum()) == 0


def _inputs(W, n, dt, op):
    return [oracle.synth(n, dt, op, SEED, r) for r in range(W)]


def _ring_expected(api, inputs, dt, op, root=0):
    W = len(inputs)
    slot = inputs[0].size // W

    def combine(s, r):
        assert oracle.expected_reduce(np.ascontiguousarray(s), r, dt, op) == 0

    def copy(d, s):
        d[:] = s

    bufs = [x.copy() for x in inputs]
    if api == "all_reduce":
        return ringsim.ring_allreduce(bufs, combine, copy)
    if api == "reduce_scatter":
        ringsim.reduce_scatter_ring(bufs, combine, *ringsim.rs_maps())
        return [bufs[r][r * slot:(r + 1) * slot] for r in range(W)]
    if api == "reduce":
        ringsim.reduce_scatter_ring(bufs, combine, *ringsim.rs_maps())
        return np.concatenate([bufs[r][r * slot:(r + 1) * slot] for r in range(W)])
    raise ValueError(api)


def _run_direct_rank(comm, r, W, n, dt, op, api, stream, torch):
    """One rank's part: returns the host copy of the output buffer."""
    import dccl_amd
    esz = dccl_amd.size_of_type(dt)
    x = oracle.synth(n, dt, op, SEED, r)
    send = torch.from_numpy(x.view(np.uint8).copy()).cuda()
    out_bytes = {"all_reduce_inplace": 0, "reduce_scatter": n // W * esz, "all_gather": W * n * esz}.get(api, n * esz)
    out = torch.zeros(out_bytes, dtype=torch.uint8, device="cuda") if out_bytes else send
    torch.cuda.synchronize()  # inputs and zeroed outputs complete before the collective's stream runs
    s, o = send.data_ptr(), out.data_ptr()
    if api in ("all_reduce_inplace", "all_reduce"):
        rc = comm.all_reduce(s, o, n, dt, op, stream)
    elif api == "reduce_scatter":
        rc = comm.reduce_scatter(s, o, n // W, dt, op, stream)
    elif api == "reduce":
        rc = comm.reduce(s, o, n, dt, op, 1 % W, stream)
    elif api == "all_gather":
        rc = comm.all_gather(s, o, n, dt, stream)
    elif api == "broadcast":
        rc = comm.broadcast(s, o, n, dt, W - 1, stream)
    else:
        raise ValueError(api)
    assert rc == 0, (api, rc)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _check(api, outs, W, n, dt, op):
    npd = oracle.NP_DTYPES[dt]
    inputs = _inputs(W, n, dt, op)
    if api in ("all_reduce", "all_reduce_inplace"):
        want = _ring_expected("all_reduce", inputs, dt, op)
        for r in range(W):
            assert outs[r].view(npd).tobytes() == want[r].tobytes(), (api, r)
    elif api == "reduce_scatter":
        want = _ring_expected("reduce_scatter", inputs, dt, op)
        for r in range(W):
            assert outs[r].view(npd).tobytes() == want[r].tobytes(), (api, r)
    elif api == "reduce":
        want = _ring_expected("reduce", inputs, dt, op)
        assert outs[1 % W].view(npd).tobytes() == want.tobytes()
    elif api == "all_gather":
        want = np.concatenate(inputs)
        for r in range(W):
            assert outs[r].view(npd).tobytes() == want.tobytes(), (api, r)
    elif api == "broadcast":
        for r in range(W):
            assert outs[r].view(npd).tobytes() == inputs[W - 1].tobytes(), (api, r)


APIS = ["all_reduce_inplace", "all_reduce", "reduce_scatter", "reduce", "all_gather", "broadcast"]


@pytest.mark.gpu
@pytest.mark.parametrize("W,n,dt,op", [(2, 2 * 4099, 7, 0), (4, 4 * 65536, 9, 2), (8, 8 * 1001, 4, 1),
                                       (3, 3 * 777, 6, 3), (5, 5 * 77, 5, 0)])
def test_direct_in_process(gpu, monkeypatch, W, n, dt, op):
    import torch
    import dccl_amd
    monkeypatch.setenv("DCCL_ALLREDUCE_ALGORITHM", "direct")
    for api in APIS:
        outs, errs = [None] * W, []

        def worker(r):
            try:
                comm = dccl_amd.Comm.in_process(W, r)
                try:
                    st = torch.cuda.Stream()
                    outs[r] = _run_direct_rank(comm, r, W, n, dt, op, api, st.cuda_stream, torch)
                finally:
                    comm.finalize()
            except Exception as e:  # pragma: no cover - reported below
                errs.append((r, repr(e)))

        ts = [threading.Thread(target=worker, args=(r,)) for r in range(W)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=300)
        assert not errs, (api, errs)
        _check(api, outs, W, n, dt, op)


def _ipc_rank(r, W, n, dt, op, tag, q):
    os.environ["DCCL_BOOTSTRAP_TAG"] = tag
    os.environ.setdefault("DCCL_IPC_TIMEOUT_S", "60")  # a failed peer ends the others' barriers early
    try:
        import torch
        import dccl_amd
        torch.cuda.set_device(0)
        comm = dccl_amd.Comm.ipc(W, r)
        outs = {}
        try:
            st = torch.cuda.Stream()
            for api in APIS:
                outs[api] = _run_direct_rank(comm, r, W, n, dt, op, api, st.cuda_stream, torch)
            outs["host_rejected"] = comm.all_reduce(np.zeros(4, np.float32).ctypes.data,
                                                    np.zeros(4, np.float32).ctypes.data, 4, 7, 0) == 5
        finally:
            outs["finalize"] = comm.finalize()
        q.put((r, outs, None))
    except Exception as e:  # pragma: no cover - reported by the parent
        q.put((r, None, repr(e)))


@pytest.mark.gpu
@pytest.mark.parametrize("W,n,dt,op", [(2, 2 * 65536, 7, 0), (4, 4 * 4099, 2, 1), (3, 3 * 1000, 9, 3),
                                      (8, 8 * 65536, 7, 0)])
def test_ipc_transport_processes(gpu, W, n, dt, op):
    """One process per rank (all on the box's one GPU), buffers exported with hipIpcGetMemHandle and
    read by the peers: every direct collective bit-exact against the ring simulation."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    tag = "test_" + uuid.uuid4().hex[:12]
    ps = [ctx.Process(target=_ipc_rank, args=(r, W, n, dt, op, tag, q)) for r in range(W)]
    for p in ps:
        p.start()
    results = {}
    try:
        for _ in range(W):
            r, outs, err = q.get(timeout=240)
            assert err is None, (r, err)
            results[r] = outs
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for api in APIS:
        _check(api, [results[r][api] for r in range(W)], W, n, dt, op)
    assert all(results[r]["host_rejected"] for r in range(W))
    assert all(results[r]["finalize"] == 0 for r in range(W))


def _ipc_realloc_rank(r, W, nbytes, rounds, grow, tag, q, two_comms=False, hold=False, register=False):
    """All-gathers over fresh allocations: before each round every buffer of the previous round is freed back to
    the driver (torch.cuda.empty_cache), so the next allocation may reuse its address; every round carries new
    data.  `grow`: odd rounds send W times as much, so a round's input lands where the previous round's output
    was (bench.py's all_gather at 256 MiB followed by C5's).  `two_comms`: every round runs on two IPC
    communicators of the same ranks, which share the process's peer mappings.  `hold`: nothing is freed, so
    every round's buffers are new allocations and the peer mappings pile up past the cache's bound.
    `register`: every round registers its buffers (dcclRegisterCacheMemory) and deregisters them before the
    free (tracked only: inputs go through the scratch either way)."""
    os.environ["DCCL_BOOTSTRAP_TAG"] = tag
    os.environ.setdefault("DCCL_IPC_TIMEOUT_S", "60")
    log_dir = os.environ.get("DCCL_STRESS_LOG_DIR")  # tools/ipc_churn_stress.py --trace: this rank's stderr to a file
    if log_dir:
        fd = os.open(os.path.join(log_dir, f"rank{r}.log"), os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        os.dup2(fd, 2)
    try:
        import torch
        import dccl_amd
        torch.cuda.set_device(0)
        comm = dccl_amd.Comm.ipc(W, r)
        comms = [comm]
        if two_comms:
            comms.append(dccl_amd.Comm.ipc(W, r))
        bad = []  # (round, peer, what it held) of every slice that is wrong
        kept = []
        ptrs = []  # this rank's input address per round (a peer's report is read against it)
        try:
            st = torch.cuda.Stream()
            for k in range(rounds):
                n = nbytes // 4 * (W if grow and k % 2 else 1)
                g = torch.Generator(device="cuda").manual_seed(1000 * k + r)
                mine = torch.randint(-2**31, 2**31 - 1, (n,), device="cuda", dtype=torch.int32, generator=g)
                out = torch.zeros(W * n, device="cuda", dtype=torch.int32)
                torch.cuda.synchronize()
                ptrs.append(mine.data_ptr())
                if log_dir:
                    print(f"[round {k}] rank {r} mine {mine.data_ptr():#x} out {out.data_ptr():#x}", file=sys.stderr,
                          flush=True)
                if register:
                    for cm in comms:
                        assert cm.register(mine.data_ptr(), n * 4) == 0
                        assert cm.register(out.data_ptr(), W * n * 4) == 0
                want = [torch.randint(-2**31, 2**31 - 1, (n,), device="cuda", dtype=torch.int32,
                                      generator=torch.Generator(device="cuda").manual_seed(1000 * k + p))
                        for p in range(W)]
                for ci, cm in enumerate(comms):
                    out.zero_()
                    torch.cuda.synchronize()
                    rc = cm.all_gather(mine.data_ptr(), out.data_ptr(), n, 2, st.cuda_stream)
                    if rc != 0:
                        bad.append((k, -1, f"comm {ci}: all_gather returned {rc}"))
                        break
                    st.synchronize()
                    for p in range(W):
                        got = out[p * n:(p + 1) * n]
                        if not torch.equal(got, want[p]):  # stale (an earlier round's data) or other
                            stale = [j for j in range(k) if torch.equal(got, torch.randint(
                                -2**31, 2**31 - 1, (n,), device="cuda", dtype=torch.int32,
                                generator=torch.Generator(device="cuda").manual_seed(1000 * j + p)))]
                            d = got != want[p]
                            frac = f"{float(d.float().mean()):.4f} of elements"
                            bad.append((k, p, f"comm {ci}: round {stale} data" if stale else f"comm {ci}: other, {frac}"))
                if bad and bad[-1][1] == -1:
                    break
                if register:
                    for cm in comms:
                        assert cm.deregister(mine.data_ptr()) == 0
                        assert cm.deregister(out.data_ptr()) == 0
                if hold:
                    kept.append((mine, out))
                del mine, out, want
                torch.cuda.synchronize()
                if not hold:
                    torch.cuda.empty_cache()
        finally:
            fin = max(cm.finalize() for cm in comms)
        q.put((r, (bad, fin, dccl_amd.ipc_stats(), ptrs), None))
    except Exception as e:  # pragma: no cover - reported by the parent
        q.put((r, None, repr(e)))


@pytest.mark.gpu
@pytest.mark.parametrize("W,nbytes,rounds,grow,two,hold,reg", [
    # VERDICT r3's churn cases: 1 MiB buffers freed and re-allocated every round
    (2, 1 << 20, 140, False, False, False, False), (4, 1 << 20, 100, False, False, False, False),
    (2, 1 << 20, 140, False, False, False, True), (4, 1 << 20, 100, False, False, False, True),
    (4, 1 << 20, 40, True, True, False, True),
    (2, 64 << 20, 4, False, False, False, False), (4, 256 << 20, 4, False, False, False, False),
    (4, 64 << 20, 4, True, False, False, True), (4, 64 << 20, 4, True, True, False, False),
    (2, 64 << 20, 6, False, True, False, True), (2, 16 << 20, 140, False, False, True, True)])
def test_ipc_reallocated_buffers(gpu, W, nbytes, rounds, grow, two, hold, reg):
    """A peer's buffer freed and a new one of the same size allocated must be mapped afresh: a cache of peer
    mappings keyed by the IPC handle alone can hand back the freed buffer's mapping (the handle bytes of a
    dmabuf export can repeat once the old export is closed), and the collective then reads stale data.
    140 rounds at W = 2 with every buffer kept (16 MiB inputs, 32 MiB outputs: one allocation each) import 280
    peer allocations, past the 256 mappings a process keeps open (trim_mappings closes the oldest unused ones).
    `two`: two communicators of the same ranks share the process's mappings (a stale mapping one of them still
    held used to shadow the other's re-import).  `reg`: the buffers are registered every round (and registered
    on both communicators with `two`: counted registrations); inputs reach the peers through each
    communicator's scratch, exported once and verified by its token.  No mapping may alias another and every new
    scratch mapping must read back its token (alias_errors == verify_failures == 0 in every process)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    tag = "test_" + uuid.uuid4().hex[:12]
    ps = [ctx.Process(target=_ipc_realloc_rank, args=(r, W, nbytes, rounds, grow, tag, q, two, hold, reg))
          for r in range(W)]
    for p in ps:
        p.start()
    results = {}
    try:
        for _ in range(W):
            r, res, err = q.get(timeout=240)
            assert err is None, (r, err)
            results[r] = res
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(W):
        bad, fin, stats, _ = results[r]
        assert not bad and fin == 0, (r, bad[:8], len(bad), fin, stats)
        assert stats["alias_errors"] == 0 and stats["verify_failures"] == 0, (r, stats)
        # every input through the verified scratch, registered or not
        assert stats["scratch_copies"] >= rounds and stats["registered_hits"] == 0, (r, stats)


def _ipc_dying_rank(r, tag, q):
    os.environ["DCCL_BOOTSTRAP_TAG"] = tag
    os.environ["DCCL_IPC_TIMEOUT_S"] = "25"  # far above the wait the liveness check allows
    try:
        import time
        import torch
        import dccl_amd
        torch.cuda.set_device(0)
        comm = dccl_amd.Comm.ipc(2, r)
        if r == 1:
            q.put((r, None, None))
            q.close()
            q.join_thread()  # the message is in the pipe before the process vanishes
            os._exit(0)  # gone without finalize, as after a runtime abort
        x = torch.ones(1 << 20, device="cuda", dtype=torch.float32)
        t0 = time.monotonic()
        rc = comm.all_reduce(x.data_ptr(), x.data_ptr(), x.numel(), 7, 0, torch.cuda.current_stream().cuda_stream)
        dt = time.monotonic() - t0
        q.put((r, (rc, dt, comm.finalize()), None))
    except Exception as e:  # pragma: no cover - reported by the parent
        q.put((r, None, repr(e)))


@pytest.mark.gpu
def test_ipc_dead_peer_ends_wait(gpu):
    """A rank whose process dies (a runtime abort in round 3's 64 MiB churn run left its peers in the
    barrier for the whole timeout) ends the others' collective with an error within seconds."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    tag = "test_" + uuid.uuid4().hex[:12]
    ps = [ctx.Process(target=_ipc_dying_rank, args=(r, tag, q)) for r in range(2)]
    for p in ps:
        p.start()
    results = {}
    try:
        for _ in range(2):
            r, res, err = q.get(timeout=120)
            assert err is None, (r, err)
            results[r] = res
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    rc, dt, fin = results[0]
    assert rc in (2, 6), rc  # ncclRemoteError (or ncclSystemError)
    assert dt < 10.0, dt


IPC_REGISTER_CHILD = r"""
import json, os
import torch
import dccl_amd
torch.cuda.set_device(0)
comm = dccl_amd.Comm.ipc(1, 0)
x = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
p, out = x.data_ptr(), {}
out["reg"] = comm.register(p, 1 << 20)
out["reg_again"] = comm.register(p, 1 << 20)            # the same start again: counted
out["past_end"] = comm.register(p, 1 << 40)              # past its allocation (torch's segment included)
out["dereg"] = [comm.deregister(p), comm.deregister(p), comm.deregister(p)]  # twice, then unknown
out["dereg_unknown"] = comm.deregister(p + 64)
out["unaligned"] = comm.register(p + 1, 64)
y = torch.full((1024,), 2.0, device="cuda")
out["all_reduce"] = comm.all_reduce(y.data_ptr(), y.data_ptr(), 1024, 7, 0, 0)
torch.cuda.synchronize()
out["value_ok"] = bool(torch.all(y == 2.0))
stats = dccl_amd.ipc_stats()
out["exports_made"] = stats["exports_made"]
out["registered_hits"] = stats["registered_hits"]
out["finalize"] = comm.finalize()
print(json.dumps(out))
"""


@pytest.mark.gpu
def test_ipc_registration_is_track_only(gpu, tmp_path):
    """dcclRegisterCacheMemory of device memory on an IPC communicator (round 5): validated (a device allocation
    of this process, the range inside it, 64-B aligned) and counted per start address, nothing exported;
    deregistering an unknown start is ncclInvalidArgument (4)."""
    import json
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {**os.environ, "PYTHONPATH": root, "DCCL_BOOTSTRAP_DIR": str(tmp_path),
           "DCCL_BOOTSTRAP_TAG": "ipcreg_" + uuid.uuid4().hex[:10]}
    p = subprocess.run([sys.executable, "-c", IPC_REGISTER_CHILD], env=env, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["reg"] == 0 and out["reg_again"] == 0 and out["past_end"] == 4, out
    assert out["dereg"] == [0, 0, 4] and out["dereg_unknown"] == 4 and out["unaligned"] == 4, out
    assert out["all_reduce"] == 0 and out["value_ok"] and out["finalize"] == 0, out
    # registration exported nothing (and W = 1 runs no peer-read collective, so no scratch was exported either)
    assert out["exports_made"] == 0 and out["registered_hits"] == 0, out
