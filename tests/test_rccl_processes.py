"""The namespace-dccl collectives over the RCCL transport (dccl_comm_init_rccl, rccl_transport.cpp) with W = 2-8 real
RCCL ranks, one process each, on the box's one GPU.

RCCL refuses two ranks on one device of one host ("Duplicate GPU detected"), so every rank process gets its own
NCCL_HOSTID: RCCL then takes the ranks for W hosts and connects them over its socket transport on loopback
(NCCL_SOCKET_IFNAME=lo).  The data path is RCCL's ncclSend / ncclRecv as on a real node; only the wire differs
(sockets instead of xGMI), so the ring's step loop, rank maps, scratchpads and the gfx950 combine between the
receives run exactly as in the driver's 8-GPU run.  Every result is checked bit for bit against the ring
simulation (tests/ringsim.py) or the Rabenseifner simulation (tests/rabsim.py) over the oracle restatement.
"""
import multiprocessing as mp
import os
import uuid

import numpy as np
import pytest

import oracle
from tests import rabsim, ringsim
from tests.test_direct import APIS, _check, _run_direct_rank

pytestmark = pytest.mark.gpu
SEED = 0xDCC1


def _rccl_rank(r, W, n, dt, op, hostid, conn, algo):
    os.environ.update({"NCCL_HOSTID": f"{hostid}-{r}", "NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1",
                       "DCCL_ALLREDUCE_ALGORITHM": algo})
    try:
        import torch
        import dccl_amd
        torch.cuda.set_device(0)
        if r == 0:
            uid = dccl_amd.Comm.unique_id()
            for c in conn:
                c.send(uid)
            conn = conn[0] if conn else None
        else:
            uid = conn.recv()
        comm = dccl_amd.Comm.rccl(W, r, uid)
        outs = {}
        try:
            st = torch.cuda.Stream()
            for api in (APIS if algo in ("ring", "grouped") else ["all_reduce"]):
                outs[api] = _run_direct_rank(comm, r, W, n, dt, op, api, st.cuda_stream, torch)
            # device memory only on this transport: a host buffer is ncclInvalidUsage
            outs["host_rejected"] = comm.all_reduce(np.zeros(4, np.float32).ctypes.data,
                                                    np.zeros(4, np.float32).ctypes.data, 4, 7, 0) == 5
        finally:
            outs["finalize"] = comm.finalize()
        return outs, None
    except Exception as e:  # reported by the parent
        return None, repr(e)


def _entry(r, W, n, dt, op, hostid, conn, algo, q):
    q.put((r, *_rccl_rank(r, W, n, dt, op, hostid, conn, algo)))


def _run(W, n, dt, op, algo):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pipes = [ctx.Pipe() for _ in range(W - 1)]
    hostid = "dccl-test-" + uuid.uuid4().hex[:10]
    ps = [ctx.Process(target=_entry, args=(r, W, n, dt, op, hostid,
                                           [a for a, _ in pipes] if r == 0 else pipes[r - 1][1], algo, q))
          for r in range(W)]
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
    return results


@pytest.mark.parametrize("algo", ["ring", "grouped"])
@pytest.mark.parametrize("W,n,dt,op", [(2, 2 * 65536, 7, 0), (3, 3 * 4099, 2, 1), (4, 4 * 1000, 9, 3),
                                      (8, 8 * 777, 7, 2)])
def test_rccl_transport_processes(gpu, W, n, dt, op, algo):
    """`ring` (the default): the reference's ring step loop over RCCL send/recv; `grouped`: all_reduce and
    reduce_scatter take the grouped forms (one RCCL group per phase, one chain combine in the ring's order,
    algorithms.hpp).  Both bit-exact against the ring simulation."""
    import dccl_amd
    if not dccl_amd.lib.dccl_rccl_available():
        pytest.skip("librccl not loadable")
    results = _run(W, n, dt, op, algo)
    for api in APIS:
        _check(api, [results[r][api] for r in range(W)], W, n, dt, op)
    assert all(results[r]["host_rejected"] for r in range(W))
    assert all(results[r]["finalize"] == 0 for r in range(W))


@pytest.mark.parametrize("W,n,dt,op", [(3, 3 * 840, 7, 0), (4, 4 * 4096, 7, 2)])
def test_rccl_rabenseifner_processes(gpu, W, n, dt, op):
    """The Rabenseifner all-reduce (fold to 2^k ranks, recursive halving, recursive doubling) over real RCCL."""
    import dccl_amd
    if not dccl_amd.lib.dccl_rccl_available():
        pytest.skip("librccl not loadable")
    results = _run(W, n, dt, op, "rabenseifner")
    want = [oracle.synth(n, dt, op, SEED, r) for r in range(W)]

    def combine(send, recv):
        assert oracle.expected_reduce(np.ascontiguousarray(send), recv, dt, op) == 0

    rabsim.rabenseifner_allreduce(want, combine)
    npd = oracle.NP_DTYPES[dt]
    for r in range(W):
        assert results[r]["all_reduce"].view(npd).tobytes() == want[r].tobytes(), r
        assert results[r]["finalize"] == 0
