#!/usr/bin/env python3
"""The namespace-dccl all_reduce over the RCCL transport, ring vs grouped,
with W real RCCL ranks on one GPU (one NCCL_HOSTID each, loopback sockets: tests/test_rccl_processes.py's
rehearsal).  Every rank runs `--calls` all_reduces of `--mib` MiB fp32 Sum with DCCL_ALLREDUCE_ALGORITHM=ALGO,
checks the first result bit for bit against the ring's, and prints one JSON line (rank 0) with the wall time per
call.  Under `rocprofv3 --kernel-trace --stats` the combine kernels' time per collective is the sum of the
reduce_* kernels' durations / (W * calls): the ring launches W - 1 pairwise combines of count/W elements per
rank, the grouped form one chain combine.

    python tools/rccl_ring_vs_grouped.py ALGO [--world 4] [--mib 64] [--calls 10]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_main(r, W, n, calls, algo, hostid, conn, q):
    os.environ.update({"NCCL_HOSTID": f"{hostid}-{r}", "NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1"})
    try:
        import torch
        import dccl_amd
        torch.cuda.set_device(0)
        if r == 0:
            uid = dccl_amd.Comm.unique_id()
            for c in conn:
                c.send(uid)
        else:
            uid = conn.recv()
        comm = dccl_amd.Comm.rccl(W, r, uid)
        st = torch.cuda.Stream()
        g = torch.Generator(device="cuda").manual_seed(100 + r)
        x = torch.rand(n, device="cuda", generator=g).mul_(2).sub_(1)
        res = {}
        for a in ("ring", algo):  # the ring's result is the reference for the other
            os.environ["DCCL_ALLREDUCE_ALGORITHM"] = a
            y = x.clone()
            torch.cuda.synchronize()
            dccl_amd.check(comm.all_reduce(y.data_ptr(), y.data_ptr(), n, 7, 0, st.cuda_stream), a)
            st.synchronize()
            res[a] = y
        exact = bool(torch.equal(res["ring"].view(torch.int32), res[algo].view(torch.int32)))
        os.environ["DCCL_ALLREDUCE_ALGORITHM"] = algo
        y = x.clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            dccl_amd.check(comm.all_reduce(y.data_ptr(), y.data_ptr(), n, 7, 0, st.cuda_stream), algo)
        st.synchronize()
        t = (time.perf_counter() - t0) / calls
        fin = comm.finalize()
        q.put((r, {"exact_vs_ring": exact, "ms_per_call": round(t * 1e3, 3), "finalize": fin}, None))
    except Exception as e:  # reported by the parent
        q.put((r, None, repr(e)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("algo", choices=["ring", "grouped"])
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--calls", type=int, default=10)
    a = ap.parse_args()
    W = a.world
    n = (a.mib << 20) // 4 // W * W
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pipes = [ctx.Pipe() for _ in range(W - 1)]
    hostid = "dccl-rvg-" + uuid.uuid4().hex[:8]
    ps = [ctx.Process(target=rank_main, args=(r, W, n, a.calls, a.algo, hostid,
                                              [x for x, _ in pipes] if r == 0 else pipes[r - 1][1], q))
          for r in range(W)]
    for p in ps:
        p.start()
    out = {}
    try:
        for _ in range(W):
            r, res, err = q.get(timeout=300)
            out[r] = res if err is None else {"error": err}
    finally:
        for p in ps:
            p.join(60)
            if p.is_alive():
                p.kill()
    print(json.dumps({"algo": a.algo, "world": W, "mib": a.mib, "count": n, "calls": a.calls,
                      "ranks": [out.get(r) for r in range(W)]}), flush=True)


if __name__ == "__main__":
    main()
