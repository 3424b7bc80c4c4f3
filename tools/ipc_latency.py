#!/usr/bin/env python3
"""All-reduce (or all-gather) latency over the cross-process IPC transport (the direct peer-read collectives,
DESIGN.md §7.3): W processes, here all on one GPU, fp32 Sum, in place, µs per call (max over ranks).
    python tools/ipc_latency.py [--worlds 2,4,8] [--counts 1024,262144,4194304] [--iters 200] [--out f.jsonl]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rank_main(r, W, counts, iters, tag, q, api="all_reduce"):
    os.environ["DCCL_BOOTSTRAP_TAG"] = tag
    sys.path.insert(0, ROOT)
    try:
        import torch
        import dccl_amd
        torch.cuda.set_device(0)
        comm = dccl_amd.Comm.ipc(W, r)
        out = {}
        try:
            st = torch.cuda.Stream()
            for n in counts:
                n = n // W * W
                x = torch.full((n,), float(r + 1), device="cuda")
                mine = torch.full((n // W,), float(r + 1), device="cuda")
                if api == "all_reduce":
                    call = lambda: comm.all_reduce(x.data_ptr(), x.data_ptr(), n, 7, 0, st.cuda_stream)
                else:  # all_gather of n / W elements per rank into x
                    call = lambda: comm.all_gather(mine.data_ptr(), x.data_ptr(), n // W, 7, st.cuda_stream)
                torch.cuda.synchronize()
                for _ in range(10):
                    dccl_amd.check(call(), api)
                st.synchronize()
                reps = iters if n <= (1 << 18) else max(20, iters // 10)
                t0 = time.perf_counter()
                for _ in range(reps):
                    dccl_amd.check(call(), api)
                st.synchronize()
                out[n] = (time.perf_counter() - t0) / reps * 1e6
        finally:
            comm.finalize()
        q.put((r, out, None))
    except Exception as e:  # reported by the parent
        q.put((r, None, repr(e)))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--worlds", default="2,4,8")
    p.add_argument("--counts", default="1024,262144,4194304")
    p.add_argument("--iters", type=int, default=200)
    p.add_argument("--api", default="all_reduce", choices=["all_reduce", "all_gather"])
    p.add_argument("--out", default="")
    a = p.parse_args()
    ctx = mp.get_context("spawn")
    counts = [int(c) for c in a.counts.split(",")]
    rows = []
    for W in (int(w) for w in a.worlds.split(",")):
        q = ctx.Queue()
        tag = "lat_" + uuid.uuid4().hex[:12]
        ps = [ctx.Process(target=rank_main, args=(r, W, counts, a.iters, tag, q, a.api)) for r in range(W)]
        for pr in ps:
            pr.start()
        res = {}
        for _ in range(W):
            r, out, err = q.get(timeout=300)
            if err:
                raise SystemExit(f"rank {r}: {err}")
            res[r] = out
        for pr in ps:
            pr.join(timeout=60)
        for n in res[0]:
            rows.append({"api": a.api, "world": W, "count": n, "us": round(max(res[r][n] for r in range(W)), 2)})
            print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(json.dumps(x) for x in rows) + "\n")


if __name__ == "__main__":
    main()
