#!/usr/bin/env python3
"""Mid-size block shapes of the aligned pairwise combine (tools/tune/pair_small.hip; tuning only, DESIGN.md
§3.3): fp32 Sum at 4-128 MiB per operand, operand pairs (recv, then send 4 KiB past its end, one allocation
per pair) rotated over enough sets that the working set passes the 256 MiB Infinity Cache; per variant and size
the eager time per launch (HIP events around back-to-back launches) and the graph-replayed one (one HIP graph
of 100 launches, replayed 10 times, median of three windows), as a fraction of 3 * bytes at 8 TB/s.  Every
variant is checked bit for bit against the product on one pair first.

    python tools/pair_small.py [--variants 0,1,2,3,4,5,6,7] [--mib 4,8,16,32,64,128] [--out f.json]

A variant "V@L" runs variant V with L bytes of unused dynamic LDS per one-wave block (a resident-wave cap).
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dccl_amd  # noqa: E402

PEAK = 8e12
LIB = os.path.join(ROOT, "tools", "lib", "libpair_small.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,3,4,5,6,7")
    ap.add_argument("--mib", default="4,8,16,32,64,128")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    lib = ctypes.CDLL(LIB)
    lib.ps_combine.restype = ctypes.c_int
    lib.ps_combine.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                               ctypes.c_void_p]
    variants = a.variants.split(",")
    dev = torch.device("cuda", 0)
    rows = []
    for mib in (int(x) for x in a.mib.split(",")):
        nb = mib << 20
        n = nb // 4
        sets = max(2, -(-(768 << 20) // (2 * nb)))
        bufs = [torch.empty(2 * nb + 4096, dtype=torch.uint8, device=dev) for _ in range(sets)]
        st = torch.cuda.current_stream(dev)
        for j, b in enumerate(bufs):
            dccl_amd.check(dccl_amd.synth_fill(b.data_ptr(), 7, (2 * nb + 4096) // 4, 0, 0xDCC1, 50 + j,
                                               st.cuda_stream), "synth")
        pairs = [(b.data_ptr() + nb + 4096, b.data_ptr()) for b in bufs]  # (send, recv)

        def call(v, ps, pr, sh):
            if v == "-1":
                return dccl_amd.local_reduce(ps, pr, 7, n, 0, sh)
            var, _, lds = v.partition("@")
            return lib.ps_combine(int(var), int(lds or 0), ps, pr, n, sh)

        # bit-exactness on pair 0 (recv restored between runs)
        saved = bufs[0][:nb].clone()
        outs = []
        for v in ["-1"] + variants:
            bufs[0][:nb].copy_(saved)
            torch.cuda.synchronize()
            assert call(v, *pairs[0], st.cuda_stream) == 0, v
            torch.cuda.synchronize()
            outs.append(bufs[0][:nb].clone())
        exact = {v: bool(torch.equal(outs[0], o)) for v, o in zip(variants, outs[1:])}
        bufs[0][:nb].copy_(saved)
        del outs, saved
        launches = max(20, min(400, int(200 * 64 / mib)))
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        eager = {v: [] for v in ["-1"] + variants}
        for _ in range(a.rounds):
            for v in ["-1"] + variants:
                for i in range(3):
                    call(v, *pairs[i % sets], st.cuda_stream)
                ev0.record(st)
                for i in range(launches):
                    call(v, *pairs[i % sets], st.cuda_stream)
                ev1.record(st)
                ev1.synchronize()
                eager[v].append(ev0.elapsed_time(ev1) * 1e3 / launches)
        graph = {}
        for v in ["-1"] + variants:
            side = torch.cuda.Stream(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(side):
                call(v, *pairs[0], side.cuda_stream)
                side.synchronize()
                with torch.cuda.graph(g, stream=side):
                    for i in range(100):
                        assert call(v, *pairs[i % sets], side.cuda_stream) == 0
            g.replay()
            torch.cuda.synchronize()
            runs = []
            for _ in range(3):
                ev0.record(st)
                for _ in range(10):
                    g.replay()
                ev1.record(st)
                ev1.synchronize()
                runs.append(ev0.elapsed_time(ev1) * 1e3 / 1000)
            graph[v] = sorted(runs)[1]
            del g
        frac = lambda us: round(3 * nb / (us * 1e-6) / PEAK, 4)  # noqa: E731
        row = {"mib": mib, "sets": sets, "launches": launches,
               "eager_us": {str(v): round(statistics.median(eager[v]), 2) for v in eager},
               "graph_us": {str(v): round(graph[v], 2) for v in graph},
               "eager_frac": {str(v): frac(statistics.median(eager[v])) for v in eager},
               "graph_frac": {str(v): frac(graph[v]) for v in graph}, "bit_exact": {str(v): exact[v] for v in exact}}
        rows.append(row)
        print(f"{mib:4d} MiB eager " + " ".join(f"{k}:{100 * x:.1f}" for k, x in row["eager_frac"].items()) +
              " | graph " + " ".join(f"{k}:{100 * x:.1f}" for k, x in row["graph_frac"].items()) +
              f"  exact {all(exact.values())}", flush=True)
        del bufs
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
