#!/usr/bin/env python3
"""Occupancy caps of the k-way and chain combines at 1 GiB per operand.

For k = 1..8 and two operand layouts (separate allocations; one allocation with a 4 KiB x (j+1) stagger),
times the shipped entry points (dccl_local_reduce_multi, dccl_local_reduce_chain in place) and the same
kernels through the tuning library at a fixed number of resident one-wave blocks per CU (set with unused
LDS), interleaved over --rounds rounds; reports the median fraction of the 8 TB/s peak on (k+2)*N bytes.

    python tools/kway_waves.py [--mib 1024] [--rounds 3] [--out gpurun_out/kway_waves.json]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402
from tools import tune_lib  # noqa: E402
from tools.tune_multi import lds_for, operands  # noqa: E402

PEAK = 8.0e12
WAVES = [32, 24, 20, 16, 13, 11, 9, 7]


def time_ms(fn, reps):
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mib", type=int, default=1024)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--ks", default="1,2,3,4,5,6,7,8")
    p.add_argument("--out", default="gpurun_out/kway_waves.json")
    a = p.parse_args()
    nbytes = a.mib << 20
    n = nbytes // 4
    st = torch.cuda.current_stream().cuda_stream
    rows = []
    for layout in ("separate", "staggered"):
        keep, ptrs = operands(8, nbytes, layout)  # recv/own + 8 sources
        for j, q in enumerate(ptrs):
            dccl_amd.check(dccl_amd.synth_fill(q, 7, n, 0, 0xDCC1, j, st))
        recv, srcs = ptrs[0], ptrs[1:]
        for k in [int(x) for x in a.ks.split(",")]:
            sends = srcs[:k]
            arr = (ctypes.c_void_p * k)(*sends)
            cases = {
                "multi_shipped": lambda: dccl_amd.local_reduce_multi(sends, recv, 7, n, 0, st),
                "chain_shipped": lambda: dccl_amd.local_reduce_chain(sends, recv, recv, 7, n, 0, st),
            }
            for w in WAVES:
                cases[f"multi_w{w}"] = (lambda w=w: tune_lib.lib.dccl_tune_multi_f32_sum(arr, k, recv, n, 0,
                                                                                       lds_for(w), st))
                cases[f"chain_w{w}"] = (lambda w=w: tune_lib.lib.dccl_tune_chain_f32_sum(arr, k, recv, recv, n,
                                                                                       lds_for(w), st))
            t = {c: [] for c in cases}
            for _ in range(a.rounds):
                for c, fn in cases.items():
                    t[c].append(time_ms(fn, a.reps))
            row = {"layout": layout, "k": k}
            for c in cases:
                row[c] = round((k + 2) * nbytes / (statistics.median(t[c]) * 1e-3) / PEAK, 4)
            rows.append(row)
            print(json.dumps(row), flush=True)
        del keep
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"device": torch.cuda.get_device_name(), "bytes_per_operand": nbytes, "waves": WAVES,
                   "note": "fraction of 8 TB/s on (k+2)*N bytes; median over rounds of back-to-back launches",
                   "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
