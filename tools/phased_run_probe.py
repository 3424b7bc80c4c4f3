#!/usr/bin/env python3
"""Tuning only (round 3): the phased k-way combine (every source + 4 B, recv aligned) in tile-run orders (each XCD
walks `run` consecutive tiles in every group of 8 * run blocks; run 1 = block order), per-operand and loads-first
forms, caps swept, the product's own launch beside them.  1 GiB fp32 Sum per operand, ten operands in one
allocation (4 KiB x (j+1) stagger), destination first.

    python tools/phased_run_probe.py [--ks 3,4,5,6,8] [--rounds 3] [--out f.json]
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
from tools import tune_lib  # noqa: E402

PEAK = 8e12


def lds_for(w):
    return 0 if w >= 32 else ((160 << 10) // w + 255) // 256 * 256


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--ks", default="3,4,5,6,8")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--launches", type=int, default=6)
    p.add_argument("--out", default="")
    a = p.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 1 << 30
    n = nbytes // 4 - 64
    pool = torch.empty(10 * nbytes + 4096 * 55 + 1024, dtype=torch.uint8, device="cuda")
    ptrs, off = [], 0
    for j in range(10):
        ptrs.append(pool.data_ptr() + off)
        dccl_amd.check(dccl_amd.synth_fill(ptrs[-1], 7, nbytes // 4, 0, 0xDCC1, 10 + j, st), "synth")
        off += nbytes + 4096 * (j + 1)
    dst, srcs = ptrs[0], ptrs[1:9]
    T = tune_lib.lib
    configs = []
    for k in [int(x) for x in a.ks.split(",")]:
        arr = (ctypes.c_void_p * k)(*[q + 4 for q in srcs[:k]])
        configs.append(({"k": k, "form": "shipped"}, k,
                        lambda arr=arr, k=k: dccl_amd.lib.dccl_local_reduce_multi(arr, k, dst, 7, n, 0, st)))
        for first in (0, 1):
            for run in (1, 2, 4, 8):
                for w in ((32, 16, 13, 11) if first else (32, 24, 16)):
                    configs.append(({"k": k, "form": "first" if first else "per_operand", "run": run, "waves": w}, k,
                                    lambda arr=arr, k=k, f=first, r=run, l=lds_for(w):
                                    T.dccl_tune_phased_run_f32_sum(arr, k, dst, n, l, f, r, st)))
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = [[] for _ in configs]
    for rnd in range(a.rounds):
        for i, (key, k, fn) in enumerate(configs):
            assert fn() == 0, key
            ev0.record()
            for _ in range(a.launches):
                fn()
            ev1.record()
            ev1.synchronize()
            times[i].append(ev0.elapsed_time(ev1) / a.launches)
        print(f"round {rnd} done", file=sys.stderr, flush=True)
    rows = []
    for (key, k, _), ts in zip(configs, times):
        ms = statistics.median(ts)
        rows.append({**key, "ms": round(ms, 4), "frac": round((k + 2) * n * 4 / (ms * 1e-3) / PEAK, 4)})
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"bytes_per_operand": nbytes, "count": n, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
