#!/usr/bin/env python3
"""Tuning only (round 3): the straddling and phased k-way / chain launches in tile-run orders (reduce_kernels.hpp
run_tile<RUN>: each XCD walks RUN consecutive tiles of every group of 8 RUN blocks; RUN 1 = block order) and
wave caps, beside the product's own launch of each case (`shipped`).  1 GiB fp32 Sum per operand, ten operands
in one allocation (4 KiB x (j+1) stagger), destination first; straddling sources at + 16 (2j + 1) B (in phase,
off the destination's 128-B lines), phased sources at + 4 B; chain in place (own = destination).

    python tools/runs_probe.py [--kinds 0,1,2,3] [--ks 3,4,5,6,7,8] [--rounds 3] [--out f.json]
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
KINDS = {0: "multi_straddle", 1: "chain_straddle", 2: "multi_phased", 3: "chain_phased"}


def lds_for(w):
    return 0 if w >= 32 else ((160 << 10) // w + 255) // 256 * 256


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--kinds", default="0,1,2,3")
    p.add_argument("--ks", default="3,4,5,6,7,8")
    p.add_argument("--runs", default="1,2,4")
    p.add_argument("--waves", default="32,16,13,11,9")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--launches", type=int, default=5)
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
    for kind in [int(x) for x in a.kinds.split(",")]:
        chain = kind & 1
        for k in [int(x) for x in a.ks.split(",")]:
            if not chain and k < 2:
                continue
            ss = ([q + 16 * (2 * j + 1) for j, q in enumerate(srcs[:k])] if kind < 2 else [q + 4 for q in srcs[:k]])
            arr = (ctypes.c_void_p * k)(*ss)
            base = {"kind": KINDS[kind], "k": k}
            if chain:
                ship = lambda arr=arr, k=k: dccl_amd.lib.dccl_local_reduce_chain(arr, k, dst, dst, 7, n, 0, st)
            else:
                ship = lambda arr=arr, k=k: dccl_amd.lib.dccl_local_reduce_multi(arr, k, dst, 7, n, 0, st)
            configs.append(({**base, "form": "shipped"}, k, ship))
            own = dst if chain else None
            for first in ((0, 1) if kind >= 2 else (0,)):
                for run in [int(x) for x in a.runs.split(",")]:
                    for w in [int(x) for x in a.waves.split(",")]:
                        configs.append(({**base, "form": "first" if first else "plain", "run": run, "waves": w}, k,
                                        lambda arr=arr, k=k, kd=kind, o=own, l=lds_for(w), r=run, f=first:
                                        T.dccl_tune_runs_f32_sum(kd, arr, k, o, dst, n, l, r, f, st)))
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
