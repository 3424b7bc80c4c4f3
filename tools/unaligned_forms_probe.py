#!/usr/bin/env python3
"""Tuning only: the combines into a destination that is not element-aligned, by form and wave cap (round 3).

The kernels read the destination's window through aligned loads and the lane exchange (reduce_kernels.hpp,
reduce_unaligned_kernel / reduce_multi_unaligned_kernel / reduce_chain_unaligned_kernel).  This sweeps, on
1 GiB fp32 Sum operands (ten from one allocation, 4 KiB x (j+1) stagger; destination first, so the pair is
bench.py's pooled layout):
  pair   recv + 1 B (send aligned) and recv + 2 B (send + 3 B), caps 32 / 26 / 24 / 20 waves per CU,
         in the three tile orders of reduce_kernels.hpp tile_order (XCD-contiguous, block, group-interleaved);
  multi, chain  k = 2, 4, 8, destination + 2 B, sources aligned and + 4 B, the per-operand form and the
         loads-first form, the three tile orders, caps 32 / 24 / 16;
and the product's own launch of every case beside them (`shipped`).  Interleaved rounds, HIP events around
--launches launches, median per configuration.

    python tools/unaligned_forms_probe.py [--rounds 3] [--ks 2,3,4,6,8] [--out f.json]
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
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--launches", type=int, default=8)
    p.add_argument("--ks", default="2,4,8")
    p.add_argument("--kinds", default="pair,multi,chain")
    p.add_argument("--orders", default="0,1,2", help="tile orders: 0 XCD ranges, 1 block, 2 group (run 8), 3 run 4, 4 run 2")
    p.add_argument("--waves", default="32,24,16")
    p.add_argument("--src-offs", default="0,4")
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
    configs = []  # (key dict, k, fn)
    kinds = a.kinds.split(",")
    if "pair" in kinds:
        for soff, doff in ((0, 1), (3, 2)):
            s_, d_ = srcs[0] + soff, dst + doff
            base = {"kind": "pair", "k": 1, "dst_off": doff, "src_off": soff}
            configs.append(({**base, "form": "shipped"}, 1,
                            lambda s_=s_, d_=d_: dccl_amd.local_reduce(s_, d_, 7, n, 0, st)))
            for order in [int(x) for x in a.orders.split(",")]:
                for w in (32, 26, 24, 20):
                    configs.append(({**base, "form": "phased", "order": order, "waves": w}, 1,
                                    lambda s_=s_, d_=d_, l=lds_for(w), o=order:
                                    T.dccl_tune_unaligned_pair_f32_sum(s_, d_, n, l, o, st)))
    for kind in ("multi", "chain"):
        if kind not in kinds:
            continue
        for k in [int(x) for x in a.ks.split(",")]:
            for soff in [int(x) for x in a.src_offs.split(",")]:
                ss = [q + soff for q in srcs[:k]]
                arr = (ctypes.c_void_p * k)(*ss)
                d_ = dst + 2
                base = {"kind": kind, "k": k, "dst_off": 2, "src_off": soff}
                if kind == "multi":
                    ship = lambda arr=arr, k=k, d_=d_: dccl_amd.lib.dccl_local_reduce_multi(arr, k, d_, 7, n, 0, st)
                else:
                    ship = lambda arr=arr, k=k, d_=d_: dccl_amd.lib.dccl_local_reduce_chain(arr, k, d_, d_, 7, n, 0, st)
                configs.append(({**base, "form": "shipped"}, k, ship))
                own = None if kind == "multi" else d_
                for first in (0, 1):
                    for order in [int(x) for x in a.orders.split(",")]:
                        for w in [int(x) for x in a.waves.split(",")]:
                            configs.append(({**base, "form": "first" if first else "per_operand", "order": order,
                                             "waves": w}, k,
                                            lambda arr=arr, k=k, d_=d_, own=own, l=lds_for(w), f=first + 2 * order:
                                            T.dccl_tune_unaligned_kway_f32_sum(arr, k, own, d_, n, l, f, st)))
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
            json.dump({"bytes_per_operand": nbytes, "count": n, "rounds": a.rounds, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
