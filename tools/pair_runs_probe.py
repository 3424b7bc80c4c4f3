#!/usr/bin/env python3
"""Tuning only (round 3): the pairwise launches in tile-run orders (reduce_kernels.hpp run_tile<RUN>), beside the
product's own launch: aligned; send off recv's lines (+16 B); send at another 16-B phase (+4 B, + 20 B) or a byte
offset (+1 B); recv not element-aligned (+1 B, the runtime order of reduce_unaligned_kernel: XCD ranges, block,
group (run 8), run 4, run 2).  bench.py's pooled layout: recv first, send 4 KiB past its end, 1 GiB fp32 Sum.

    python tools/pair_runs_probe.py [--rounds 5] [--out f.json]
"""
import argparse
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--launches", type=int, default=10)
    p.add_argument("--separate", type=int, default=0,
                   help="instead: N separately allocated aligned 1 GiB pairs, runs 1/2/4/8, uncapped and 22 waves")
    p.add_argument("--out", default="")
    a = p.parse_args()
    if a.separate:
        return separate(a)
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 1 << 30
    n = nbytes // 4 - 64
    pool = torch.empty(2 * nbytes + 8192, dtype=torch.uint8, device="cuda")
    recv, send = pool.data_ptr(), pool.data_ptr() + nbytes + 4096
    dccl_amd.check(dccl_amd.synth_fill(send, 7, nbytes // 4, 0, 0xDCC1, 0, st), "synth")
    dccl_amd.check(dccl_amd.synth_fill(recv, 7, nbytes // 4, 0, 0xDCC1, 1, st), "synth")
    T = tune_lib.lib
    configs = []
    for soff, roff, what in ((0, 0, "aligned"), (16, 0, "send+16"), (4, 0, "send+4"), (20, 0, "send+20"),
                             (1, 0, "send+1")):
        s_, r_ = send + soff, recv + roff
        configs.append(({"case": what, "form": "shipped"}, lambda s_=s_, r_=r_: dccl_amd.local_reduce(s_, r_, 7, n, 0, st)))
        for run in (1, 2, 4, 8):
            configs.append(({"case": what, "run": run},
                            lambda s_=s_, r_=r_, run=run: T.dccl_tune_pair_run_f32_sum(s_, r_, n, 0, run, st)))
    s_, r_ = send, recv + 1
    configs.append(({"case": "recv+1", "form": "shipped"}, lambda: dccl_amd.local_reduce(s_, r_, 7, n, 0, st)))
    for order, name in ((0, "xcd"), (1, "block"), (2, "run8"), (3, "run4"), (4, "run2")):
        configs.append(({"case": "recv+1", "order": name},
                        lambda o=order: T.dccl_tune_unaligned_pair_f32_sum(s_, r_, n, 0, o, st)))
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = [[] for _ in configs]
    for _ in range(a.rounds):
        for i, (key, fn) in enumerate(configs):
            assert fn() == 0, key
            ev0.record()
            for _ in range(a.launches):
                fn()
            ev1.record()
            ev1.synchronize()
            times[i].append(ev0.elapsed_time(ev1) / a.launches)
    rows = []
    for (key, _), ts in zip(configs, times):
        ms = statistics.median(ts)
        rows.append({**key, "ms": round(ms, 4), "frac": round(3 * n * 4 / (ms * 1e-3) / PEAK, 4)})
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"bytes_per_operand": nbytes, "rows": rows}, f, indent=1)


def separate(a):
    """Aligned fp32 Sum on separately allocated 1 GiB pairs (DCCL's scratchpad + user chunk shape) in every
    tile-run order, uncapped and at the shipped 22-wave cap for separate allocations."""
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 1 << 30
    n = nbytes // 4
    pairs = []
    for j in range(a.separate):
        sv = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        rv = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        dccl_amd.check(dccl_amd.synth_fill(sv.data_ptr(), 7, n, 0, 0xDCC1, 2 * j, st), "synth")
        dccl_amd.check(dccl_amd.synth_fill(rv.data_ptr(), 7, n, 0, 0xDCC1, 2 * j + 1, st), "synth")
        pairs.append((sv, rv))
    T = tune_lib.lib
    configs = []
    for j, (sv, rv) in enumerate(pairs):
        s_, r_ = sv.data_ptr(), rv.data_ptr()
        configs.append(({"pair": j, "form": "shipped"}, lambda s_=s_, r_=r_: dccl_amd.local_reduce(s_, r_, 7, n, 0, st)))
        for run in (1, 2, 4, 8):
            for lds in (0, 7168):
                configs.append(({"pair": j, "run": run, "lds": lds},
                                lambda s_=s_, r_=r_, run=run, lds=lds: T.dccl_tune_pair_run_f32_sum(s_, r_, n, lds, run, st)))
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = [[] for _ in configs]
    for _ in range(a.rounds):
        for i, (key, fn) in enumerate(configs):
            assert fn() == 0, key
            ev0.record()
            for _ in range(a.launches):
                fn()
            ev1.record()
            ev1.synchronize()
            times[i].append(ev0.elapsed_time(ev1) / a.launches)
    rows = []
    for (key, _), ts in zip(configs, times):
        ms = statistics.median(ts)
        rows.append({**key, "ms": round(ms, 4), "frac": round(3 * n * 4 / (ms * 1e-3) / PEAK, 4)})
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"bytes_per_operand": nbytes, "layout": "separate", "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
