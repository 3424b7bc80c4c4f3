#!/usr/bin/env python3
"""Tile orders of the aligned pairwise combine on separately allocated operands (tuning only):
DCCL's real shape is a library scratchpad combined into a user chunk, two allocations whose relative physical
placement varies from pair to pair (the bench's `other_layout`: 82-84 % against 85.6 % pooled).  For
--pairs pairs of separately allocated 1 GiB fp32 operands, plus one pooled pair for reference, every variant
of tools/tune/pair_small.hip (code@lds: variant code, LDS bytes per block, 7168 = the product's 22-wave cap for
separate allocations) is timed interleaved with the product (HIP events around --launches launches, median
of --rounds); per variant the median and minimum over the separate pairs, as fractions of 3 GiB at 8 TB/s.

    python tools/pair_layout.py [--variants 0@0,0@7168,8@0,10@7168] [--pairs 6] [--out f.json]
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
    ap.add_argument("--variants", default="0@0,0@7168,8@0,8@7168,9@7168,10@0,10@7168,11@0,11@7168")
    ap.add_argument("--pairs", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    lib = ctypes.CDLL(LIB)
    lib.ps_combine.restype = ctypes.c_int
    lib.ps_combine.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                               ctypes.c_void_p]
    variants = [tuple(int(x) for x in v.split("@")) for v in a.variants.split(",")]
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    nb = 1 << 30
    n = nb // 4
    bufs, pairs = [], []
    for j in range(a.pairs):  # separately allocated, as DCCL's scratchpad and user buffer
        s_ = torch.empty(nb, dtype=torch.uint8, device=dev)
        r_ = torch.empty(nb, dtype=torch.uint8, device=dev)
        bufs += [s_, r_]
        pairs.append(("separate", s_.data_ptr(), r_.data_ptr()))
    pool = torch.empty(2 * nb + 4096, dtype=torch.uint8, device=dev)  # the bench's pooled pair
    bufs.append(pool)
    pairs.append(("pooled", pool.data_ptr() + nb + 4096, pool.data_ptr()))
    for j, (_, ps, pr) in enumerate(pairs):
        for k, p in enumerate((ps, pr)):
            dccl_amd.check(dccl_amd.synth_fill(p, 7, n, 0, 0xDCC1, 60 + 2 * j + k, st.cuda_stream), "synth")

    def call(v, ps, pr):
        if v is None:
            return dccl_amd.local_reduce(ps, pr, 7, n, 0, st.cuda_stream)
        return lib.ps_combine(v[0], v[1], ps, pr, n, st.cuda_stream)

    keys = [None] + variants
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {(j, k): [] for j in range(len(pairs)) for k in range(len(keys))}
    for _ in range(a.rounds):
        for j, (_, ps, pr) in enumerate(pairs):
            for k, v in enumerate(keys):
                assert call(v, ps, pr) == 0
                ev0.record(st)
                for _ in range(a.launches):
                    call(v, ps, pr)
                ev1.record(st)
                ev1.synchronize()
                times[(j, k)].append(ev0.elapsed_time(ev1) / a.launches)
    frac = {(j, k): round(3 * nb / (statistics.median(t) * 1e-3) / PEAK, 4) for (j, k), t in times.items()}
    names = ["product"] + [f"{v[0]}@{v[1]}" for v in variants]
    sep = [j for j, p in enumerate(pairs) if p[0] == "separate"]
    pooled = [j for j, p in enumerate(pairs) if p[0] == "pooled"][0]
    rows = []
    for k, name in enumerate(names):
        fs = [frac[(j, k)] for j in sep]
        rows.append({"variant": name, "separate_median": round(statistics.median(fs), 4), "separate_min": min(fs),
                     "separate": fs, "pooled": frac[(pooled, k)]})
        print(f"{name:10s} separate median {100 * statistics.median(fs):.2f} min {100 * min(fs):.2f}  "
              f"pooled {100 * frac[(pooled, k)]:.2f}   " + " ".join(f"{100 * x:.1f}" for x in fs), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"pairs": a.pairs, "rounds": a.rounds, "launches": a.launches, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
