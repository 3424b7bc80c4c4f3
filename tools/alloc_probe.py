#!/usr/bin/env python3
"""Allocation probe (tuning only): the shipped fp32 Sum combine over 1 GiB operands in bench.py's pooled
layout (recv, then send 4 KiB past its end), with the pool allocated three ways: torch's caching
allocator, hipMalloc, and hipExtMallocWithFlags with hipDeviceMallocContiguous, hipDeviceMallocUncached and
hipDeviceMallocFinegrained (the last two change the memory type the caches and the Infinity Cache see).
Timed interleaved.
    python tools/alloc_probe.py [--rounds 9] [--out f.json]
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
from tools.bench_suite import PEAK, time_launches  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=9)
    p.add_argument("--out", default="")
    a = p.parse_args()
    hip = ctypes.CDLL("libamdhip64.so.7")
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 1 << 30
    n = nbytes // 4
    size = 2 * nbytes + 4096
    keep = torch.empty(size, dtype=torch.uint8, device="cuda")
    pools = {"torch": keep.data_ptr()}
    for name, flags in (("hipMalloc", None), ("contiguous", 0x4), ("uncached", 0x3), ("finegrained", 0x1),
                        ("hipMalloc_2", None)):
        ptr = ctypes.c_void_p()
        rc = hip.hipMalloc(ctypes.byref(ptr), ctypes.c_size_t(size)) if flags is None else \
            hip.hipExtMallocWithFlags(ctypes.byref(ptr), ctypes.c_size_t(size), ctypes.c_uint(flags))
        if rc != 0:
            print(f"{name}: allocation failed ({rc})", flush=True)
            continue
        pools[name] = ptr.value
    for base in pools.values():
        dccl_amd.check(dccl_amd.synth_fill(base, 7, n, 0, 0xDCC1, 1, st), "synth")
        dccl_amd.check(dccl_amd.synth_fill(base + nbytes + 4096, 7, n, 0, 0xDCC1, 0, st), "synth")
    t = {k: [] for k in pools}
    for _ in range(a.rounds):
        for k, base in pools.items():
            fn = lambda base=base: dccl_amd.local_reduce(base + nbytes + 4096, base, 7, n, 0, st)
            t[k].append(time_launches([fn], rounds=1, min_ms=20.0)[0])
    rows = []
    for k in pools:
        ms = statistics.median(t[k])
        rows.append({"allocation": k, "ms": round(ms, 4), "ms_min": round(min(t[k]), 4),
                     "frac": round(3 * nbytes / (ms * 1e-3) / 1e9 / PEAK, 4)})
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
