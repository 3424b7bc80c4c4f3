#!/usr/bin/env python3
"""A/B of two builds of the combine on one box (tuning only): libraries built from two revisions of
dccl_amd/csrc/local_reduce.hip, loaded side by side (RTLD_LOCAL), timed interleaved on the same
operands: fp32 Sum, 1 GiB per operand, bench.py's pooled layout, plus displaced operands.
    python tools/ab_combine.py LIB_A LIB_B [--rounds 15]
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
    p.add_argument("libs", nargs=2)
    p.add_argument("--rounds", type=int, default=15)
    p.add_argument("--out", default="")
    a = p.parse_args()
    libs = []
    for path in a.libs:
        lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
        lib.dccl_local_reduce.restype = ctypes.c_int
        lib.dccl_local_reduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t,
                                          ctypes.c_int, ctypes.c_void_p]
        libs.append(lib)
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 1 << 30
    n = nbytes // 4 - 64
    pool = torch.empty(2 * nbytes + 4096, dtype=torch.uint8, device="cuda")
    base = pool.data_ptr()
    for off, bid in ((0, 2), (nbytes + 4096, 1)):
        dccl_amd.check(dccl_amd.synth_fill(base + off, 7, nbytes // 4, 0, 0xDCC1, bid, st), "synth")
    recv0, send0 = base, base + nbytes + 4096
    rows = []
    for soff, roff in ((0, 0), (16, 0), (4, 0)):
        t = {0: [], 1: []}
        for _ in range(a.rounds):
            for i, lib in enumerate(libs):
                fn = lambda lib=lib: lib.dccl_local_reduce(send0 + soff, recv0 + roff, 7, n, 0, st)
                t[i].append(time_launches([fn], rounds=1, min_ms=20.0)[0])
        for i in (0, 1):
            ms = statistics.median(t[i])
            rows.append({"lib": os.path.basename(a.libs[i]), "send_offset": soff, "recv_offset": roff,
                         "ms": round(ms, 4), "frac": round(3 * n * 4 / (ms * 1e-3) / 1e9 / PEAK, 4),
                         "ms_min": round(min(t[i]), 4)})
            print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
