#!/usr/bin/env python3
"""A/B of two builds of the combine on one box (tuning only): two product libraries (e.g. the shipped one
and one from tools/build_ab.sh) loaded side by side (RTLD_LOCAL), timed interleaved on the same operands,
fp32 Sum, 1 GiB per operand:
  pairwise   aligned, send off its lines, send at another 16-B phase, send at a byte offset, recv not
             element-aligned (bench.py's pooled layout, displaced);
  phased     k-way (k = 4) and chain (k = 7) with every source 4 B off the destination's 16-B phase, and
             with sources or the destination not element-aligned;
  misaligned the shape variants of the misaligned-recv kernel through the tuning library (--tune).
    python tools/ab_combine.py LIB_A LIB_B [--rounds 7] [--tune | --tune-only [--vars 25,30] [--roffs 1,2]] [--out f.json]
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


def bind(path):
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    c_int, c_size_t, c_void_p = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p
    lib.dccl_local_reduce.restype = c_int
    lib.dccl_local_reduce.argtypes = [c_void_p, c_void_p, c_int, c_size_t, c_int, c_void_p]
    lib.dccl_local_reduce_multi.restype = c_int
    lib.dccl_local_reduce_multi.argtypes = [ctypes.POINTER(c_void_p), c_int, c_void_p, c_int, c_size_t, c_int,
                                            c_void_p]
    lib.dccl_local_reduce_chain.restype = c_int
    lib.dccl_local_reduce_chain.argtypes = [ctypes.POINTER(c_void_p), c_int, c_void_p, c_void_p, c_int, c_size_t,
                                            c_int, c_void_p]
    return lib


VARS = [16, 20, 25, 21]  # 16: the kernel uncapped; 20 / 25 / 21: capped at 26 / 24 / 22 waves


def main():
    p = argparse.ArgumentParser()
    p.add_argument("libs", nargs=2)
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--tune", action="store_true", help="also time the misaligned-recv shape variants")
    p.add_argument("--tune-only", action="store_true", help="only the misaligned-recv shape variants")
    p.add_argument("--vars", default="", help="comma list of misaligned-recv tuning variants (default: VARS)")
    p.add_argument("--roffs", default="1", help="comma list of recv byte offsets for the tuning variants")
    p.add_argument("--out", default="")
    a = p.parse_args()
    tvars = [int(x) for x in a.vars.split(",")] if a.vars else VARS
    roffs = [int(x) for x in a.roffs.split(",")]
    libs = [bind(x) for x in a.libs]
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 1 << 30
    n = nbytes // 4 - 64
    pool = torch.empty(2 * nbytes + 4096, dtype=torch.uint8, device="cuda")
    base = pool.data_ptr()
    for off, bid in ((0, 2), (nbytes + 4096, 1)):
        dccl_amd.check(dccl_amd.synth_fill(base + off, 7, nbytes // 4, 0, 0xDCC1, bid, st), "synth")
    recv0, send0 = base, base + nbytes + 4096
    # phased k-way / chain: eight 1 GiB sources at +4 B, recv / own aligned
    srcs = torch.empty(8 * (nbytes + 4096) + 512, dtype=torch.uint8, device="cuda")
    sp = [srcs.data_ptr() + j * (nbytes + 4096) + 4 for j in range(8)]
    for j, q in enumerate(sp):
        dccl_amd.check(dccl_amd.synth_fill(q, 7, n, 0, 0xDCC1, 10 + j, st), "synth")
    arr4 = (ctypes.c_void_p * 4)(*sp[:4])
    arr7 = (ctypes.c_void_p * 7)(*sp[:7])
    cases = []
    for soff, roff, what in ((0, 0, "aligned"), (16, 0, "send off its lines"), (4, 0, "send 16-B phase +4"),
                             (1, 0, "send at byte offset 1"), (0, 1, "recv not element-aligned (+1)"),
                             (3, 2, "recv +2, send +3")):
        cases.append((f"pairwise: {what}", 3, lambda lib, s=soff, r=roff: lib.dccl_local_reduce(
            send0 + s, recv0 + r, 7, n, 0, st)))
    cases.append(("k-way k=4, sources +4 B (phased)", 6,
                  lambda lib: lib.dccl_local_reduce_multi(arr4, 4, recv0, 7, n, 0, st)))
    cases.append(("chain k=7, sources +4 B (phased)", 9,
                  lambda lib: lib.dccl_local_reduce_chain(arr7, 7, recv0, recv0, 7, n, 0, st)))
    arrp = {k: (ctypes.c_void_p * k)(*sp[:k]) for k in (5, 6, 8)}
    for k in (5, 6, 8):
        cases.append((f"k-way k={k}, sources +4 B (phased)", k + 2,
                      lambda lib, k=k: lib.dccl_local_reduce_multi(arrp[k], k, recv0, 7, n, 0, st)))
    arr4p = (ctypes.c_void_p * 4)(*sp[:4])
    for k, arr in ((4, arr4p), (6, arrp[6]), (8, arrp[8])):
        cases.append((f"chain k={k}, sources +4 B (phased)", k + 2,
                      lambda lib, k=k, arr=arr: lib.dccl_local_reduce_chain(arr, k, recv0, recv0, 7, n, 0, st)))
    sps = [q - 4 + 16 * (2 * j + 1) for j, q in enumerate(sp)]  # in phase, off recv's 128-B lines
    arrs = {k: (ctypes.c_void_p * k)(*sps[:k]) for k in (3, 4, 6, 7, 8)}
    for k in (4, 6, 7, 8):
        cases.append((f"k-way k={k}, sources off recv's lines (straddle)", k + 2,
                      lambda lib, k=k: lib.dccl_local_reduce_multi(arrs[k], k, recv0, 7, n, 0, st)))
    for k in (3, 4):
        cases.append((f"chain k={k}, sources off recv's lines (straddle)", k + 2,
                      lambda lib, k=k: lib.dccl_local_reduce_chain(arrs[k], k, recv0, recv0, 7, n, 0, st)))
    spb = [q - 4 + 1 for q in sp]  # sources at +1 B: not element-aligned
    arr4b = (ctypes.c_void_p * 4)(*spb[:4])
    arr7b = (ctypes.c_void_p * 7)(*spb[:7])
    cases.append(("k-way k=4, sources +1 B", 6, lambda lib: lib.dccl_local_reduce_multi(arr4b, 4, recv0, 7, n, 0, st)))
    cases.append(("k-way k=4, sources +4 B, recv +2 B", 6,
                  lambda lib: lib.dccl_local_reduce_multi(arr4, 4, recv0 + 2, 7, n, 0, st)))
    cases.append(("chain k=7, sources +1 B", 9,
                  lambda lib: lib.dccl_local_reduce_chain(arr7b, 7, recv0, recv0, 7, n, 0, st)))
    cases.append(("chain k=4, sources +4 B, own = dst +2 B", 6,
                  lambda lib: lib.dccl_local_reduce_chain(arr4, 4, recv0 + 2, recv0 + 2, 7, n, 0, st)))
    rows = []
    if a.tune_only:
        a.tune, cases = True, []
    for name, mult, call in cases:
        t = {0: [], 1: []}
        for _ in range(a.rounds):
            for i, lib in enumerate(libs):
                t[i].append(time_launches([lambda lib=lib: call(lib)], rounds=1, min_ms=20.0)[0])
        for i in (0, 1):
            ms = statistics.median(t[i])
            rows.append({"lib": os.path.basename(a.libs[i]), "case": name, "ms": round(ms, 4),
                         "frac": round(mult * n * 4 / (ms * 1e-3) / 1e9 / PEAK, 4)})
            print(json.dumps(rows[-1]), flush=True)
    if a.tune:
        from tools import tune_lib
        del srcs
        s2 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        r2 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        dccl_amd.check(dccl_amd.synth_fill(s2.data_ptr(), 7, nbytes // 4, 0, 0xDCC1, 3, st), "synth")
        dccl_amd.check(dccl_amd.synth_fill(r2.data_ptr(), 7, nbytes // 4, 0, 0xDCC1, 4, st), "synth")
        for layout, sb, rb in (("pooled", send0, recv0), ("separate", s2.data_ptr(), r2.data_ptr())):
            for roff in roffs:
                t = {v: [] for v in tvars}
                for _ in range(a.rounds):
                    for v in tvars:
                        fn = lambda v=v: tune_lib.lib.dccl_tune_misaligned_f32_sum(sb, rb + roff, n, v, st)
                        t[v].append(time_launches([fn], rounds=1, min_ms=20.0)[0])
                for v in tvars:
                    ms = statistics.median(t[v])
                    rows.append({"lib": "tune", "case": f"{layout}: misaligned recv +{roff} variant {v}",
                                 "ms": round(ms, 4), "frac": round(3 * n * 4 / (ms * 1e-3) / 1e9 / PEAK, 4)})
                    print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
