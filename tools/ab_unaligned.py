#!/usr/bin/env python3
"""A/B of the unaligned-destination k-way / chain variants (tools/tune/unaligned_v4.hip) against the product
kernels, fp32 Sum, 1 GiB per operand (tuning only).  Operands: ten 1 GiB buffers from one
allocation, 4 KiB x (j+1) stagger (tools/ab_cases.py's layout).  Every case is checked bit for bit against
the product on a 1 Mi-element slice, then timed interleaved (HIP events around --launches back-to-back
launches per round, median over --rounds), as a fraction of (k+2) * N * 4 B at 8 TB/s.

    python tools/ab_unaligned.py [--variants 110,260110,...] [--ks 4,8] [--cases ...] [--rounds 5] [--out f.json]

Variant codes: tools/tune/unaligned_v4.hip (10000 * waves + 1000 * loads-first + 100 * order + 10).
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
LIB = os.path.join(ROOT, "tools", "lib", "libunaligned_v4.so")


def cases(ptrs, ks):
    recv, src = ptrs[0], ptrs[1:9]
    t = {}
    for k in ks:
        for so, sname in ((0, ""), (4, "_src+4")):
            s = [p + so for p in src[:k]]
            t[f"multi{k}_dst+2{sname}"] = (k, s, None, recv + 2)
            t[f"chain{k}_dst+2{sname}"] = (k, s, recv + 2, recv + 2)
        t[f"chain{k}_src+4"] = (k, [p + 4 for p in src[:k]], recv, recv)
        t[f"multi{k}_src+4"] = (k, [p + 4 for p in src[:k]], None, recv)
        t[f"chain{k}"] = (k, src[:k], recv, recv)  # every operand in phase and on the line grid
        t[f"multi{k}"] = (k, src[:k], None, recv)
        strad = [p + 16 * (2 * j + 1) for j, p in enumerate(src[:k])]  # in phase, off recv's 128-B lines
        t[f"chain{k}_strad"] = (k, strad, recv, recv)
        t[f"multi{k}_strad"] = (k, strad, None, recv)
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="110,260110,121110,121210")
    ap.add_argument("--ks", default="4,8")
    ap.add_argument("--mib", type=int, default=1024, help="bytes per operand (MiB)")
    ap.add_argument("--cases", default="")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    uv = ctypes.CDLL(LIB)
    uv.uv4_combine.restype = ctypes.c_int
    uv.uv4_combine.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    lib = dccl_amd.lib
    st = torch.cuda.current_stream().cuda_stream
    nbytes = a.mib << 20
    n = nbytes // 4 - 64
    pool = torch.empty(10 * nbytes + 4096 * 55 + 1024, dtype=torch.uint8, device="cuda")
    ptrs, off = [], 0
    for j in range(10):
        ptrs.append(pool.data_ptr() + off)
        dccl_amd.check(dccl_amd.synth_fill(ptrs[-1], 7, nbytes // 4, 0, 0xDCC1, 10 + j, st), "synth")
        off += nbytes + 4096 * (j + 1)
    table = cases(ptrs, [int(x) for x in a.ks.split(",")])
    names = a.cases.split(",") if a.cases else list(table)
    variants = [int(v) for v in a.variants.split(",")]

    def call(v, name, count):
        k, s, own, dst = table[name]
        arr = (ctypes.c_void_p * k)(*s)
        if v < 0:  # the product
            if own is None:
                return lib.dccl_local_reduce_multi(arr, k, dst, 7, count, 0, st)
            return lib.dccl_local_reduce_chain(arr, k, own, dst, 7, count, 0, st)
        return uv.uv4_combine(v, arr, k, own, dst, count, st)

    # bit-exactness against the product on a 1 Mi-element slice (the destination restored between runs)
    m = 1 << 20
    region = pool[: 4 * m + 64]
    saved = region.clone()
    exact = {}
    for name in names:
        outs = []
        for v in [-1] + variants:
            region.copy_(saved)
            torch.cuda.synchronize()
            assert call(v, name, m + 3) == 0, (v, name)
            torch.cuda.synchronize()
            outs.append(region.clone())
        exact[name] = [bool(torch.equal(outs[0], o)) for o in outs[1:]]
    region.copy_(saved)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {(name, v): [] for name in names for v in [-1] + variants}
    for _ in range(a.rounds):
        for name in names:
            for v in [-1] + variants:
                assert call(v, name, n) == 0
                ev0.record()
                for _ in range(a.launches):
                    call(v, name, n)
                ev1.record()
                ev1.synchronize()
                times[(name, v)].append(ev0.elapsed_time(ev1) / a.launches)
    rows = []
    for name in names:
        k = table[name][0]
        fr = {v: round((k + 2) * n * 4 / (statistics.median(times[(name, v)]) * 1e-3) / PEAK, 4) for v in [-1] + variants}
        best = max(variants, key=lambda v: fr[v])
        rows.append({"case": name, "k": k, "product": fr[-1], "variants": {str(v): fr[v] for v in variants},
                     "best": best, "best_delta_points": round(100 * (fr[best] - fr[-1]), 2),
                     "bit_exact": dict(zip(map(str, variants), exact[name]))})
        print(f"{name:22s} product {100 * fr[-1]:6.2f}%  best {best:4d} {100 * fr[best]:6.2f}%  " +
              " ".join(f"{v}:{100 * fr[v]:.1f}" for v in variants) + f"  exact {all(exact[name])}", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"count": n, "rounds": a.rounds, "launches": a.launches, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
