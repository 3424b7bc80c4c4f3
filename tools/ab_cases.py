#!/usr/bin/env python3
"""A/B of two builds of the product library on the alignment classes of tools/issue_probe.py (tuning only):
both libraries loaded side by side (RTLD_LOCAL), every case timed interleaved on the same operands (ten 1 GiB
fp32 operands from one allocation, 4 KiB x (j+1) stagger), HIP events around --launches back-to-back
launches per round, the median over --rounds rounds reported per library; each case's result is also
compared bit for bit between the two libraries at the timed count (so at the size whose dispatch is timed).

    python tools/ab_cases.py LIB_A LIB_B [--cases pair_dst+1,multi4_dst+2] [--rounds 5] [--out f.json]
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


def bind(path):
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    c_int, c_size_t, c_void_p = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p
    lib.dccl_local_reduce.restype = c_int
    lib.dccl_local_reduce.argtypes = [c_void_p, c_void_p, c_int, c_size_t, c_int, c_void_p]
    for f in (lib.dccl_local_reduce_multi,):
        f.restype = c_int
        f.argtypes = [ctypes.POINTER(c_void_p), c_int, c_void_p, c_int, c_size_t, c_int, c_void_p]
    lib.dccl_local_reduce_chain.restype = c_int
    lib.dccl_local_reduce_chain.argtypes = [ctypes.POINTER(c_void_p), c_int, c_void_p, c_void_p, c_int, c_size_t,
                                            c_int, c_void_p]
    return lib


def case_table(ptrs):
    """name -> (k, call(lib, count, stream)); destination ptrs[0], sources ptrs[1..8] (the pair is bench.py's
    pooled layout: send 4 KiB past the end of recv)."""
    recv, ptrs = ptrs[0], ptrs[1:9]

    def arr(ps):
        return (ctypes.c_void_p * len(ps))(*ps)

    def multi(ps, dst):
        a = arr(ps)
        return lambda lib, n, st: lib.dccl_local_reduce_multi(a, len(ps), dst, 7, n, 0, st)

    def chain(ps, own, dst):
        a = arr(ps)
        return lambda lib, n, st: lib.dccl_local_reduce_chain(a, len(ps), own, dst, 7, n, 0, st)

    t = {
        "pair": (1, lambda lib, n, st: lib.dccl_local_reduce(ptrs[0], recv, 7, n, 0, st)),
        "pair_dst+1": (1, lambda lib, n, st: lib.dccl_local_reduce(ptrs[0], recv + 1, 7, n, 0, st)),
        "pair_dst+2_src+3": (1, lambda lib, n, st: lib.dccl_local_reduce(ptrs[0] + 3, recv + 2, 7, n, 0, st)),
        "pair_src+4": (1, lambda lib, n, st: lib.dccl_local_reduce(ptrs[0] + 4, recv, 7, n, 0, st)),
    }
    for k in (2, 3, 4, 5, 6, 7, 8):
        t[f"multi{k}"] = (k, multi(ptrs[:k], recv))
        t[f"multi{k}_dst+2"] = (k, multi(ptrs[:k], recv + 2))
        t[f"multi{k}_dst+2_src+4"] = (k, multi([p + 4 for p in ptrs[:k]], recv + 2))
        t[f"multi{k}_src+4"] = (k, multi([p + 4 for p in ptrs[:k]], recv))
        t[f"multi{k}_strad"] = (k, multi([p + 16 * (2 * j + 1) for j, p in enumerate(ptrs[:k])], recv))
        t[f"chain{k}"] = (k, chain(ptrs[:k], recv, recv))
        t[f"chain{k}_dst+2"] = (k, chain(ptrs[:k], recv + 2, recv + 2))
        t[f"chain{k}_dst+2_src+4"] = (k, chain([p + 4 for p in ptrs[:k]], recv + 2, recv + 2))
        t[f"chain{k}_src+4"] = (k, chain([p + 4 for p in ptrs[:k]], recv, recv))
        t[f"chain{k}_strad"] = (k, chain([p + 16 * (2 * j + 1) for j, p in enumerate(ptrs[:k])], recv, recv))
        # element-aligned destinations off the 128-B line grid (phased launches)
        t[f"multi{k}_dst+4"] = (k, multi(ptrs[:k], recv + 4))
        t[f"chain{k}_dst+4"] = (k, chain(ptrs[:k], recv + 4, recv + 4))
        t[f"multi{k}_dst+16_src+4"] = (k, multi([p + 4 for p in ptrs[:k]], recv + 16))
        t[f"chain{k}_dst+16_src+4"] = (k, chain([p + 4 for p in ptrs[:k]], recv + 16, recv + 16))
    return t


def main():
    p = argparse.ArgumentParser()
    p.add_argument("libs", nargs=2)
    p.add_argument("--cases", default="pair,pair_dst+1,pair_dst+2_src+3,multi2_dst+2,multi4_dst+2,multi8_dst+2,"
                                      "multi2_dst+2_src+4,multi4_dst+2_src+4,multi8_dst+2_src+4,chain2_dst+2,"
                                      "chain4_dst+2,chain8_dst+2,chain4_dst+2_src+4,chain8_dst+2_src+4,multi4,"
                                      "multi8_strad,multi6_src+4")
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--launches", type=int, default=10)
    p.add_argument("--mib", type=int, default=1024)
    p.add_argument("--out", default="")
    p.add_argument("--all-k", default="", help="comma-separated case stems expanded over k = 2..8, e.g. multi,chain_strad")
    a = p.parse_args()
    libs = [bind(x) for x in a.libs]
    st = torch.cuda.current_stream().cuda_stream
    nbytes = a.mib << 20
    n = nbytes // 4 - 64
    pool = torch.empty(10 * nbytes + 4096 * 55 + 1024, dtype=torch.uint8, device="cuda")
    ptrs, off = [], 0
    for j in range(10):
        ptrs.append(pool.data_ptr() + off)
        dccl_amd.check(dccl_amd.synth_fill(ptrs[-1], 7, nbytes // 4, 0, 0xDCC1, 10 + j, st), "synth")
        off += nbytes + 4096 * (j + 1)
    table = case_table(ptrs)
    names = a.cases.split(",") if a.cases else []
    for stem in filter(None, a.all_k.split(",")):
        head, _, tail = stem.partition("_")
        names += [f"{head}{k}" + (f"_{tail}" if tail else "") for k in range(2, 9)]
    # bit-exactness of B against A at the timed count (the destination restored between the two runs)
    exact = {}
    m = n
    for name in names:
        k, call = table[name]
        dst = ptrs[0]
        saved = torch.empty(4 * m + 64, dtype=torch.uint8, device="cuda")
        region = pool[: 4 * m + 64]
        assert region.data_ptr() == dst
        saved.copy_(region)
        outs = []
        for lib in libs:
            region.copy_(saved)
            torch.cuda.synchronize()
            assert call(lib, m, st) == 0
            torch.cuda.synchronize()
            outs.append(region.clone())
        exact[name] = bool(torch.equal(outs[0], outs[1]))
        region.copy_(saved)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {(name, i): [] for name in names for i in range(2)}
    for _ in range(a.rounds):
        for name in names:
            k, call = table[name]
            for i, lib in enumerate(libs):
                assert call(lib, n, st) == 0
                ev0.record()
                for _ in range(a.launches):
                    call(lib, n, st)
                ev1.record()
                ev1.synchronize()
                times[(name, i)].append(ev0.elapsed_time(ev1) / a.launches)
    rows = []
    for name in names:
        k = table[name][0]
        fr = [round((k + 2) * n * 4 / (statistics.median(times[(name, i)]) * 1e-3) / PEAK, 4) for i in range(2)]
        rows.append({"case": name, "k": k, "frac_a": fr[0], "frac_b": fr[1], "delta_points": round(100 * (fr[1] - fr[0]), 2),
                     "bit_exact_b_vs_a": exact[name]})
        print(f"{name:22s} A {100 * fr[0]:6.2f}%  B {100 * fr[1]:6.2f}%  ({100 * (fr[1] - fr[0]):+.2f})  exact {exact[name]}",
              flush=True)
    res = {"libs": a.libs, "bytes_per_operand": nbytes, "count": n, "rounds": a.rounds, "launches": a.launches,
           "rows": rows}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
