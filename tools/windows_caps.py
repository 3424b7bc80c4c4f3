#!/usr/bin/env python3
"""Resident-wave cap sweep of the misaligned-destination k-way / chain launches (reduce_windows_kernel,
DESIGN.md §3.4; tuning only): the product library's dccl_local_reduce_multi / _chain with DCCL_WINDOWS_WAVES set
per timing loop (read at every launch), fp32 Sum, 1 GiB per operand, destination +2 B, sources in phase or
+4 B; ten operands from one allocation (tools/ab_cases.py's layout).  Every cap of a case is timed in every
round (interleaved), median over --rounds; fraction of (k+2) * N * 4 B at 8 TB/s.

    python tools/windows_caps.py [--ks 3,4,6,8] [--waves 32,24,20,16,13,11,9] [--rounds 5] [--out f.json]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="3,4,6,8")
    ap.add_argument("--waves", default="32,24,20,16,13,11,9")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    lib = dccl_amd.lib
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 1 << 30
    n = nbytes // 4 - 64
    pool = torch.empty(10 * nbytes + 4096 * 55 + 1024, dtype=torch.uint8, device="cuda")
    ptrs, off = [], 0
    for j in range(10):
        ptrs.append(pool.data_ptr() + off)
        dccl_amd.check(dccl_amd.synth_fill(ptrs[-1], 7, nbytes // 4, 0, 0xDCC1, 10 + j, st), "synth")
        off += nbytes + 4096 * (j + 1)
    recv, src = ptrs[0], ptrs[1:9]
    cases = {}
    for k in (int(x) for x in a.ks.split(",")):
        for so, sname in ((0, ""), (4, "_src+4")):
            arr = (ctypes.c_void_p * k)(*[p + so for p in src[:k]])
            cases[f"multi{k}_dst+2{sname}"] = (k, lambda c, arr=arr, k=k: lib.dccl_local_reduce_multi(
                arr, k, recv + 2, 7, c, 0, st))
            cases[f"chain{k}_dst+2{sname}"] = (k, lambda c, arr=arr, k=k: lib.dccl_local_reduce_chain(
                arr, k, recv + 2, recv + 2, 7, c, 0, st))
    waves = [int(w) for w in a.waves.split(",")]
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {(c, w): [] for c in cases for w in waves}
    for _ in range(a.rounds):
        for name, (k, call) in cases.items():
            for w in waves:
                os.environ["DCCL_WINDOWS_WAVES"] = str(w)
                assert call(n) == 0
                ev0.record()
                for _ in range(a.launches):
                    call(n)
                ev1.record()
                ev1.synchronize()
                times[(name, w)].append(ev0.elapsed_time(ev1) / a.launches)
    os.environ.pop("DCCL_WINDOWS_WAVES", None)
    rows = []
    for name, (k, _) in cases.items():
        fr = {w: round((k + 2) * n * 4 / (statistics.median(times[(name, w)]) * 1e-3) / 8e12, 4) for w in waves}
        best = max(waves, key=lambda w: fr[w])
        rows.append({"case": name, "k": k, "frac": {str(w): fr[w] for w in waves}, "best_waves": best,
                     "gain_over_uncapped_points": round(100 * (fr[best] - fr[32]), 2) if 32 in fr else None})
        print(f"{name:22s} " + " ".join(f"{w}:{100 * fr[w]:.1f}" for w in waves) + f"  best {best}", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"count": n, "rounds": a.rounds, "launches": a.launches, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
