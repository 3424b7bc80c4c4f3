#!/usr/bin/env python3
"""How much does the physical placement of the two 1 GiB operands move the combine? (MI355X)

Times the shipped fp32-Sum combine (dccl_local_reduce) on:
  sep-k      two separate torch allocations (as bench.py), re-allocated k times
  one-d      one allocation, recv at 0 and send at 1 GiB + d (d = 0, 4 KiB, 64 KiB, 2 MiB)
  hip-sep    two separate hipMalloc allocations (outside torch's caching allocator)
  big-sep    two separate 2 GiB allocations, operands at their starts
"""
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402
from tools import tune_lib  # noqa: E402

N = (1 << 30) // 4
ST = 0


VARIANTS = {}


def timeit(sp, rp, rounds=10, iters=10, variant=None):
    st = torch.cuda.current_stream().cuda_stream
    if variant is None:
        call = lambda: dccl_amd.local_reduce(sp, rp, 7, N, 0, st)
    else:
        call = lambda: tune_lib.lib.dccl_tune_reduce_f32_sum_lds(sp, rp, N, variant, 0, 7 << 10, st)
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            call()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / iters)
    med = statistics.median(ts)
    return {"ms": round(med, 4), "gb_s": round(3 * N * 4 / (med * 1e-3) / 1e9, 1)}


def main():
    rows = []
    info = tune_lib.tune_variants()
    v_plain = next(i for i, v in enumerate(info) if v == {"block": 64, "unroll": 1, "policy": 7, "xcd": 0})
    v_xcd = next(i for i, v in enumerate(info) if v == {"block": 64, "unroll": 1, "policy": 7, "xcd": 1})
    keep = []  # hold allocations so later pairs land elsewhere in physical memory
    for k in range(6):
        s = torch.empty(N, device="cuda").uniform_(-1, 1)
        r = torch.empty(N, device="cuda").uniform_(-1, 1)
        row = {"case": f"sep-{k}", "delta_mib": (s.data_ptr() - r.data_ptr()) / 2**20,
               "shipped": timeit(s.data_ptr(), r.data_ptr())["ms"],
               "plain_capped": timeit(s.data_ptr(), r.data_ptr(), variant=v_plain)["ms"],
               "xcd_capped": timeit(s.data_ptr(), r.data_ptr(), variant=v_xcd)["ms"]}
        rows.append(row)
        print(row, flush=True)
        if k % 2:
            keep.append((s, r))
        else:
            del s, r
        torch.cuda.empty_cache()
    del keep
    torch.cuda.empty_cache()
    big = torch.empty(2 * N + (4 << 20) // 4, device="cuda").uniform_(-1, 1)
    for d in (0, 4096, 65536, 2 << 20):
        rp = big.data_ptr()
        rows.append({"case": f"one-{d}", **timeit(rp + N * 4 + d, rp)})
        print(rows[-1], flush=True)
    del big
    torch.cuda.empty_cache()
    hip = ctypes.CDLL("libamdhip64.so.7")
    ps, pr = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(ps), ctypes.c_size_t(N * 4)) == 0
    assert hip.hipMalloc(ctypes.byref(pr), ctypes.c_size_t(N * 4)) == 0
    hip.hipMemset(ps, 0, ctypes.c_size_t(N * 4))
    hip.hipMemset(pr, 0, ctypes.c_size_t(N * 4))
    rows.append({"case": "hip-sep", "delta_mib": (ps.value - pr.value) / 2**20, **timeit(ps.value, pr.value)})
    print(rows[-1], flush=True)
    hip.hipFree(ps)
    hip.hipFree(pr)
    s = torch.zeros(2 * N, device="cuda")
    r = torch.zeros(2 * N, device="cuda")
    rows.append({"case": "big-sep", "delta_mib": (s.data_ptr() - r.data_ptr()) / 2**20,
                 **timeit(s.data_ptr(), r.data_ptr())})
    print(rows[-1], flush=True)
    if len(sys.argv) > 1:
        json.dump(rows, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
