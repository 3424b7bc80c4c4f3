#!/usr/bin/env python3
"""A/B the fp32-Sum combine kernel variants in ONE process, interleaved rounds (MI355X).

Variants: UNROLL (16-B vectors per thread per operand in flight) x cache policy
(nt send / nt recv / nt store) x grid shape (one block per tile vs persistent grid).
Prints a JSON table of median / min kernel times and achieved HBM GB/s (3N bytes).

    python tools/tune_reduce.py [--mib 1024] [--rounds 7] [--iters 10]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mib", type=int, default=1024)
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--out", default="")
    a = p.parse_args()
    n = (a.mib << 20) // 4
    s = torch.rand(n, device="cuda")
    r = torch.rand(n, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    variants = []
    for unroll in (1, 2, 4, 8):
        for policy in (0, 1, 3, 5, 7):
            variants.append((unroll, policy, 0))
    for unroll in (2, 4, 8):
        for k in (2, 4, 8, 16):
            variants.append((unroll, 1, cus * k))
    times = {v: [] for v in variants}
    for v in variants:  # warm
        assert dccl_amd.lib.dccl_tune_reduce_f32_sum(s.data_ptr(), r.data_ptr(), n, v[0], v[1], v[2], st) == 0
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                dccl_amd.lib.dccl_tune_reduce_f32_sum(s.data_ptr(), r.data_ptr(), n, v[0], v[1], v[2], st)
            e1.record()
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.iters)
    rows = []
    for v, ts in times.items():
        med = statistics.median(ts)
        rows.append({"unroll": v[0], "policy": v[1], "grid_cap": v[2], "ms_median": round(med, 4),
                     "ms_min": round(min(ts), 4), "gb_s": round(3 * n * 4 / (med * 1e-3) / 1e9, 1)})
    rows.sort(key=lambda x: x["ms_median"])
    out = {"mib": a.mib, "cus": cus, "rows": rows}
    txt = json.dumps(out, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
