#!/usr/bin/env python3
"""Pairwise combine: deeper per-lane unroll / fatter blocks under resident-wave caps (MI355X).

The shipped shape (one-wave blocks, one 16-B vector per lane and operand, 32 resident waves per CU) was chosen
over unroll 2/4 and 128-1024-thread blocks uncapped (profiles/r1_tune_shapes.json), and the one-vector kernel
under caps (profiles/r1_tune_occupancy_sweep.json).  Deeper unroll at full occupancy doubles or quadruples the
reads in flight per CU; this probe asks whether unroll 2/4 at 1/2 or 1/4 of the waves (the same bytes in flight
as the shipped launch, half or a quarter of the workgroups to dispatch) is faster.  fp32 Sum, 1 GiB per operand,
the bench's pooled layout (recv, send 4 KiB past its end), recv aligned to 128 B like production
(DCCL_TUNE_ALIGN=128), interleaved rounds in one process.

    python tools/unroll_cap_probe.py [--mib 1024] [--rounds 7] [--iters 10] [--out file]
"""
import argparse
import json
import os
import statistics
import sys

os.environ.setdefault("DCCL_TUNE_ALIGN", "128")
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import tune_lib  # noqa: E402

LDS_PER_CU = 160 << 10


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mib", type=int, default=1024)
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--out", default="")
    p.add_argument("--layout", default="pooled", choices=["pooled", "separate"])
    a = p.parse_args()
    nb = a.mib << 20
    n = nb // 4
    if a.layout == "pooled":
        pool = torch.empty(2 * nb + 4096, dtype=torch.uint8, device="cuda")
        recv, send = pool[:nb], pool[nb + 4096:]
    else:  # two allocations (DCCL's scratchpad + user chunk)
        recv = torch.empty(nb, dtype=torch.uint8, device="cuda")
        send = torch.empty(nb, dtype=torch.uint8, device="cuda")
    recv.view(torch.float32).uniform_(-1, 1)
    send.view(torch.float32).uniform_(-1, 1)
    pr, ps = recv.data_ptr(), send.data_ptr()
    st = torch.cuda.current_stream().cuda_stream
    info = tune_lib.tune_variants()
    want = {(64, 1, 7, 0), (64, 2, 7, 0), (64, 4, 7, 0), (128, 1, 7, 0), (256, 1, 7, 0), (256, 4, 7, 0)}
    cases = {}
    for v, inf in enumerate(info):
        key = (inf["block"], inf["unroll"], inf["policy"], inf["xcd"])
        if key not in want:
            continue
        wpb = inf["block"] // 64
        for waves in (32, 24, 20, 16, 12, 8):
            if waves % wpb or (waves < 32 and waves // wpb < 1):
                continue
            blocks = waves // wpb
            lds = 0 if waves == 32 else (LDS_PER_CU // blocks + 255) // 256 * 256
            if lds > (64 << 10):
                continue
            cases[(v, waves)] = ({**inf, "waves_per_cu": waves, "lds_bytes": lds,
                                  "bytes_in_flight_per_cu": waves * 64 * 16 * 2 * inf["unroll"]},
                                 lambda v=v, lds=lds: tune_lib.lib.dccl_tune_reduce_f32_sum_lds(ps, pr, n, v, 0, lds, st))
    for k, (_, fn) in cases.items():
        assert fn() == 0, k
    torch.cuda.synchronize()
    times = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, (_, fn) in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / a.iters)
    rows = []
    for k, ts in times.items():
        med = statistics.median(ts)
        rows.append({**cases[k][0], "ms_median": round(med, 4), "ms_min": round(min(ts), 4),
                     "frac": round(3 * nb / (med * 1e-3) / 1e9 / 8000.0, 4)})
    rows.sort(key=lambda x: x["ms_median"])
    out = {"mib": a.mib, "layout": a.layout, "rows": rows}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    for row in rows:
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
