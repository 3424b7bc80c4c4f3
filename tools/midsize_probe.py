#!/usr/bin/env python3
"""Tuning only: kernel shapes for mid-size combines (BASELINE C4's 1-64 MiB range), fp32 Sum.

Each (size, variant) runs as HIP-graph replays of 100 launches cycling over operand sets spread across
8 GiB (as bench.py's c4 leg, so the Infinity Cache does not hold them), interleaved over --rounds; the
variants are the tuning library's template shapes (block x vectors per lane x cache policy,
dccl_tune_reduce_f32_sum) plus the shipped dccl_local_reduce.  Prints us per launch and % of HBM peak.
    python tools/midsize_probe.py [--rounds 3] [--out f.json]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402
from tools import tune_lib  # noqa: E402

PEAK = 8e12
SHAPES = [(64, 1, 7), (64, 2, 7), (64, 4, 7), (128, 1, 7), (256, 1, 7), (256, 2, 7), (256, 4, 7), (1024, 1, 7)]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--out", default="")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    info = tune_lib.tune_variants()
    idx = {}
    for shape in SHAPES:
        for v, d in enumerate(info):
            if (d["block"], d["unroll"], d["policy"], d["xcd"]) == (*shape, 0):
                idx[shape] = v
    top = 4 << 30
    pool = torch.empty(2 * top + 4096, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    dccl_amd.check(dccl_amd.synth_fill(pool.data_ptr(), 7, top // 4, 0, 0xDCC1, 1, st), "synth")
    dccl_amd.check(dccl_amd.synth_fill(pool.data_ptr() + top + 4096, 7, top // 4, 0, 0xDCC1, 2, st), "synth")
    pr0, ps0 = pool.data_ptr(), pool.data_ptr() + top + 4096
    side = torch.cuda.Stream(dev)
    rows = []
    for mib in (1, 2, 4, 8, 16, 32, 64):
        nb = mib << 20
        n = nb // 4
        sets = max(2, (512 << 20) // (2 * nb))
        stride = top // sets // 4096 * 4096
        pairs = [(ps0 + j * stride, pr0 + j * stride) for j in range(sets)]
        graphs = {}
        names = ["shipped"] + [f"{b}x{u} pol{pol}" for b, u, pol in SHAPES if (b, u, pol) in idx]
        for name in names:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(side):
                def call(ps, pr, name=name):
                    if name == "shipped":
                        return dccl_amd.local_reduce(ps, pr, 7, n, 0, side.cuda_stream)
                    b, u, pol = (int(x) for x in name.replace("x", " ").replace(" pol", " ").split())
                    return tune_lib.lib.dccl_tune_reduce_f32_sum(ps, pr, n, idx[(b, u, pol)], 0, side.cuda_stream)
                dccl_amd.check(call(*pairs[0]), name)
                side.synchronize()
                with torch.cuda.graph(g, stream=side):
                    for i in range(100):
                        dccl_amd.check(call(*pairs[i % sets]), name)
            graphs[name] = g
        t = {name: [] for name in names}
        cur = torch.cuda.current_stream(dev)
        for _ in range(a.rounds):
            for name in names:
                g = graphs[name]
                g.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(cur)
                for _ in range(5):
                    g.replay()
                e1.record(cur)
                e1.synchronize()
                t[name].append(e0.elapsed_time(e1) * 1e3 / 500)
        for name in names:
            us = statistics.median(t[name])
            rows.append({"mib": mib, "shape": name, "us": round(us, 2), "frac": round(3 * nb / (us * 1e-6) / PEAK, 4)})
            print(json.dumps(rows[-1]), flush=True)
        del graphs
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
