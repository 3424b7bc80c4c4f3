#!/usr/bin/env python3
"""Separately allocated operand pairs (tuning only): DCCL's own layout (scratchpad + user chunk) lands in
one of several physical placements.  Allocates --pairs pairs of 1 GiB fp32 operands,
and for each pair times the shipped combine and a few vector-kernel variants (cache policy, block size,
XCD order, occupancy cap), interleaved, to see whether any shape is robust to the placement.
    python tools/pair_probe.py [--pairs 8] [--rounds 3] [--out f.json]
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
from tools.bench_suite import PEAK, time_launches  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pairs", type=int, default=8)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--out", default="")
    a = p.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 1 << 30
    n = nbytes // 4
    pairs = []
    for i in range(a.pairs):
        s = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        r = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        dccl_amd.check(dccl_amd.synth_fill(s.data_ptr(), 7, n, 0, 0xDCC1, 2 * i, st), "synth")
        dccl_amd.check(dccl_amd.synth_fill(r.data_ptr(), 7, n, 0, 0xDCC1, 2 * i + 1, st), "synth")
        pairs.append((s, r))
    vinfo = tune_lib.tune_variants()
    want = {(64, 1, 7, 0): "64x1 nt (shipped shape)", (64, 1, 6, 0): "64x1 send cached",
            (64, 1, 7, 1): "64x1 xcd", (128, 1, 7, 0): "128x1", (256, 1, 7, 0): "256x1"}
    variants = [(i, want[(v["block"], v["unroll"], v["policy"], v["xcd"])]) for i, v in enumerate(vinfo)
                if (v["block"], v["unroll"], v["policy"], v["xcd"]) in want]
    rows = []
    for pi, (s, r) in enumerate(pairs):
        ps, pr = s.data_ptr(), r.data_ptr()
        cases = [("production", lambda: dccl_amd.local_reduce(ps, pr, 7, n, 0, st))]
        cases += [(name, lambda i=i: tune_lib.lib.dccl_tune_reduce_f32_sum(ps, pr, n, i, 0, st)) for i, name in variants]
        cases.append(("64x1 nt, 22 waves/CU (LDS cap)",
                      lambda: tune_lib.lib.dccl_tune_reduce_f32_sum_lds(ps, pr, n, 0, 0, 7168, st)))
        t = {k: [] for k in range(len(cases))}
        for _ in range(a.rounds):
            for k, (_, fn) in enumerate(cases):
                t[k].append(time_launches([fn], rounds=1, min_ms=15.0)[0])
        for k, (name, _) in enumerate(cases):
            ms = statistics.median(t[k])
            rows.append({"pair": pi, "delta_mib": round((pr - ps) / 2**20, 1), "variant": name, "ms": round(ms, 4),
                         "frac": round(3 * nbytes / (ms * 1e-3) / 1e9 / PEAK, 4)})
            print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
