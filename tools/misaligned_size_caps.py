#!/usr/bin/env python3
"""Tuning only: the misaligned-recv kernel's wave cap (kUnalignedWaves = 24, tuned at 1 GiB) at smaller operands.
fp32 Sum, recv +1 B, send aligned, operand sets rotated past the Infinity Cache below 1 GiB; the kernel uncapped
(tuning variant 16), at 26 waves (20) and at 24 waves (25), and the product entry point; median of interleaved
rounds, fraction of 3N at 8 TB/s.
    python tools/misaligned_size_caps.py [--sizes 16,32,64,128,1024] [--rounds 5] [--out f.json]
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

VARIANTS = {"uncapped": 16, "26 waves": 20, "24 waves (shipped)": 25}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--sizes", default="16,32,64,128,1024")
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--out", default="")
    a = p.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    gib = 1 << 30
    pool = torch.empty(2 * gib + 8192, dtype=torch.uint8, device="cuda")
    r0, s0 = pool.data_ptr(), pool.data_ptr() + gib + 4096
    dccl_amd.check(dccl_amd.synth_fill(r0, 7, gib // 4, 0, 0xDCC1, 1, st), "synth")
    dccl_amd.check(dccl_amd.synth_fill(s0, 7, gib // 4, 0, 0xDCC1, 2, st), "synth")
    rows = []
    for mib in (int(x) for x in a.sizes.split(",")):
        nb = mib << 20
        n = nb // 4 - 64
        sets = max(1, min(8, gib // nb))
        configs = list(VARIANTS) + ["product"]
        t = {c: [] for c in configs}
        launches = max(10, min(400, int(0.02 / (3 * nb / 6.0e12))))
        for _ in range(a.rounds):
            for c in configs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(launches):
                    off = (i % sets) * nb
                    if c == "product":
                        rc = dccl_amd.local_reduce(s0 + off, r0 + off + 1, 7, n, 0, st)
                    else:
                        rc = tune_lib.lib.dccl_tune_misaligned_f32_sum(s0 + off, r0 + off + 1, n, VARIANTS[c], st)
                    assert rc == 0, (c, rc)
                e1.record()
                e1.synchronize()
                t[c].append(e0.elapsed_time(e1) / launches)
        for c in configs:
            ms = statistics.median(t[c])
            rows.append({"mib": mib, "config": c, "sets": sets, "us": round(ms * 1e3, 2),
                         "frac": round(3 * n * 4 / (ms * 1e-3) / 1e9 / 8000.0, 4)})
            print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
