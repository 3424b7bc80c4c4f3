#!/usr/bin/env python3
"""Tuning only: the shifted kernel (send at another 16-B phase or a byte offset, recv element-aligned)
under wave caps, 1 GiB fp32 Sum, pooled layout, interleaved over --rounds.
    python tools/shift_cap_probe.py [--rounds 3] [--out f.json]
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
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--out", default="")
    a = p.parse_args()
    nbytes = 1 << 30
    n = nbytes // 4 - 64
    st = torch.cuda.current_stream().cuda_stream
    pool = torch.empty(2 * nbytes + 4096, dtype=torch.uint8, device="cuda")
    base = pool.data_ptr()
    for off, bid in ((0, 2), (nbytes + 4096, 1)):
        dccl_amd.check(dccl_amd.synth_fill(base + off, 7, nbytes // 4, 0, 0xDCC1, bid, st), "synth")
    waves = [32, 28, 26, 24, 22, 20]
    rows = []
    for soff in (4, 1, 20):
        t = {w: [] for w in waves}
        for _ in range(a.rounds):
            for w in waves:
                lds = 0 if w >= 32 else ((160 << 10) // w + 255) // 256 * 256
                fn = lambda lds=lds: dccl_amd.check(tune_lib.lib.dccl_tune_shift_caps_f32_sum(
                    base + nbytes + 4096 + soff, base, n, lds, st), "shift")
                t[w].append(time_launches([fn], rounds=1, min_ms=20.0)[0])
        for w in waves:
            ms = statistics.median(t[w])
            rows.append({"send_offset": soff, "waves": w, "frac": round(3 * n * 4 / (ms * 1e-3) / 1e9 / PEAK, 4)})
            print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
