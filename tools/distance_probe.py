#!/usr/bin/env python3
"""Tuning only: the shipped fp32 Sum combine on two 1 GiB operands carved from ONE allocation, recv at its
start and send at a distance of 1 GiB + delta, for deltas from 0 to 1 GiB (interleaved over --rounds,
median of 5 launches each): does the operands' distance decide the placement mode?
    python tools/distance_probe.py [--rounds 3] [--out f.json]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402

PEAK = 8e12
MIB = 1 << 20
DELTAS = [0, 4096, 2 * MIB, 2 * MIB + 4096, 16 * MIB, 64 * MIB, 256 * MIB, 512 * MIB, 512 * MIB + 4096,
          768 * MIB, 1024 * MIB, 1024 * MIB + 4096]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--out", default="")
    a = p.parse_args()
    nbytes = 1 << 30
    n = nbytes // 4
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    pool = torch.empty(3 * nbytes + 8192, dtype=torch.uint8, device="cuda")
    base = pool.data_ptr()
    dccl_amd.check(dccl_amd.synth_fill(base, 7, (3 * nbytes + 8192) // 4, 0, 0xDCC1, 1, sh), "synth")
    torch.cuda.synchronize()

    def t_of(ps, pr):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        dccl_amd.check(dccl_amd.local_reduce(ps, pr, 7, n, 0, sh))
        e0.record(st)
        for _ in range(5):
            dccl_amd.check(dccl_amd.local_reduce(ps, pr, 7, n, 0, sh))
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / 5

    t = {d: [] for d in DELTAS}
    for _ in range(a.rounds):
        for d in DELTAS:
            t[d].append(t_of(base + nbytes + d, base))
    rows = [{"distance": nbytes + d, "delta": d, "frac": round(3 * nbytes / (statistics.median(t[d]) * 1e-3) / PEAK, 4)}
            for d in DELTAS]
    for r in rows:
        print(json.dumps(r), flush=True)
    # a second allocation of the same size for comparison: separate operands on this box
    other = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dccl_amd.check(dccl_amd.synth_fill(other.data_ptr(), 7, n, 0, 0xDCC1, 2, sh), "synth")
    ts = [t_of(other.data_ptr(), base) for _ in range(a.rounds)]
    rows.append({"separate": True, "frac": round(3 * nbytes / (statistics.median(ts) * 1e-3) / PEAK, 4),
                 "distance": other.data_ptr() - base})
    print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
