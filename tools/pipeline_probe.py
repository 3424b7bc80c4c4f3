#!/usr/bin/env python3
"""Persistent software-pipelined combine against the shipped one-wave-per-tile grid (tuning only): fp32 Sum,
1 GiB operands in bench.py's pooled layout; persistent grids of 256 x {1, 2, 4, 8, 16, 32} one-wave blocks with
one or two tiles of loads in flight ahead; results checked bit-exact against the shipped kernel first.
    python tools/pipeline_probe.py [--rounds 5] [--out f.json]
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
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--out", default="")
    a = p.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 1 << 30
    n = nbytes // 4
    pool = torch.empty(2 * nbytes + 4096, dtype=torch.uint8, device="cuda")
    recv, send = pool[:nbytes], pool[nbytes + 4096:]
    dccl_amd.check(dccl_amd.synth_fill(send.data_ptr(), 7, n, 0, 0xDCC1, 0, st), "synth")
    dccl_amd.check(dccl_amd.synth_fill(recv.data_ptr(), 7, n, 0, 0xDCC1, 1, st), "synth")
    variants = [(d, g) for d in (1, 2) for g in (256 * 1, 256 * 2, 256 * 4, 256 * 8, 256 * 16, 256 * 32)]
    # correctness: one launch of each variant from the same starting recv equals the shipped kernel's
    r0 = recv.clone()
    want = r0.clone()
    dccl_amd.check(dccl_amd.local_reduce(send.data_ptr(), want.data_ptr(), 7, n, 0, st), "ref")
    for d, g in variants:
        got = r0.clone()
        assert tune_lib.lib.dccl_tune_pipelined_f32_sum(send.data_ptr(), got.data_ptr(), n, d, g, st) == 0
        torch.cuda.synchronize()
        assert torch.equal(got, want), (d, g)
        del got
    del r0, want
    torch.cuda.empty_cache()
    ps, pr = send.data_ptr(), recv.data_ptr()
    cases = [("shipped (one tile per one-wave block)", lambda: dccl_amd.local_reduce(ps, pr, 7, n, 0, st))]
    cases += [(f"persistent depth {d} grid {g}", lambda d=d, g=g: tune_lib.lib.dccl_tune_pipelined_f32_sum(ps, pr, n, d, g, st))
              for d, g in variants]
    t = {k: [] for k in range(len(cases))}
    for _ in range(a.rounds):
        for k, (_, fn) in enumerate(cases):
            t[k].append(time_launches([fn], rounds=1, min_ms=15.0)[0])
    rows = []
    for k, (name, _) in enumerate(cases):
        ms = statistics.median(t[k])
        rows.append({"variant": name, "ms": round(ms, 4), "frac": round(3 * nbytes / (ms * 1e-3) / 1e9 / PEAK, 4)})
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
