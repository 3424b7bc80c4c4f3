#!/usr/bin/env python3
"""Tuning only (round 3): the persistent work-queue combine (tools/tune/tune_kernels.hip, tune_wq_kernel) against
the shipped one-shot grid, fp32 Sum, 1 GiB per operand in bench.py's pooled layout (recv, then send 4 KiB past
its end).  Every configuration is first checked bit for bit against the shipped kernel on the same inputs (a
counter that lost coherence across the XCDs would combine some tiles twice or skip them), then timed in
interleaved rounds (HIP events around --launches launches, median).

    python tools/wq_probe.py [--rounds 3] [--out f.json]
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dccl_amd  # noqa: E402
from tools import tune_lib  # noqa: E402

PEAK = 8e12


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--launches", type=int, default=20)
    p.add_argument("--out", default="")
    a = p.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 1 << 30
    n = nbytes // 4
    pool = torch.empty(2 * nbytes + 4096, dtype=torch.uint8, device="cuda")
    recv, send = pool.data_ptr(), pool.data_ptr() + nbytes + 4096
    dccl_amd.check(dccl_amd.synth_fill(send, 7, n, 0, 0xDCC1, 0, st), "synth")
    dccl_amd.check(dccl_amd.synth_fill(recv, 7, n, 0, 0xDCC1, 1, st), "synth")
    ctr = torch.zeros(2, dtype=torch.int64, device="cuda")
    T = tune_lib.lib
    configs = [("shipped", None, None, lambda: dccl_amd.local_reduce(send, recv, 7, n, 0, st))]
    for grab in (1, 4, 8, 16, 32):
        for w in (8, 16, 24, 32):
            configs.append((f"wq_grab{grab}_w{w}", grab, w,
                            lambda g=grab, w=w: T.dccl_tune_wq_f32_sum(send, recv, n, g, w, ctr.data_ptr(), st)))
    for grab in (4, 8, 16):
        for w in (8, 16, 32):
            configs.append((f"wq_pipe_grab{grab}_w{w}", 100 + grab, w,
                            lambda g=grab, w=w: T.dccl_tune_wq_f32_sum(send, recv, n, 100 + g, w, ctr.data_ptr(), st)))
    # bit-exactness against the shipped kernel on the same 1 GiB inputs (recv restored from a saved copy)
    saved = pool[:nbytes].clone()
    rv = pool[:nbytes]
    assert configs[0][3]() == 0
    torch.cuda.synchronize()
    want = rv.clone()
    exact = {}
    for name, _, _, fn in configs[1:]:
        rv.copy_(saved)
        torch.cuda.synchronize()
        assert fn() == 0, name
        torch.cuda.synchronize()
        exact[name] = bool(torch.equal(rv, want)) and int(ctr[0]) == 0 and int(ctr[1]) == 0
        print(f"{name}: exact {exact[name]}", file=sys.stderr, flush=True)
    del want, saved
    torch.cuda.empty_cache()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = [[] for _ in configs]
    for _ in range(a.rounds):
        for i, (name, _, _, fn) in enumerate(configs):
            assert fn() == 0
            ev0.record()
            for _ in range(a.launches):
                fn()
            ev1.record()
            ev1.synchronize()
            times[i].append(ev0.elapsed_time(ev1) / a.launches)
    rows = []
    for (name, grab, w, _), ts in zip(configs, times):
        ms = statistics.median(ts)
        rows.append({"config": name, "grab": grab, "waves_per_cu": w, "ms": round(ms, 4),
                     "frac": round(3 * nbytes / (ms * 1e-3) / PEAK, 4), "bit_exact": exact.get(name, True)})
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"bytes_per_operand": nbytes, "rounds": a.rounds, "launches": a.launches, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
