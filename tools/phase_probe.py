#!/usr/bin/env python3
"""Operand-phase probe (tuning only): fp32 Sum over 1 GiB operands in bench.py's pooled layout, with
send and recv displaced from their 256-B aligned slots.

  shift  operands with different 16-B phases (DCCL's chunk k of a user buffer against the aligned
         scratchpad): the production path (dccl_local_reduce -> the shifted vector kernel) and the
         shifted kernel's tuning variants (cache policy, XCD-contiguous block order)
  line   same 16-B phase, different 128-B phase (every 1 KiB tile of one operand straddles 9 lines):
         the production vector kernel and vector-kernel variants (send loaded through the caches,
         XCD-contiguous order, so a straddled line can be served to the neighbouring tile)

Variants are timed interleaved, several rounds, median per variant.
    python tools/phase_probe.py [--mib 1024] [--rounds 5] [--out file.json]
"""
import argparse
import ctypes
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
    p.add_argument("--mib", type=int, default=1024)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--out", default="")
    a = p.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    nbytes = a.mib << 20
    n = nbytes // 4 - 64  # room for the displacements
    pool = torch.empty(2 * nbytes + 4096, dtype=torch.uint8, device="cuda")
    base = pool.data_ptr()
    for off, bid in ((0, 2), (nbytes + 4096, 1)):
        dccl_amd.check(dccl_amd.synth_fill(base + off, 7, nbytes // 4, 0, 0xDCC1, bid, st), "synth")
    recv0, send0 = base, base + nbytes + 4096

    cases = []
    pol, xcd = ctypes.c_int(), ctypes.c_int()
    for soff, roff in ((4, 0), (8, 0), (12, 0), (0, 4), (20, 8)):
        s, r = send0 + soff, recv0 + roff
        cases.append(("shift", soff, roff, "production", lambda s=s, r=r: dccl_amd.local_reduce(s, r, 7, n, 0, st)))
        for v in range(tune_lib.lib.dccl_tune_shift_num_variants()):
            tune_lib.lib.dccl_tune_shift_f32_sum(s, r, 0, v, ctypes.byref(pol), ctypes.byref(xcd), st)
            cases.append(("shift", soff, roff, f"policy {pol.value} xcd {xcd.value}",
                          lambda s=s, r=r, v=v: tune_lib.lib.dccl_tune_shift_f32_sum(s, r, n, v, None, None, st)))
    vec = dict(enumerate(tune_lib.tune_variants()))
    pick = [i for i, v in vec.items() if v["block"] == 64 and v["unroll"] == 1]
    for soff, roff in ((0, 0), (16, 0), (64, 0), (0, 16), (48, 16)):
        s, r = send0 + soff, recv0 + roff
        cases.append(("line", soff, roff, "production", lambda s=s, r=r: dccl_amd.local_reduce(s, r, 7, n, 0, st)))
        for i in pick:
            cases.append(("line", soff, roff, f"policy {vec[i]['policy']} xcd {vec[i]['xcd']}",
                          lambda s=s, r=r, i=i: tune_lib.lib.dccl_tune_reduce_f32_sum(s, r, n, i, 0, st)))
    times = {k: [] for k in range(len(cases))}
    for _ in range(a.rounds):
        for k, c in enumerate(cases):
            med, _ = time_launches([c[4]], rounds=1, min_ms=15.0)
            times[k].append(med)
    rows = []
    for k, (kind, soff, roff, what, _) in enumerate(cases):
        ms = statistics.median(times[k])
        gbs = 3 * n * 4 / (ms * 1e-3) / 1e9
        rows.append({"kind": kind, "send_offset": soff, "recv_offset": roff, "variant": what, "ms": round(ms, 4),
                     "gb_s": round(gbs, 1), "frac": round(gbs / PEAK, 4)})
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(0), "mib": a.mib, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
