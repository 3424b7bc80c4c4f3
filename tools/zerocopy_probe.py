#!/usr/bin/env python3
"""Zero-copy probe (tuning only): the fp32 Sum combine on page-locked HOST operands read and written by
the GPU over PCIe (the host-staged path's kernel), for every vector-kernel tuning variant
(block size, vectors per lane, cache policy).  Payload GiB/s = bytes per operand / time; the link
carries 2 operands host->device and 1 device->host per combine.
    python tools/zerocopy_probe.py [--mib 256] [--rounds 5] [--out f.json]
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
from tools.bench_suite import time_launches  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mib", type=int, default=256)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--out", default="")
    a = p.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    nbytes = a.mib << 20
    n = nbytes // 4
    s = torch.empty(n, dtype=torch.float32).uniform_(-1, 1).pin_memory()
    r = torch.zeros(n, dtype=torch.float32).pin_memory()
    ps, pr = s.data_ptr(), r.data_ptr()  # ROCm maps page-locked memory at the same address on the device
    cases = [("production", lambda: dccl_amd.local_reduce(ps, pr, 7, n, 0, st))]
    for i, v in enumerate(tune_lib.tune_variants()):
        cases.append((f"{v['block']}x{v['unroll']} policy {v['policy']} xcd {v['xcd']}",
                      lambda i=i: tune_lib.lib.dccl_tune_reduce_f32_sum(ps, pr, n, i, 0, st)))
    times = {k: [] for k in range(len(cases))}
    for _ in range(a.rounds):
        for k, (_, fn) in enumerate(cases):
            times[k].append(time_launches([fn], rounds=1, min_ms=30.0)[0])
    rows = []
    for k, (name, _) in enumerate(cases):
        ms = statistics.median(times[k])
        rows.append({"variant": name, "ms": round(ms, 3), "payload_gib_s": round(nbytes / (ms * 1e-3) / 2**30, 2),
                     "h2d_gb_s": round(2 * nbytes / (ms * 1e-3) / 1e9, 1)})
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"mib": a.mib, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
