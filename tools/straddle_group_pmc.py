#!/usr/bin/env python3
"""Workload for rocprofv3 --pmc FETCH_SIZE over the line-straddling k-way shapes (tuning only): k sources
16 (2j+1) B off recv's 128-B lines, 1 GiB fp32 Sum per operand; tune_multi variants 8 (shipped: sources cached,
block order) and 15 / 16 (group-interleaved XCD order, sources cached / non-temporal), --launches each, under
the given wave caps.  Does the group order fetch the line two neighbouring tiles share once?
    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT -o p -- python3 tools/straddle_group_pmc.py
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402
from tools import tune_lib  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=8)
    p.add_argument("--launches", type=int, default=3)
    p.add_argument("--configs", default="8:7,15:9,16:9", help="variant:waves list")
    a = p.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 1 << 30
    n = nbytes // 4 - 64
    recv = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    srcs = torch.empty(a.k * (nbytes + 4096) + 256, dtype=torch.uint8, device="cuda")
    sp = [srcs.data_ptr() + j * (nbytes + 4096) + 16 * (2 * j + 1) for j in range(a.k)]
    for j, q in enumerate(sp):
        dccl_amd.check(dccl_amd.synth_fill(q, 7, n, 0, 0xDCC1, 10 + j, st), "synth")
    arr = (ctypes.c_void_p * a.k)(*sp)
    for cfg in a.configs.split(","):
        v, w = (int(x) for x in cfg.split(":"))
        lds = 0 if w >= 32 else ((160 << 10) // w + 255) // 256 * 256
        for _ in range(a.launches):
            dccl_amd.check(tune_lib.lib.dccl_tune_multi_f32_sum(arr, a.k, recv.data_ptr(), n, v, lds, st), "multi")
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
