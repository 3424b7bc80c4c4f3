#!/usr/bin/env python3
"""Workload for rocprofv3 passes over the misaligned-recv combine (reduce_unaligned_kernel): fp32 Sum, 1 GiB per
operand, recv at byte offset --roff (default 1) and send at --soff, --launches launches; with --roff 0 the
aligned combine for comparison.  Run under `rocprofv3 --kernel-trace --stats` (durations of the boundary
pass and the vector pass) and `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` (traffic).
    rocprofv3 --kernel-trace --stats -d OUT -o m --output-format csv -- python3 tools/misaligned_probe.py
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--roff", type=int, default=1)
    p.add_argument("--soff", type=int, default=0)
    p.add_argument("--launches", type=int, default=5)
    p.add_argument("--variant", type=int, default=-1, help="a tools/tune misaligned-recv variant instead of the product")
    a = p.parse_args()
    nbytes = 1 << 30
    n = nbytes // 4 - 64
    st = torch.cuda.current_stream().cuda_stream
    pool = torch.empty(2 * nbytes + 4096, dtype=torch.uint8, device="cuda")
    base = pool.data_ptr()
    dccl_amd.check(dccl_amd.synth_fill(base, 7, nbytes // 4, 0, 0xDCC1, 1, st), "synth")
    dccl_amd.check(dccl_amd.synth_fill(base + nbytes + 4096, 7, nbytes // 4, 0, 0xDCC1, 2, st), "synth")
    for _ in range(a.launches):
        if a.variant >= 0:
            from tools import tune_lib
            dccl_amd.check(tune_lib.lib.dccl_tune_misaligned_f32_sum(base + nbytes + 4096 + a.soff, base + a.roff, n,
                                                                     a.variant, st), "tune")
        else:
            dccl_amd.check(dccl_amd.local_reduce(base + nbytes + 4096 + a.soff, base + a.roff, 7, n, 0, st), "combine")
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
