#!/usr/bin/env python3
"""Tuning only: the misaligned-recv tuning variants (tools/tune, dccl_tune_misaligned_f32_sum) give the product
kernel's result bit for bit, fp32 Sum, recv at byte offsets 1-3, send at --soffs byte offsets, sizes around a tile and across walks.
    python tools/misaligned_edge_check.py [--vars 25,30,31,32,33]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402
from tools import tune_lib  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--vars", default="25,30,31,32,33")
    p.add_argument("--soffs", default="0,1,4")
    a = p.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    bad = 0
    for n in (1, 63, 256, 1000, 4096 + 5, 65536 * 3 + 17, (1 << 22) + 3, (1 << 20) * 5 + 1):
        for roff in (1, 2, 3):
            for soff in (int(x) for x in a.soffs.split(",")):
                src = torch.randint(0, 256, (4 * n + 64,), dtype=torch.uint8, device="cuda")
                dst0 = torch.randint(0, 256, (4 * n + 64,), dtype=torch.uint8, device="cuda")
                ref = dst0.clone()
                dccl_amd.check(dccl_amd.local_reduce(src.data_ptr() + soff, ref.data_ptr() + roff, 7, n, 0, st))
                for v in (int(x) for x in a.vars.split(",")):
                    got = dst0.clone()
                    rc = tune_lib.lib.dccl_tune_misaligned_f32_sum(src.data_ptr() + soff, got.data_ptr() + roff, n, v, st)
                    assert rc == 0, (v, rc)
                    torch.cuda.synchronize()
                    if not torch.equal(got, ref):
                        bad += 1
                        print(f"MISMATCH variant {v} n {n} roff {roff} soff {soff}", flush=True)
    print("ok" if bad == 0 else f"{bad} mismatches", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
