#!/usr/bin/env python3
"""Tuning only: can the operand DCCL owns (the scratchpad = send) be placed so that a separately
allocated pair runs in the fast mode?  --pairs separately allocated 1 GiB recv buffers and send buffers
of 1 GiB + 2 MiB; for each pair the shipped fp32 Sum combine is timed with send at several byte offsets
into its allocation (interleaved over --rounds, median), and with recv/send swapped roles.  Prints the
fraction of HBM peak per pair and offset, then every recv buffer against every send buffer.
    python tools/pair_offset_probe.py [--pairs 8] [--rounds 3] [--out f.json]
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
OFFSETS = [0, 4096, 8192, 12288, 65536, 1 << 20, (1 << 20) + 4096]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pairs", type=int, default=8)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--out", default="")
    a = p.parse_args()
    nbytes = 1 << 30
    n = nbytes // 4
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    recvs = [torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(a.pairs)]
    sends = [torch.empty(nbytes + (2 << 20), dtype=torch.uint8, device="cuda") for _ in range(a.pairs)]
    for j in range(a.pairs):
        dccl_amd.check(dccl_amd.synth_fill(recvs[j].data_ptr(), 7, n, 0, 0xDCC1, 1, sh), "synth")
        dccl_amd.check(dccl_amd.synth_fill(sends[j].data_ptr(), 7, (nbytes + (2 << 20)) // 4, 0, 0xDCC1, 2, sh), "synth")
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

    rows = []
    for j in range(a.pairs):
        pr = recvs[j].data_ptr()
        t = {o: [] for o in OFFSETS}
        for _ in range(a.rounds):
            for o in OFFSETS:
                t[o].append(t_of(sends[j].data_ptr() + o, pr))
        row = {"pair": j, "recv_mod_2m": pr % (2 << 20), "send_mod_2m": sends[j].data_ptr() % (2 << 20),
               "frac_by_send_offset": {str(o): round(3 * nbytes / (statistics.median(t[o]) * 1e-3) / PEAK, 4)
                                       for o in OFFSETS}}
        rows.append(row)
        print(json.dumps(row), flush=True)
    # every recv buffer against every send buffer (offset 0): is the slow mode a property of a pair, or of
    # one buffer's pages?
    mat = [[[] for _ in range(a.pairs)] for _ in range(a.pairs)]
    for _ in range(a.rounds):
        for i in range(a.pairs):
            for j in range(a.pairs):
                mat[i][j].append(t_of(sends[j].data_ptr(), recvs[i].data_ptr()))
    cross = [[round(3 * nbytes / (statistics.median(mat[i][j]) * 1e-3) / PEAK, 4) for j in range(a.pairs)]
             for i in range(a.pairs)]
    for i in range(a.pairs):
        print("recv", i, " ".join(f"{x:.3f}" for x in cross[i]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"pairs": rows, "cross_recv_by_send": cross}, f, indent=1)


if __name__ == "__main__":
    main()
