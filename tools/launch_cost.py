#!/usr/bin/env python3
"""Tuning only: host issue cost per small combine launch by HIP entry point (tools/tune/launch_cost.hip):
hipLaunchKernel (the product), hipModuleLaunchKernel with a cached hipFunction_t, hipExtLaunchKernel.
fp32 Sum, 1 KiB / 64 KiB / 1 MiB per operand, n back-to-back launches, 7 interleaved rounds, median; also the
time until the stream drained, per launch.

    python tools/launch_cost.py [--n 2000] [--out f.json]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "tools", "lib", "liblaunch_cost.so")
MODES = {0: "hipLaunchKernel", 1: "hipModuleLaunchKernel(cached)", 2: "hipExtLaunchKernel"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=2000)
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--out", default="")
    a = p.parse_args()
    lib = ctypes.CDLL(LIB)
    lib.lc_run.restype = ctypes.c_double
    lib.lc_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                           ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
    st = torch.cuda.Stream()
    res = {"n": a.n, "rounds": a.rounds, "rows": []}
    for nbytes in (1 << 10, 64 << 10, 1 << 20):
        s = torch.ones(nbytes // 4, device="cuda")
        r = torch.zeros(nbytes // 4, device="cuda")
        issue = {m: [] for m in MODES}
        drain = {m: [] for m in MODES}
        for m in MODES:  # warm
            d = ctypes.c_double()
            assert lib.lc_run(m, 50, s.data_ptr(), r.data_ptr(), nbytes // 4, st.cuda_stream, ctypes.byref(d)) > 0
        for _ in range(a.rounds):
            for m in MODES:
                d = ctypes.c_double()
                t = lib.lc_run(m, a.n, s.data_ptr(), r.data_ptr(), nbytes // 4, st.cuda_stream, ctypes.byref(d))
                assert t > 0, (m, t)
                issue[m].append(t)
                drain[m].append(d.value)
        for m, name in MODES.items():
            row = {"bytes_per_operand": nbytes, "mode": name, "issue_us": round(statistics.median(issue[m]) * 1e6, 3),
                   "until_drained_us": round(statistics.median(drain[m]) * 1e6, 3)}
            res["rows"].append(row)
            print(row, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
