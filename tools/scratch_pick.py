#!/usr/bin/env python3
"""Tuning only: can the library pick, per user buffer, a scratchpad that lands in the fast DRAM mode?
DCCL's ring-step shape (send = a scratch slot, recv = chunk (2j+1) of a separate 2 GiB user buffer, fp32 Sum)
for every (user buffer, candidate scratch) pair: the full-size eager rate at 512 and 128 MiB per operand, and a
short calibration proxy that leaves the user's bits unchanged (uint32 Sum of a zero scratch over a --probe-mib
slice, as a collective could run it on its own output buffer).  Reports the rate matrix, the proxy's choice per
user buffer and what picking by the proxy gains over the first candidate.

    python tools/scratch_pick.py [--users 3] [--cands 4] [--probe-mib 64] [--out f.json]
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--users", type=int, default=3)
    p.add_argument("--cands", type=int, default=4)
    p.add_argument("--probe-mib", type=int, default=64)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--out", default="")
    a = p.parse_args()
    dccl = bench._native()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    user_bytes = 2 << 30
    users, cands = [], []
    for u in range(a.users):
        t = torch.empty(user_bytes, dtype=torch.uint8, device=dev)
        bench.synth_into(t.view(torch.float32), user_bytes // 4, 7, 0, 40 + u)
        users.append(t)
    for c in range(a.cands):
        t = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
        bench.synth_into(t.view(torch.float32), (512 << 20) // 4, 7, 0, 60 + c)
        cands.append(t)

    def rate(ps, pr, nbytes, dt=7, launches=None):
        n = nbytes // 4
        k0 = time_pairs([(ps, pr)], n, dt, 3)
        launches = launches or int(min(400, max(10, 20.0 / max(k0, 1e-4))))
        ts = [time_pairs([(ps, pr)], n, dt, launches) for _ in range(a.rounds)]
        return 3 * nbytes / (statistics.median(ts) * 1e-3) / 1e9 / bench.HBM_PEAK_GBS

    def time_pairs(pairs, n, dt, launches):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for ps, pr in pairs[:1]:
            dccl.check(dccl.local_reduce(ps, pr, dt, n, 0, st.cuda_stream))
        ev0.record(st)
        for i in range(launches):
            ps, pr = pairs[i % len(pairs)]
            dccl.check(dccl.local_reduce(ps, pr, dt, n, 0, st.cuda_stream))
        ev1.record(st)
        ev1.synchronize()
        return ev0.elapsed_time(ev1) / launches

    res = {"users": a.users, "cands": a.cands, "probe_mib": a.probe_mib, "rows": []}
    for u, user in enumerate(users):
        row = {"user": u, "full_512": [], "full_128": [], "proxy": []}
        for c, cand in enumerate(cands):
            pr = user.data_ptr() + (512 << 20)  # chunk 1 of 4 (a 2 GiB all-reduce at W = 4)
            row["full_512"].append(round(rate(cand.data_ptr(), pr, 512 << 20), 4))
            row["full_128"].append(round(rate(cand.data_ptr(), pr + (128 << 20), 128 << 20), 4))
            # the proxy: the candidate's first probe-mib bytes against the chunk's first probe-mib bytes; a zero
            # scratch copy keeps the user's bits (uint32 Sum of 0)
            cand_zero = cand[: a.probe_mib << 20]
            saved = cand_zero.clone()
            cand_zero.zero_()
            row["proxy"].append(round(rate(cand_zero.data_ptr(), pr, a.probe_mib << 20, dt=3, launches=20), 4))
            cand_zero.copy_(saved)
            del saved
        best_proxy = max(range(a.cands), key=lambda c: row["proxy"][c])
        row["pick"] = best_proxy
        row["gain_512_vs_first"] = round(100 * (row["full_512"][best_proxy] - row["full_512"][0]), 2)
        row["gain_128_vs_first"] = round(100 * (row["full_128"][best_proxy] - row["full_128"][0]), 2)
        row["best_512"] = max(row["full_512"])
        res["rows"].append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
