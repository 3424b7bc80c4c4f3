#!/usr/bin/env python3
"""Tuning only: the pairwise combine's occupancy cap (DCCL_REDUCE_LDS_CAP, read once per process) for the
aligned and the line-straddling (send 16 B off its lines) cases, 1 GiB fp32 Sum, pooled layout; one child
process per cap, interleaved over --rounds.
    python tools/pairwise_cap_probe.py [--rounds 3] [--out f.json]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

CHILD = r"""
import json, sys, torch
sys.path.insert(0, sys.argv[1])
import dccl_amd
from tools.bench_suite import PEAK, time_launches
nbytes = 1 << 30; n = nbytes // 4 - 64
st = torch.cuda.current_stream().cuda_stream
pool = torch.empty(2 * nbytes + 4096, dtype=torch.uint8, device="cuda")
base = pool.data_ptr()
for off, bid in ((0, 2), (nbytes + 4096, 1)):
    dccl_amd.check(dccl_amd.synth_fill(base + off, 7, nbytes // 4, 0, 0xDCC1, bid, st), "synth")
out = {}
for name, soff in (("aligned", 0), ("send off its lines", 16), ("send 16-B phase +4", 4)):
    ms = time_launches([lambda s=soff: dccl_amd.local_reduce(base + nbytes + 4096 + s, base, 7, n, 0, st)],
                       rounds=3, min_ms=20.0)
    out[name] = ms[0]
print(json.dumps(out))
"""


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--out", default="")
    a = p.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    caps = [0, 5120, 6144, 7168, 8192]  # bytes of dynamic LDS per one-wave block: 32, 32, 26, 22, 20 waves
    res = {c: [] for c in caps}
    for _ in range(a.rounds):
        for c in caps:
            env = {**os.environ, "DCCL_REDUCE_LDS_CAP": str(c)}
            r = subprocess.run([sys.executable, "-c", CHILD, root], env=env, capture_output=True, text=True,
                               timeout=120)
            res[c].append(json.loads(r.stdout.strip().splitlines()[-1]))
    rows = []
    for c in caps:
        row = {"lds_cap": c}
        for name in res[c][0]:
            ms = statistics.median(x[name] for x in res[c])
            row[name] = round(3 * (2 ** 30 - 256) / (ms * 1e-3) / 8e12, 4)
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
