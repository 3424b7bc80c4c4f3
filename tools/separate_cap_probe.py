#!/usr/bin/env python3
"""Tuning only: the aligned pairwise combine's occupancy cap (DCCL_REDUCE_LDS_CAP, read once per process) on
separately allocated 1 GiB pairs (DCCL's scratchpad + user chunk shape) and on the pooled pair, one child
process per cap (each allocates its pairs afresh, so the pairs' placements differ between children; the
per-cap median over pairs is what compares).
    python tools/separate_cap_probe.py [--pairs 6] [--out f.json]
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
from tools.bench_suite import time_launches
pairs = int(sys.argv[2])
nbytes = 1 << 30; n = nbytes // 4
st = torch.cuda.current_stream().cuda_stream
out = {"separate": [], "pooled": None}
bufs = []
for j in range(pairs):
    s = torch.empty(nbytes, dtype=torch.uint8, device="cuda"); r = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dccl_amd.check(dccl_amd.synth_fill(s.data_ptr(), 7, n, 0, 0xDCC1, 2, st), "synth")
    dccl_amd.check(dccl_amd.synth_fill(r.data_ptr(), 7, n, 0, 0xDCC1, 1, st), "synth")
    bufs.append((s, r))
for s, r in bufs:
    ms = time_launches([lambda s=s, r=r: dccl_amd.local_reduce(s.data_ptr(), r.data_ptr(), 7, n, 0, st)], rounds=3, min_ms=20.0)[0]
    out["separate"].append(3 * nbytes / (ms * 1e-3) / 8e12)
del bufs
pool = torch.empty(2 * nbytes + 4096, dtype=torch.uint8, device="cuda")
b = pool.data_ptr()
dccl_amd.check(dccl_amd.synth_fill(b, 7, n, 0, 0xDCC1, 1, st), "synth")
dccl_amd.check(dccl_amd.synth_fill(b + nbytes + 4096, 7, n, 0, 0xDCC1, 2, st), "synth")
ms = time_launches([lambda: dccl_amd.local_reduce(b + nbytes + 4096, b, 7, n, 0, st)], rounds=3, min_ms=20.0)[0]
out["pooled"] = 3 * nbytes / (ms * 1e-3) / 8e12
print(json.dumps(out))
"""


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pairs", type=int, default=6)
    p.add_argument("--out", default="")
    a = p.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    caps = [0, 6400, 7680, 8192, 9216, 10240]  # 32 (uncapped), 25, 21, 20, 17, 16 waves per CU
    rows = []
    for c in caps + caps:  # two passes, so each cap sees two sets of placements
        env = {**os.environ, "DCCL_REDUCE_LDS_CAP": str(c)}
        r = subprocess.run([sys.executable, "-c", CHILD, root, str(a.pairs)], env=env, capture_output=True,
                           text=True, timeout=180)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        row = {"lds_cap": c, "separate": [round(x, 4) for x in d["separate"]],
               "separate_median": round(statistics.median(d["separate"]), 4), "pooled": round(d["pooled"], 4)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
