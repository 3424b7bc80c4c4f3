#!/usr/bin/env python3
"""Fine occupancy sweep of the fp32-Sum combine (1 GiB, pooled operand layout): waves per CU capped
by unused dynamic LDS per block, for 64x1, 128x1 and 64x2 shapes.  Interleaved rounds, one process."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402
from tools import tune_lib  # noqa: E402


def main():
    n = (1 << 30) // 4
    pool = torch.empty(2 * n * 4 + 4096, dtype=torch.uint8, device="cuda")
    r = pool[: n * 4].view(torch.float32)
    s = pool[n * 4 + 4096:].view(torch.float32)
    r.uniform_(-1, 1)
    s.uniform_(-1, 1)
    st = torch.cuda.current_stream().cuda_stream
    info = tune_lib.tune_variants()
    idx = {(v["block"], v["unroll"], v["policy"], v["xcd"]): i for i, v in enumerate(info)}
    cases = {}
    for lds in (0, 6656, 6912, 7168, 7424, 7680, 7936, 8192):
        cases[(64, 1, lds)] = idx[(64, 1, 7, 0)]
    for lds in (12288, 13312, 14336, 15360, 16384):
        cases[(128, 1, lds)] = idx[(128, 1, 7, 0)]
    for lds in (10240, 12288, 14336, 16384):
        cases[(64, 2, lds)] = idx[(64, 2, 7, 0)]
    fn = lambda v, lds: tune_lib.lib.dccl_tune_reduce_f32_sum_lds(s.data_ptr(), r.data_ptr(), n, v, 0, lds, st)
    for (b, u, lds), v in cases.items():
        assert fn(v, lds) == 0
    torch.cuda.synchronize()
    times = {k: [] for k in cases}
    for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 15):
        for k, v in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn(v, k[2])
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / 20)
    rows = []
    for (b, u, lds), ts in times.items():
        med = statistics.median(ts)
        blocks = (160 << 10) // lds if lds else 2048 // b
        rows.append({"block": b, "unroll": u, "lds": lds, "blocks_per_cu": min(blocks, 2048 // b),
                     "waves_per_cu": min(blocks, 2048 // b) * b // 64, "ms": round(med, 4),
                     "frac": round(3 * n * 4 / (med * 1e-3) / 8e12, 4)})
    rows.sort(key=lambda x: x["ms"])
    for x in rows:
        print(json.dumps(x))
    if len(sys.argv) > 1:
        json.dump(rows, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
