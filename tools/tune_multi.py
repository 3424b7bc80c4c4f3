"""A/B the k-way combine (dccl_local_reduce_multi) shapes on MI355X.

For k = 1..8 sends of --mib MiB fp32 and two operand placements (separate allocations; one pool
with a 4 KiB x (j+1) stagger between operand j and j+1), times each variant of
dccl_tune_multi_f32_sum (tools/tune/dccl_reduce_tuning.h) and the shipped entry point.
Algorithmic bytes per launch: (k + 2) * operand bytes.  Use 1 GiB operands (--mib 1024) for decisions:
at 256 MiB a recv buffer written with the default cache policy partly survives in the 256 MiB
Infinity Cache between back-to-back launches, which flatters variants 3 (profiles/r1_tune_multi_*.json).

    python tools/tune_multi.py [--mib 1024] [--out gpurun_out/tune_multi.json]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402
from tools import tune_lib  # noqa: E402

PEAK = 8.0e12
VARIANTS = {0: "64x1 nt-all (shipped)", 1: "64x2 nt-all", 2: "256x1 nt-all", 3: "64x1 nt-send", 4: "64x4 nt-all",
            5: "staged: recv+s0, then 1 send at a time", 6: "staged: recv+s0, then 2 at a time",
            7: "staged: recv+s0, then 3 at a time"}
LDS_PER_CU = 160 << 10
WAVES = [32, 24, 20, 16, 13, 11, 9, 7, 5]  # one-wave blocks resident per CU, set through unused LDS


def lds_for(waves: int) -> int:
    return 0 if waves >= 32 else -(-LDS_PER_CU // waves // 256) * 256


def operands(k, nbytes, layout):
    if layout == "separate":
        bufs = [torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(k + 1)]
        return bufs, [b.data_ptr() for b in bufs]
    gap = 4096
    pool = torch.empty((k + 1) * nbytes + gap * (k + 1) * (k + 2) // 2, dtype=torch.uint8, device="cuda")
    ptrs, off = [], 0
    for j in range(k + 1):
        ptrs.append(pool.data_ptr() + off)
        off += nbytes + gap * (j + 1)
    return [pool], ptrs


def median_ms(fn, reps=30):
    st = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn()
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mib", type=int, default=1024)
    p.add_argument("--out", default="gpurun_out/tune_multi.json")
    p.add_argument("--ks", default="1,2,3,4,5,6,7,8")
    p.add_argument("--no-waves", action="store_true", help="skip the occupancy-cap sweep of variant 0")
    a = p.parse_args()
    nbytes = a.mib << 20
    n = nbytes // 4
    st = torch.cuda.current_stream().cuda_stream
    rows = []
    for layout in ("separate", "staggered"):
        for k in [int(x) for x in a.ks.split(",")]:
            keep, ptrs = operands(k, nbytes, layout)
            for j, q in enumerate(ptrs):
                dccl_amd.check(dccl_amd.synth_fill(q, 7, n, 0, 0xDCC1, j, st))
            recv, sends = ptrs[0], ptrs[1:]
            arr = (ctypes.c_void_p * k)(*sends)
            row = {"layout": layout, "k": k, "bytes_per_launch": (k + 2) * nbytes}
            ms = median_ms(lambda: dccl_amd.local_reduce_multi(sends, recv, 7, n, 0, st))
            row["shipped_ms"] = round(ms, 4)
            row["shipped_frac"] = round((k + 2) * nbytes / (ms * 1e-3) / PEAK, 4)
            for v in VARIANTS:
                ms = median_ms(lambda: tune_lib.lib.dccl_tune_multi_f32_sum(arr, k, recv, n, v, 0, st))
                row[f"v{v}_ms"] = round(ms, 4)
                row[f"v{v}_frac"] = round((k + 2) * nbytes / (ms * 1e-3) / PEAK, 4)
            for w in ([] if a.no_waves else WAVES):
                ms = median_ms(lambda: tune_lib.lib.dccl_tune_multi_f32_sum(arr, k, recv, n, 0, lds_for(w), st))
                row[f"w{w}_frac"] = round((k + 2) * nbytes / (ms * 1e-3) / PEAK, 4)
            rows.append(row)
            print(json.dumps(row), flush=True)
            del keep
            torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"device": torch.cuda.get_device_name(), "variants": VARIANTS,
                   "waves": {w: lds_for(w) for w in WAVES}, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
