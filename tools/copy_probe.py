"""dccl_copy_multi on one MI355X: 8 pairs of 128 MiB local copies, dst aligned, src at 16-B phase 0
(plain vector loads) or off it (cross-lane funnel shift), HIP-event timed; GB/s on 2 x bytes x pairs.
    python tools/copy_probe.py [--out file.json]"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    nbytes, npairs = 128 << 20, 8
    srcs = [torch.randint(0, 255, (nbytes + 64,), dtype=torch.uint8, device="cuda") for _ in range(npairs)]
    dsts = [torch.zeros(nbytes + 64, dtype=torch.uint8, device="cuda") for _ in range(npairs)]
    st = torch.cuda.current_stream()
    rows = []
    for soff in (0, 16, 4, 1, 9):
        sp = [s.data_ptr() + soff for s in srcs]
        dp = [d.data_ptr() for d in dsts]
        fn = lambda: dccl_amd.check(dccl_amd.copy_multi(sp, dp, nbytes, st.cuda_stream), "copy_multi")
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        res = []
        for _ in range(5):
            e0.record(st)
            for _ in range(10):
                fn()
            e1.record(st)
            e1.synchronize()
            res.append(e0.elapsed_time(e1) / 10)
        ms = statistics.median(res)
        ok = all(torch.equal(d[:nbytes], s[soff:soff + nbytes]) for s, d in zip(srcs, dsts))
        gbs = 2 * nbytes * npairs / (ms * 1e-3) / 1e9
        rows.append({"src_offset": soff, "ms": round(ms, 4), "gb_s": round(gbs, 1), "frac": round(gbs / PEAK, 4),
                     "bit_exact": ok})
        print("copy_multi", rows[-1], flush=True)
    # the previous fallback for differing 16-B phases: the runtime's copy, pair after pair
    for soff in (4,):
        fn = lambda: [d[:nbytes].copy_(s[soff:soff + nbytes]) for s, d in zip(srcs, dsts)]
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        res = []
        for _ in range(5):
            e0.record(st)
            for _ in range(10):
                fn()
            e1.record(st)
            e1.synchronize()
            res.append(e0.elapsed_time(e1) / 10)
        ms = statistics.median(res)
        gbs = 2 * nbytes * npairs / (ms * 1e-3) / 1e9
        rows.append({"src_offset": soff, "path": "runtime copy per pair (previous fallback)", "ms": round(ms, 4),
                     "gb_s": round(gbs, 1), "frac": round(gbs / PEAK, 4)})
        print("runtime copy", rows[-1], flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"bytes_per_pair": nbytes, "pairs": npairs, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
