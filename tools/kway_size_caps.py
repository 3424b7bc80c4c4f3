#!/usr/bin/env python3
"""Tuning only: do the k-way / chain wave caps (kMultiWaves / kChainWaves, tuned at 1 GiB per operand) also
suit the chunk sizes DCCL's direct collectives combine (count / W per rank: tens of MiB)?  For each size and
k, the in-phase k-way (tune_multi variant 0) and chain (policy 7, in place) kernels under the shipped cap, no
cap and a middle cap, fp32 Sum, sources and recv in one staggered pool; below 1 GiB the launches rotate over
operand sets at different offsets so the Infinity Cache does not hold them.  Median of interleaved rounds,
fraction of (k+2)*N*4 B at 8 TB/s.
    python tools/kway_size_caps.py [--sizes 16,32,64,128,256,1024] [--ks 2,4,7] [--caps 16,32] [--rounds 5] [--out f.json]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

os.environ.setdefault("DCCL_TUNE_ALIGN", "128")
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402
from tools import tune_lib  # noqa: E402

MULTI_WAVES = [32, 32, 18, 13, 13, 11, 11, 10, 9]  # kMultiWaves, dccl_amd/csrc/reduce_kernels.hpp
CHAIN_WAVES = [32, 32, 24, 20, 16, 13, 11, 10, 9]  # kChainWaves
STRADDLE_WAVES = [32, 32, 18, 13, 13, 11, 9, 9, 7]  # kStraddleWaves
PHASED_FIRST = [0, 0, 0, 0, 0, 13, 0, 12, 11]  # kPhasedFirstWaves (0: per-operand form, uncapped)
CHAIN_PHASED_FIRST = [0, 0, 0, 0, 13, 13, 0, 11, 11]  # kChainPhasedFirstWaves
CHAIN_STRADDLE_WAVES = [32, 32, 24, 18, 13, 13, 11, 10, 9]  # kChainStraddleWaves


def lds_of(w: int) -> int:
    return 0 if w >= 32 else ((160 << 10) // w + 255) // 256 * 256


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--sizes", default="16,32,64,128,256,1024", help="MiB per operand")
    p.add_argument("--ks", default="2,4,7")
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--caps", default="16,32", help="wave caps timed beside the shipped one")
    p.add_argument("--product", action="store_true", help="also time the product entry points (their own caps)")
    p.add_argument("--phased", action="store_true",
                   help="sources 4 B off the destination's 16-B phase (the phased launches: the loads-first form under "
                        "caps for k in kPhasedFirstWaves / kChainPhasedFirstWaves, else the per-operand form)")
    p.add_argument("--straddle", action="store_true",
                   help="sources 16 (2j+1) B off recv's 128-B lines (the line-straddling launches: tune_multi variant 8, "
                        "chain policy 6, caps kStraddleWaves / kChainStraddleWaves)")
    p.add_argument("--out", default="")
    a = p.parse_args()
    global MULTI_WAVES, CHAIN_WAVES
    soff = (lambda j: 16 * (2 * j + 1)) if a.straddle else (lambda j: 4) if a.phased else (lambda j: 0)
    variant, policy = (8, 6) if a.straddle else (0, 7)
    if a.straddle:
        MULTI_WAVES, CHAIN_WAVES = STRADDLE_WAVES, CHAIN_STRADDLE_WAVES
    if a.phased:
        MULTI_WAVES = [w or 32 for w in PHASED_FIRST]
        CHAIN_WAVES = [w or 32 for w in CHAIN_PHASED_FIRST]
    prod = tune_lib.lib.dccl_tune_phased_prod_f32_sum
    st = torch.cuda.current_stream().cuda_stream
    gib = 1 << 30
    kmax = max(int(x) for x in a.ks.split(","))
    pool = torch.empty((kmax + 1) * (gib + 4096) + 4096, dtype=torch.uint8, device="cuda")
    base = [pool.data_ptr() + j * (gib + 4096) for j in range(kmax + 1)]  # base[0] = recv / own
    for j, b in enumerate(base):
        dccl_amd.check(dccl_amd.synth_fill(b, 7, gib // 4, 0, 0xDCC1, 40 + j, st), "synth")
    multi, chain = tune_lib.lib.dccl_tune_multi_f32_sum, tune_lib.lib.dccl_tune_chain_policy_f32_sum
    rows = []
    for mib in (int(x) for x in a.sizes.split(",")):
        nb = mib << 20
        n = nb // 4
        sets = max(1, min(8, gib // nb))
        for k in (int(x) for x in a.ks.split(",")):
            arrs = [(ctypes.c_void_p * k)(*[base[1 + j] + s * nb + soff(j) for j in range(k)]) for s in range(sets)]
            lists = [[base[1 + j] + s * nb + soff(j) for j in range(k)] for s in range(sets)]
            dsts = [base[0] + s * nb for s in range(sets)]
            configs = []
            for what, shipped in (("multi", MULTI_WAVES[k]), ("chain", CHAIN_WAVES[k])):  # noqa: F821
                for w in sorted({shipped, *(int(x) for x in a.caps.split(","))}):
                    configs.append((what, w))
                if a.product:
                    configs.append((what, "product"))  # dccl_local_reduce_multi / _chain: the shipped choice
            t = {c: [] for c in configs}
            for _ in range(a.rounds):
                for what, w in configs:
                    lds = lds_of(w) if w != "product" else None
                    launches = max(10, min(400, int(0.02 / ((k + 2) * nb / 6.5e12))))
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for i in range(launches):
                        s = i % sets
                        if lds is None:
                            rc = (dccl_amd.local_reduce_multi(lists[s], dsts[s], 7, n, 0, st) if what == "multi" else
                                  dccl_amd.local_reduce_chain(lists[s], dsts[s], dsts[s], 7, n, 0, st))
                        elif a.phased:
                            first = int((PHASED_FIRST if what == "multi" else CHAIN_PHASED_FIRST)[k] != 0)
                            rc = prod(arrs[s], k, None if what == "multi" else dsts[s], dsts[s], n, first,
                                      int(not first and k <= 4), lds, st)
                        elif what == "multi":
                            rc = multi(arrs[s], k, dsts[s], n, variant, lds, st)
                        else:
                            rc = chain(arrs[s], k, dsts[s], dsts[s], n, lds, policy, st)
                        assert rc == 0, (what, k, w, rc)
                    e1.record()
                    e1.synchronize()
                    t[(what, w)].append(e0.elapsed_time(e1) / launches)
            for what, w in configs:
                ms = statistics.median(t[(what, w)])
                shipped = (MULTI_WAVES if what == "multi" else CHAIN_WAVES)[k]
                rows.append({"mib": mib, "k": k, "what": what, "waves": w, "shipped_1gib_cap": w == shipped, "sets": sets,
                             "us": round(ms * 1e3, 2), "frac": round((k + 2) * nb / (ms * 1e-3) / 1e9 / 8000.0, 4)})
                print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
