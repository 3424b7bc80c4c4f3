#!/usr/bin/env python3
"""A/B the fp32-Sum combine kernel variants in ONE process, interleaved rounds (MI355X).

Variants (tools/tune/dccl_reduce_tuning.h):
  * template variants: block threads x UNROLL x cache policy (nt send / nt recv / nt store)
    x XCD-contiguous remap, one block per tile or a persistent grid;
  * asm flavours: one-wave blocks with explicit sc0/sc1/nt bits on loads and stores;
  * placement: the best template variant with `send` placed at several byte offsets from
    `recv` inside one allocation (HBM channel/bank sensitivity to the operands' distance).
Prints a JSON table of median / min kernel times and achieved HBM GB/s (3N bytes).

    python tools/tune_reduce.py [--mib 1024] [--rounds 7] [--iters 10] [--out file]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402
from tools import tune_lib  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mib", type=int, default=1024)
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--out", default="")
    p.add_argument("--lds-kib", type=float, default=0.0)
    p.add_argument("--only", default="", help="comma list of kinds to run: template,occupancy,asm,placement")
    a = p.parse_args()
    n = (a.mib << 20) // 4
    s = torch.rand(n, device="cuda")
    r = torch.rand(n, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    info = tune_lib.tune_variants()

    # placement experiment: one allocation, send at recv + n*4 + delta
    big = torch.empty(2 * n + (8 << 20) // 4, device="cuda")
    deltas = [0, 4096, 65536, (1 << 20) + 4096, 3 << 20]

    cases = {}
    for v, inf in enumerate(info):
        cases[("tpl", v, 0)] = (lambda v=v: tune_lib.lib.dccl_tune_reduce_f32_sum(s.data_ptr(), r.data_ptr(), n, v, 0, st),
                                {**inf, "kind": "template", "grid_cap": 0})
        if inf["block"] == 256 and inf["unroll"] == 4 and inf["policy"] == 7:
            for k in (4, 16):
                cap = cus * k
                cases[("tpl", v, cap)] = (
                    lambda v=v, cap=cap: tune_lib.lib.dccl_tune_reduce_f32_sum(s.data_ptr(), r.data_ptr(), n, v, cap, st),
                    {**inf, "kind": "template", "grid_cap": cap})
    for lds in [int(a.lds_kib * 1024)] if a.lds_kib else (5 << 10, 6 << 10, 7 << 10, 8 << 10, 9 << 10, 10 << 10, 20 << 10):
        cases[("lds", lds)] = (
            lambda lds=lds: tune_lib.lib.dccl_tune_reduce_f32_sum_lds(s.data_ptr(), r.data_ptr(), n, 0, 0, lds, st),
            {"kind": "occupancy", "variant": info[0], "lds_bytes": lds, "max_waves_per_cu": (160 << 10) // lds})
    for waves, skew in ((8, 0), (8, 1), (8, 2), (8, 4), (4, 0), (4, 2), (16, 8), (16, 4)):
        cases[("skew", waves, skew)] = (
            lambda waves=waves, skew=skew: tune_lib.lib.dccl_tune_skew_f32_sum(s.data_ptr(), r.data_ptr(), n, waves, skew, st),
            {"kind": "skew", "waves": waves, "skew_kib": skew})
    for fl in range(7):
        cases[("asm", fl)] = (lambda fl=fl: tune_lib.lib.dccl_tune_asm_f32_sum(s.data_ptr(), r.data_ptr(), n, fl, st),
                              {"kind": "asm", "flavor": fl})
    for d in deltas:
        rp = big.data_ptr()
        sp = rp + n * 4 + d
        cases[("place", d)] = (lambda sp=sp, rp=rp: tune_lib.lib.dccl_tune_reduce_f32_sum(sp, rp, n, 0, 0, st),
                               {"kind": "placement", "variant": info[0], "send_minus_recv_end": d})
    if a.only:
        keep = set(a.only.split(","))
        cases = {k: v for k, v in cases.items() if v[1]["kind"] in keep or (k[0] == "tpl" and k[1] == 0)}
    for k, (fn, _) in cases.items():
        assert fn() == 0, k
    torch.cuda.synchronize()
    times = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, (fn, _) in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / a.iters)
    rows = []
    for k, ts in times.items():
        med = statistics.median(ts)
        rows.append({**cases[k][1], "ms_median": round(med, 4), "ms_min": round(min(ts), 4),
                     "gb_s": round(3 * n * 4 / (med * 1e-3) / 1e9, 1)})
    rows.sort(key=lambda x: x["ms_median"])
    out = {"mib": a.mib, "cus": cus, "rows": rows}
    txt = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)
    for row in rows:
        try:
            print(json.dumps(row))
        except BrokenPipeError:
            break


if __name__ == "__main__":
    main()
