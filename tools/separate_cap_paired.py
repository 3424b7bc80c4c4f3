#!/usr/bin/env python3
"""Paired occupancy-cap probe of the aligned pairwise combine (tuning only, MI355X).

tools/separate_cap_probe.py compares caps across child processes, so every cap sees other placements.  Here
the SAME operand pairs are timed under every cap, interleaved in one process: `--pairs` separately allocated
`--mib` pairs (default 1 GiB; DCCL's scratchpad + user chunk shape) and the bench's pooled pair (one allocation, send 4 KiB
past recv).  The shipped kernel shape runs through the tuning entry with an explicit dynamic-LDS size per
one-wave block (160 KiB / lds resident waves per CU).  Per pair and cap: median kernel time and fraction of
the 8 TB/s HBM peak; per cap: the change against uncapped for every pair.  Column `product`: the
shipped entry point dccl_local_reduce on the same pairs (its own cap choice, local_reduce.hip).

    python tools/separate_cap_paired.py [--kind aligned|straddle|shift] [--pairs 8] [--mib 1024] [--rounds 5] [--iters 10] [--out f.json]
"""
import argparse
import json
import os
import statistics
import sys

os.environ.setdefault("DCCL_TUNE_ALIGN", "128")
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402
from tools import tune_lib  # noqa: E402

CAPS = {32: 0, 27: 5888, 26: 6144, 25: 6400, 24: 6656, 22: 7168, 21: 7680, 20: 8192}  # waves per CU -> LDS bytes per block
if os.environ.get("DCCL_PAIRED_CAPS") == "fine":  # 28-30 waves
    CAPS = {32: 0, 30: 5376, 29: 5632, 28: 5760}  # nominal: LDS allocation granularity may merge some


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pairs", type=int, default=8)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--out", default="")
    p.add_argument("--mib", type=int, default=1024, help="bytes per operand, MiB")
    p.add_argument("--kind", default="aligned", choices=["aligned", "straddle", "shift", "shift_straddle", "group"],
                   help="aligned: send and recv on equal 128-B phases (DefaultCfg); straddle: send 16 B further "
                        "(StraddleCfg, send loads cached); shift: send 4 B further (the shifted kernel); shift_straddle: "
                        "send 20 B further (the shifted kernel with cached send loads); group: aligned, the shipped shape in "
                        "the group-interleaved XCD tile order (dccl_tune_group_f32_sum)")
    a = p.parse_args()
    nb = a.mib << 20
    soff = {"aligned": 0, "straddle": 16, "shift": 4, "shift_straddle": 20, "group": 0}[a.kind]
    n = nb // 4 - (16 if soff else 0)
    st = torch.cuda.current_stream().cuda_stream
    pairs, keep = [], []
    for j in range(a.pairs):
        s = torch.empty(nb, dtype=torch.uint8, device="cuda")
        r = torch.empty(nb, dtype=torch.uint8, device="cuda")
        keep += [s, r]
        pairs.append((f"separate{j}", s.data_ptr(), r.data_ptr()))
    pool = torch.empty(2 * nb + 4096, dtype=torch.uint8, device="cuda")
    keep.append(pool)
    pairs.append(("pooled", pool.data_ptr() + nb + 4096, pool.data_ptr()))
    for _, ps, pr in pairs:
        dccl_amd.check(dccl_amd.synth_fill(ps, 7, n, 0, 0xDCC1, 2, st), "synth")
        dccl_amd.check(dccl_amd.synth_fill(pr, 7, n, 0, 0xDCC1, 1, st), "synth")
    tune = tune_lib.lib.dccl_tune_reduce_f32_sum_lds
    straddle_variant = next(v for v, inf in enumerate(tune_lib.tune_variants())
                            if (inf["block"], inf["unroll"], inf["policy"], inf["xcd"]) == (64, 1, 6, 0))

    def fn(ps, pr, n, v, cap, lds, st):  # lds None: the product entry point, which picks its own cap
        ps += soff
        if lds is None:
            return dccl_amd.local_reduce(ps, pr, 7, n, 0, st)
        if a.kind == "group":
            return tune_lib.lib.dccl_tune_group_f32_sum(ps, pr, n, lds, st)
        if a.kind.startswith("shift"):
            return tune_lib.lib.dccl_tune_shift_caps_f32_sum(ps, pr, n, lds, st)
        return tune(ps, pr, n, straddle_variant if a.kind == "straddle" else v, cap, lds, st)

    caps = {**CAPS, "product": None}
    times = {(name, w): [] for name, _, _ in pairs for w in caps}
    for _, ps, pr in pairs:
        for lds in caps.values():
            assert fn(ps, pr, n, 0, 0, lds, st) == 0
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for name, ps, pr in pairs:
            for w, lds in caps.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn(ps, pr, n, 0, 0, lds, st)
                e1.record()
                e1.synchronize()
                times[(name, w)].append(e0.elapsed_time(e1) / a.iters)
    frac = {k: 3 * n * 4 / (statistics.median(v) * 1e-3) / 1e9 / 8000.0 for k, v in times.items()}
    out = {"mib": a.mib, "kind": a.kind, "pairs": {}, "by_cap": {}}
    for name, _, _ in pairs:
        out["pairs"][name] = {str(w): round(frac[(name, w)], 4) for w in caps}
    seps = [name for name, _, _ in pairs if name != "pooled"]
    for w in caps:
        d = [frac[(nm, w)] - frac[(nm, 32)] for nm in seps]
        out["by_cap"][str(w)] = {"separate_median": round(statistics.median(frac[(nm, w)] for nm in seps), 4),
                                 "separate_min": round(min(frac[(nm, w)] for nm in seps), 4),
                                 "delta_median": round(statistics.median(d), 4), "delta_min": round(min(d), 4),
                                 "delta_max": round(max(d), 4), "pooled": round(frac[("pooled", w)], 4)}
    txt = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)
    print(txt, flush=True)


if __name__ == "__main__":
    main()
