#!/usr/bin/env python3
"""Tuning only: the phased k-way combine's shape variants (tools/tune/tune_kernels.hip,
dccl_tune_phased_f32_sum) at 1 GiB per operand, fp32 Sum, k = 2-5 and 7 sources at a 16-B phase of +4 B
(and +12 B for k = 2; k = 2 again at the end, after the other allocations); then the phased chain
kernel (in place, own = recv) for k = 1-5, 7 with the XCD tile order off and on. against a 128-B aligned recv, interleaved over --rounds; HBM fraction of (k+2)N.
    python tools/phased_probe.py [--rounds 5] [--out f.json]
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
from tools.bench_suite import PEAK, time_launches  # noqa: E402

VARIANTS = (0, 1, 32, 64)  # the lane-exchange forms; 2-3 (unaligned loads) lost 3-8 points at every k (round 2)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--straddle", action="store_true",
                   help="in-phase sources off recv's 128-B lines: tune_multi variants 0, 8, 9, 10 under the k-way caps")
    p.add_argument("--swap", action="store_true",
                   help="sources sharing one phase: tiles on the sources' 16-B grid (recv accessed unaligned)")
    p.add_argument("--prod-caps", action="store_true",
                   help="the shipped phased k-way and chain kernels: shipped form vs loads-first under wave caps")
    p.add_argument("--straddle-caps", action="store_true",
                   help="line-straddling sources, k = 5-8: wave-cap sweep of the shipped straddle shape (variant 8)")
    p.add_argument("--common-phase", action="store_true", help="--straddle: every source at the same line offset")
    p.add_argument("--straddle-group", action="store_true",
                   help="line-straddling sources: the shipped shape against the group-interleaved XCD order (15/16)")
    p.add_argument("--caps", action="store_true", help="wave-cap sweep of the loads-first variants (8, 9)")
    p.add_argument("--walk", action="store_true", help="the walking variants (dccl_tune_phased_walk_f32_sum) instead")
    p.add_argument("--chain", action="store_true", help="also the phased chain kernel, XCD order off / on")
    p.add_argument("--out", default="")
    a = p.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 1 << 30
    n = nbytes // 4 - 64
    recv = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    srcs = torch.empty(8 * (nbytes + 4096) + 256, dtype=torch.uint8, device="cuda")
    dccl_amd.check(dccl_amd.synth_fill(recv.data_ptr(), 7, nbytes // 4, 0, 0xDCC1, 1, st), "synth")
    rows = []
    if a.walk:
        walk(a, recv, srcs, n, nbytes, st, rows)
        return finish(a, rows)
    if a.caps:
        caps(a, recv, srcs, n, nbytes, st, rows)
        return finish(a, rows)
    if a.prod_caps:
        prod_caps(a, recv, srcs, n, nbytes, st, rows)
        return finish(a, rows)
    if a.swap:
        swap_tiling(a, recv, srcs, n, nbytes, st, rows)
        return finish(a, rows)
    if a.straddle_caps:
        straddle_caps(a, recv, srcs, n, nbytes, st, rows)
        return finish(a, rows)
    if a.straddle_group:
        straddle_group(a, recv, srcs, n, nbytes, st, rows)
        return finish(a, rows)
    if a.straddle:
        straddle(a, recv, srcs, n, nbytes, st, rows)
        return finish(a, rows)
    for k, phase in ((1, 4), (2, 4), (3, 4), (4, 4), (5, 4), (6, 4), (7, 4), (8, 4)):
        sp = [srcs.data_ptr() + j * (nbytes + 4096) + phase for j in range(k)]
        for j, q in enumerate(sp):
            dccl_amd.check(dccl_amd.synth_fill(q, 7, n, 0, 0xDCC1, 10 + j, st), "synth")
        arr = (ctypes.c_void_p * k)(*sp)
        t = {v: [] for v in VARIANTS}
        for _ in range(a.rounds):
            for v in VARIANTS:
                fn = lambda v=v: dccl_amd.check(tune_lib.lib.dccl_tune_phased_f32_sum(arr, k, recv.data_ptr(), n, v,
                                                                                     0, st), "phased")
                t[v].append(time_launches([fn], rounds=1, min_ms=20.0)[0])
        for v in VARIANTS:
            ms = statistics.median(t[v])
            rows.append({"k": k, "phase": phase, "variant": v, "ms": round(ms, 4),
                         "frac": round((k + 2) * n * 4 / (ms * 1e-3) / 1e9 / PEAK, 4)})
            print(json.dumps(rows[-1]), flush=True)
    # chain (ring order), in place: own = recv (in phase), k sources +4 B; XCD order off (0) / on (1)
    for k in ((1, 2, 3, 4, 5, 7) if a.chain else ()):
        sp = [srcs.data_ptr() + j * (nbytes + 4096) + 4 for j in range(k)]
        arr = (ctypes.c_void_p * k)(*sp)
        t = {v: [] for v in (0, 1)}
        for _ in range(a.rounds):
            for v in (0, 1):
                fn = lambda v=v: dccl_amd.check(tune_lib.lib.dccl_tune_chain_phased_f32_sum(
                    arr, k, recv.data_ptr(), recv.data_ptr(), n, v, st), "chain phased")
                t[v].append(time_launches([fn], rounds=1, min_ms=20.0)[0])
        for v in (0, 1):
            ms = statistics.median(t[v])
            rows.append({"chain_k": k, "phase": 4, "xcd": v, "ms": round(ms, 4),
                         "frac": round((k + 2) * n * 4 / (ms * 1e-3) / 1e9 / PEAK, 4)})
            print(json.dumps(rows[-1]), flush=True)
    finish(a, rows)


def finish(a, rows):
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


VSTRADDLE = (0, 8, 14)


def swap_tiling(a, recv, srcs, n, nbytes, st, rows):
    """Every source at +4 B, recv 128-B aligned: the shipped phased dispatch (dccl_local_reduce_multi /
    _chain) against the unaligned kernels started 3 elements in, so the sources' vectors are aligned and recv
    is the operand accessed at an unaligned address (the 3 head elements are not timed), under wave caps
    PHASED_WAVES."""
    ws = tuple(int(x) for x in os.environ.get("PHASED_WAVES", "32,28,24,20,16,13").split(","))
    for k in tuple(int(x) for x in os.environ.get("PHASED_K", "2,3,4,5,6,7,8").split(",")):
        sp = [srcs.data_ptr() + j * (nbytes + 4096) + 4 for j in range(k)]
        for j, q in enumerate(sp):
            dccl_amd.check(dccl_amd.synth_fill(q, 7, n, 0, 0xDCC1, 10 + j, st), "synth")
        arr = (ctypes.c_void_p * k)(*sp)
        arr_sw = (ctypes.c_void_p * k)(*[q + 12 for q in sp])
        r0 = recv.data_ptr()
        for what in ("multi", "chain"):
            t = {"shipped": []}
            t.update({w: [] for w in ws})
            for _ in range(a.rounds):
                if what == "multi":
                    f0 = lambda: dccl_amd.check(dccl_amd.local_reduce_multi(sp, r0, 7, n, 0, st), "multi")
                else:
                    f0 = lambda: dccl_amd.check(dccl_amd.local_reduce_chain(sp, r0, r0, 7, n, 0, st), "chain")
                t["shipped"].append(time_launches([f0], rounds=1, min_ms=20.0)[0])
                for w in ws:
                    lds = 0 if w >= 32 else ((160 << 10) // w + 255) // 256 * 256
                    own = None if what == "multi" else r0 + 12
                    fn = lambda lds=lds, own=own: dccl_amd.check(tune_lib.lib.dccl_tune_unaligned_kway_f32_sum(
                        arr_sw, k, own, r0 + 12, n - 3, lds, 0, st), "swap")
                    t[w].append(time_launches([fn], rounds=1, min_ms=20.0)[0])
            for key, v in t.items():
                ms = statistics.median(v)
                rows.append({"what": what, "k": k, "tiling": "shipped" if key == "shipped" else f"swap@{key}",
                             "frac": round((k + 2) * n * 4 / (ms * 1e-3) / 1e9 / PEAK, 4)})
                print(json.dumps(rows[-1]), flush=True)


def prod_caps(a, recv, srcs, n, nbytes, st, rows):
    """The shipped phased kernels (dccl_tune_phased_prod_f32_sum), k-way and chain (in place), sources +4 B:
    the shipped form (first 0, its XCD rule, no cap) against the loads-first form under wave caps PHASED_WAVES,
    for k in PHASED_K."""
    ws = tuple(int(x) for x in os.environ.get("PHASED_WAVES", "9,10,11,12,13,14,16").split(","))
    for k in tuple(int(x) for x in os.environ.get("PHASED_K", "3,4,5,6,7,8").split(",")):
        sp = [srcs.data_ptr() + j * (nbytes + 4096) + 4 for j in range(k)]
        for j, q in enumerate(sp):
            dccl_amd.check(dccl_amd.synth_fill(q, 7, n, 0, 0xDCC1, 10 + j, st), "synth")
        arr = (ctypes.c_void_p * k)(*sp)
        configs = [(0, 32)] + [(1, w) for w in ws]
        for what in ("multi", "chain"):
            own = None if what == "multi" else recv.data_ptr()
            t = {c: [] for c in configs}
            for _ in range(a.rounds):
                for f, w in configs:
                    lds = 0 if w >= 32 else ((160 << 10) // w + 255) // 256 * 256
                    x = int(k <= 4) if f == 0 else 0
                    fn = lambda f=f, lds=lds, x=x: dccl_amd.check(tune_lib.lib.dccl_tune_phased_prod_f32_sum(
                        arr, k, own, recv.data_ptr(), n, f, x, lds, st), "phased prod")
                    t[(f, w)].append(time_launches([fn], rounds=1, min_ms=20.0)[0])
            for f, w in configs:
                ms = statistics.median(t[(f, w)])
                rows.append({"what": what, "k": k, "first": f, "waves": w, "ms": round(ms, 4),
                             "frac": round((k + 2) * n * 4 / (ms * 1e-3) / 1e9 / PEAK, 4)})
                print(json.dumps(rows[-1]), flush=True)


def straddle_caps(a, recv, srcs, n, nbytes, st, rows):
    """The shipped line-straddle k-way and chain shapes (sources cached) under explicit wave caps
    (STRADDLE_WAVES, STRADDLE_K); the chain runs in place (own = dst = recv)."""
    ks = tuple(int(x) for x in os.environ.get("STRADDLE_K", "5,6,7,8").split(","))
    variant = int(os.environ.get("STRADDLE_VARIANT", "8"))  # 8: shipped shape; 11: head aligned to sends[0]
    for k in ks:
        sp = [srcs.data_ptr() + j * (nbytes + 4096) + (16 if a.common_phase else 16 * (2 * j + 1)) for j in range(k)]
        for j, q in enumerate(sp):
            dccl_amd.check(dccl_amd.synth_fill(q, 7, n, 0, 0xDCC1, 10 + j, st), "synth")
        arr = (ctypes.c_void_p * k)(*sp)
        waves = tuple(int(x) for x in os.environ.get("STRADDLE_WAVES", "9,11,13,16,20,24,32").split(","))
        t = {w: [] for w in waves}
        for _ in range(a.rounds):
            for w in waves:
                lds = 0 if w >= 32 else ((160 << 10) // w + 255) // 256 * 256
                fn = lambda lds=lds: dccl_amd.check(tune_lib.lib.dccl_tune_multi_f32_sum(
                    arr, k, recv.data_ptr(), n, variant, lds, st), "multi straddle")
                t[w].append(time_launches([fn], rounds=1, min_ms=20.0)[0])
        tc = {w: [] for w in waves}
        for _ in range(a.rounds):
            for w in waves:
                lds = 0 if w >= 32 else ((160 << 10) // w + 255) // 256 * 256
                fn = lambda lds=lds: dccl_amd.check(tune_lib.lib.dccl_tune_chain_policy_f32_sum(
                    arr, k, recv.data_ptr(), recv.data_ptr(), n, lds, 6, st), "chain straddle")
                tc[w].append(time_launches([fn], rounds=1, min_ms=20.0)[0])
        for w in waves:
            for what, tt in (("multi", t), ("chain", tc)):
                ms = statistics.median(tt[w])
                rows.append({"what": what, "k": k, "waves": w, "variant": variant if what == "multi" else 6,
                             "ms": round(ms, 4),
                             "frac": round((k + 2) * n * 4 / (ms * 1e-3) / 1e9 / PEAK, 4)})
                print(json.dumps(rows[-1]), flush=True)


STRADDLE_WAVES = [32, 32, 18, 13, 13, 11, 9, 9, 7]  # kStraddleWaves in dccl_amd/csrc/reduce_kernels.hpp


def straddle_group(a, recv, srcs, n, nbytes, st, rows):
    """Sources 16-B aligned but off recv's 128-B lines (+16 (2j+1) B), k in STRADDLE_K: the shipped straddle
    shape (variant 8, sources cached, block order) at its shipped cap against the group-interleaved XCD order
    (15: sources cached, 16: all non-temporal) under the caps STRADDLE_WAVES (32 = uncapped).  First checks
    15 and 16 against the product entry point bit for bit on a small ragged size."""
    m = 100_003
    small = [srcs.data_ptr() + j * (nbytes + 4096) + 16 * (2 * j + 1) for j in range(8)]
    for j, q in enumerate(small):
        dccl_amd.check(dccl_amd.synth_fill(q, 7, m, 0, 0xDCC1, 10 + j, st), "synth")
    for k in range(2, 9):
        arr = (ctypes.c_void_p * k)(*small[:k])
        ref = torch.empty(4 * m + 256, dtype=torch.uint8, device="cuda")
        dccl_amd.check(dccl_amd.synth_fill(ref.data_ptr() + 128, 7, m, 0, 0xDCC1, 1, st), "synth")
        base = ref.clone()
        dccl_amd.check(dccl_amd.local_reduce_multi(small[:k], ref.data_ptr() + 128, 7, m, 0, st), "multi")
        for v in (15, 16):
            got = base.clone()
            dccl_amd.check(tune_lib.lib.dccl_tune_multi_f32_sum(arr, k, got.data_ptr() + 128, m, v, 0, st), "v")
            torch.cuda.synchronize()
            assert torch.equal(got, ref), (k, v)
    print("group-order variants bit-exact against the product", flush=True)
    ws = tuple(int(x) for x in os.environ.get("STRADDLE_WAVES", "32,20,16,13,11,9").split(","))
    for k in tuple(int(x) for x in os.environ.get("STRADDLE_K", "4,5,6,7,8").split(",")):
        sp = [srcs.data_ptr() + j * (nbytes + 4096) + 16 * (2 * j + 1) for j in range(k)]
        for j, q in enumerate(sp):
            dccl_amd.check(dccl_amd.synth_fill(q, 7, n, 0, 0xDCC1, 10 + j, st), "synth")
        arr = (ctypes.c_void_p * k)(*sp)
        configs = [(8, STRADDLE_WAVES[k])] + [(v, w) for v in (15, 16) for w in ws]
        t = {c: [] for c in configs}
        for _ in range(a.rounds):
            for v, w in configs:
                lds = 0 if w >= 32 else ((160 << 10) // w + 255) // 256 * 256
                fn = lambda v=v, lds=lds: dccl_amd.check(tune_lib.lib.dccl_tune_multi_f32_sum(
                    arr, k, recv.data_ptr(), n, v, lds, st), "multi straddle")
                t[(v, w)].append(time_launches([fn], rounds=1, min_ms=20.0)[0])
        for v, w in configs:
            ms = statistics.median(t[(v, w)])
            rows.append({"k": k, "variant": v, "waves": w, "ms": round(ms, 4),
                         "frac": round((k + 2) * n * 4 / (ms * 1e-3) / 1e9 / PEAK, 4)})
            print(json.dumps(rows[-1]), flush=True)


def straddle(a, recv, srcs, n, nbytes, st, rows):
    """Sources 16-B aligned but off recv's 128-B lines (+16, +48, +80 ... B), k = 1..8, the k-way kernel under
    the shipped wave caps in four shapes: 0 all non-temporal, 8 sources cached (shipped), 9 / 10 the same
    with each XCD's tiles one contiguous range."""
    waves = [32, 32, 18, 13, 13, 11, 11, 10, 9]  # kMultiWaves in dccl_amd/csrc/reduce_kernels.hpp
    for k in range(1, 9):
        sp = [srcs.data_ptr() + j * (nbytes + 4096) + (16 if a.common_phase else 16 * (2 * j + 1)) for j in range(k)]
        for j, q in enumerate(sp):
            dccl_amd.check(dccl_amd.synth_fill(q, 7, n, 0, 0xDCC1, 10 + j, st), "synth")
        arr = (ctypes.c_void_p * k)(*sp)
        lds = 0 if waves[k] >= 32 else ((160 << 10) // waves[k] + 255) // 256 * 256
        t = {v: [] for v in VSTRADDLE}
        for _ in range(a.rounds):
            for v in VSTRADDLE:
                fn = lambda v=v: dccl_amd.check(tune_lib.lib.dccl_tune_multi_f32_sum(
                    arr, k, recv.data_ptr(), n, v, lds, st), "multi straddle")
                t[v].append(time_launches([fn], rounds=1, min_ms=20.0)[0])
        for v in VSTRADDLE:
            ms = statistics.median(t[v])
            rows.append({"k": k, "source_offsets": "16" if a.common_phase else "16 (2j+1)", "multi_variant": v, "ms": round(ms, 4),
                         "frac": round((k + 2) * n * 4 / (ms * 1e-3) / 1e9 / PEAK, 4)})
            print(json.dumps(rows[-1]), flush=True)


def caps(a, recv, srcs, n, nbytes, st, rows):
    """Variants 0 (shipped, uncapped), 8 (loads first) and 9 (loads first, XCD order) under explicit wave caps
    (unused dynamic LDS per one-wave block: 160 KiB / waves), k = 2, 4, 7, sources +4 B."""
    ws = tuple(int(x) for x in os.environ.get("PHASED_WAVES", "32,24,20,16,13,11").split(","))
    configs = [(0, 0)] + [(v, w) for v in (8, 9) for w in ws]
    for k in tuple(int(x) for x in os.environ.get("PHASED_K", "2,4,7").split(",")):
        sp = [srcs.data_ptr() + j * (nbytes + 4096) + 4 for j in range(k)]
        for j, q in enumerate(sp):
            dccl_amd.check(dccl_amd.synth_fill(q, 7, n, 0, 0xDCC1, 10 + j, st), "synth")
        arr = (ctypes.c_void_p * k)(*sp)
        t = {c: [] for c in configs}
        for _ in range(a.rounds):
            for v, w in configs:
                lds = 0 if w in (0, 32) else ((160 << 10) // w + 255) // 256 * 256
                fn = lambda v=v, lds=lds: dccl_amd.check(tune_lib.lib.dccl_tune_phased_f32_sum(
                    arr, k, recv.data_ptr(), n, v, lds, st), "phased caps")
                t[(v, w)].append(time_launches([fn], rounds=1, min_ms=20.0)[0])
        for v, w in configs:
            ms = statistics.median(t[(v, w)])
            rows.append({"k": k, "phase": 4, "variant": v, "waves": w or 32, "ms": round(ms, 4),
                         "frac": round((k + 2) * n * 4 / (ms * 1e-3) / 1e9 / PEAK, 4)})
            print(json.dumps(rows[-1]), flush=True)


def walk(a, recv, srcs, n, nbytes, st, rows):
    """Variants 0-8 of the walking kernel (U = 1, 2, 4 tiles per wave x block order in order / range split per
    XCD / group-interleaved), each first checked bit-exact against dccl_local_reduce_multi on a fresh copy."""
    ref = recv.clone()
    for k in (1, 2, 4, 7):
        sp = [srcs.data_ptr() + j * (nbytes + 4096) + 4 for j in range(k)]
        for j, q in enumerate(sp):
            dccl_amd.check(dccl_amd.synth_fill(q, 7, n, 0, 0xDCC1, 10 + j, st), "synth")
        arr = (ctypes.c_void_p * k)(*sp)
        want = ref.clone()
        dccl_amd.check(dccl_amd.local_reduce_multi(sp, want.data_ptr(), 7, n, 0, st), "multi")
        ok = {}
        for v in range(9):
            got = ref.clone()
            dccl_amd.check(tune_lib.lib.dccl_tune_phased_walk_f32_sum(arr, k, got.data_ptr(), n, v, st), "walk")
            torch.cuda.synchronize()
            ok[v] = bool(torch.equal(got, want))
            del got
        t = {v: [] for v in range(9)}
        for _ in range(a.rounds):
            for v in range(9):
                fn = lambda v=v: dccl_amd.check(tune_lib.lib.dccl_tune_phased_walk_f32_sum(
                    arr, k, recv.data_ptr(), n, v, st), "walk")
                t[v].append(time_launches([fn], rounds=1, min_ms=20.0)[0])
        for v in range(9):
            ms = statistics.median(t[v])
            rows.append({"k": k, "phase": 4, "walk_variant": v, "tiles_per_wave": 1 << (v % 3),
                         "order": ("blocks in order", "range split per XCD", "group-interleaved")[v // 3],
                         "bit_exact": ok[v], "ms": round(ms, 4),
                         "frac": round((k + 2) * n * 4 / (ms * 1e-3) / 1e9 / PEAK, 4)})
            print(json.dumps(rows[-1]), flush=True)
        del want


if __name__ == "__main__":
    main()
