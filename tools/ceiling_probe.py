#!/usr/bin/env python3
"""Where the combine sits between the chip's own HBM streaming limits (MI355X).

Times, interleaved in one process, the shipped access shape (one-wave blocks, 16 B per lane, all
non-temporal) doing: read one operand, read both, write one, copy one into the other, and the fp32
Sum combine (2 reads + 1 write); the read-both and write probes again in 256-thread x 4-vector
blocks (a quarter of the workgroups); and the shipped grid of empty workgroups (dispatch alone).  Operands are 1 GiB each, carved from one allocation as in bench.py
(recv, then send 4 KiB past its end).  Reports the bytes each kernel actually moves per second, so
the combine's rate can be compared with the pure-read and pure-write ceilings of the same shape.

    python tools/ceiling_probe.py [--mib 1024] [--rounds 7] [--iters 20] [--out file]
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

KINDS = {0: ("read send", 1), 1: ("read send + recv", 2), 2: ("write recv", 1), 3: ("copy send -> recv", 2),
         4: ("combine recv += send", 3), 5: ("read send + recv, 256x4 blocks", 2),
         6: ("write recv, 256x4 blocks", 1), 7: ("empty workgroups, shipped grid", 0),
         8: ("combine, recv load first", 3)}
SPLITS = (2, 4)  # the production combine split into this many slices on as many streams


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mib", type=int, default=1024)
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--out", default="")
    a = p.parse_args()
    n = (a.mib << 20) // 4
    pool = torch.empty(2 * n * 4 + 4096, dtype=torch.uint8, device="cuda")
    recv = pool[: n * 4].view(torch.float32)
    send = pool[n * 4 + 4096:].view(torch.float32)
    send.uniform_(-1, 1)
    recv.uniform_(-1, 1)
    st = torch.cuda.current_stream().cuda_stream
    for k in KINDS:
        assert tune_lib.lib.dccl_tune_ceiling(k, send.data_ptr(), recv.data_ptr(), n, st) == 0, k
    streams = [torch.cuda.Stream() for _ in range(max(SPLITS))]

    def split_combine(parts):
        # slices of the production combine on `parts` streams, joined back into the current stream
        start = torch.cuda.Event()
        start.record()
        per = n // parts
        for j in range(parts):
            sj = streams[j]
            sj.wait_event(start)
            dccl_amd.check(dccl_amd.local_reduce(send.data_ptr() + 4 * j * per, recv.data_ptr() + 4 * j * per, 7,
                                                 per, 0, sj.cuda_stream))
            done = torch.cuda.Event()
            done.record(sj)
            torch.cuda.current_stream().wait_event(done)

    torch.cuda.synchronize()
    times = {k: [] for k in list(KINDS) + [f"split{p}" for p in SPLITS]}
    for _ in range(a.rounds):
        for k in times:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                if isinstance(k, str):
                    split_combine(int(k[5:]))
                else:
                    tune_lib.lib.dccl_tune_ceiling(k, send.data_ptr(), recv.data_ptr(), n, st)
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / a.iters)
    rows = []
    for k, (name, streams) in KINDS.items():
        med = statistics.median(times[k])
        moved = streams * n * 4
        rows.append({"kind": k, "what": name, "bytes_moved": moved, "ms_median": round(med, 4),
                     "ms_min": round(min(times[k]), 4), "gb_s": round(moved / (med * 1e-3) / 1e9, 1), "workgroups_per_us": round(
                         (n // 256 if k not in (5, 6) else n // 4096) / (med * 1e3), 1),
                     "frac_of_8tbs": round(moved / (med * 1e-3) / 8e12, 4)})
    for p_ in SPLITS:
        med = statistics.median(times[f"split{p_}"])
        rows.append({"kind": f"split{p_}", "what": f"production combine in {p_} slices on {p_} streams",
                     "bytes_moved": 3 * n * 4, "ms_median": round(med, 4), "ms_min": round(min(times[f"split{p_}"]), 4),
                     "gb_s": round(3 * n * 4 / (med * 1e-3) / 1e9, 1),
                     "frac_of_8tbs": round(3 * n * 4 / (med * 1e-3) / 8e12, 4)})
    # write-only ceiling over block shapes and store policies (dccl_tune_write_probe)
    import ctypes
    wrows = []
    nw = tune_lib.lib.dccl_tune_write_num_variants()
    shapes = []
    for v in range(nw):
        b, u, pol = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        assert tune_lib.lib.dccl_tune_write_probe(v, recv.data_ptr(), n, ctypes.byref(b), ctypes.byref(u), ctypes.byref(pol),
                                         ctypes.c_void_p(~0 & ((1 << 64) - 1))) == 0
        shapes.append((b.value, u.value, ("plain", "nt", "sc1")[pol.value]))
    dummy = [ctypes.c_int() for _ in range(3)]
    wt = {v: [] for v in range(nw)}
    for _ in range(a.rounds):
        for v in range(nw):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                tune_lib.lib.dccl_tune_write_probe(v, recv.data_ptr(), n, *[ctypes.byref(x) for x in dummy], st)
            e1.record()
            e1.synchronize()
            wt[v].append(e0.elapsed_time(e1) / a.iters)
    for v in range(nw):
        med = statistics.median(wt[v])
        b, u, pol = shapes[v]
        wrows.append({"block": b, "vectors_per_lane": u, "store": pol, "ms_median": round(med, 4),
                      "gb_s": round(n * 4 / (med * 1e-3) / 1e9, 1), "frac_of_8tbs": round(n * 4 / (med * 1e-3) / 8e12, 4)})
    wrows.sort(key=lambda x: x["ms_median"])
    out = {"mib_per_operand": a.mib, "device": torch.cuda.get_device_name(0), "rows": rows, "write_shapes": wrows}
    txt = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
