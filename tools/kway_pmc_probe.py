#!/usr/bin/env python3
"""HBM traffic of the k-way and chain combines per k: is it (k+2)*N or more?

Workload (run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-trace): ten 1 GiB fp32 operands
carved from one allocation with a 4 KiB x (j+1) stagger (tools/bench_suite.py's "staggered" layout);
for k = 1..8, --launches launches of dccl_local_reduce_multi (recv = recv + s0 + ... ) and of
dccl_local_reduce_chain (own in place), in that order; --phase P puts every source P bytes further (P = 4:
the phased kernels, sources off the destination's 16-B phase).  Counts are N - 16 elements.  The parse step joins each dispatch's duration
with its counters and reports, per kernel and k, read bytes = 2 x FETCH_SIZE (gfx950 wide-read halving,
MI355X_MICROARCH.md §HBM), write bytes = WRITE_SIZE, their ratio to (k+1)*N and N, and the fraction
of the 8 TB/s peak the dispatch ran at.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT/fetch -o p -- python3 tools/kway_pmc_probe.py
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d OUT/write -o p -- python3 tools/kway_pmc_probe.py
    python3 tools/kway_pmc_probe.py --parse OUT [--out profiles/x.json]
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NBYTES = 1 << 30
PEAK = 8e12


def run(launches: int, mib: int, phase: int = 0) -> None:
    import torch
    sys.path.insert(0, ROOT)
    import dccl_amd
    nbytes = mib << 20
    n = nbytes // 4
    st = torch.cuda.current_stream().cuda_stream
    pool = torch.empty(10 * nbytes + 4096 * 55 + 64, dtype=torch.uint8, device="cuda")
    ptrs, off = [], 0
    for j in range(10):
        ptrs.append(pool.data_ptr() + off)
        dccl_amd.check(dccl_amd.synth_fill(ptrs[-1], 7, n, 0, 0xDCC1, 10 + j, st), "synth")
        off += nbytes + 4096 * (j + 1)
    sends, recv = [q + phase for q in ptrs[:8]], ptrs[8]  # phase != 0: the phased kernels
    torch.cuda.synchronize()
    order = []
    for k in range(1, 9):
        for _ in range(launches):
            dccl_amd.check(dccl_amd.local_reduce_multi(sends[:k], recv, 7, n - 16, 0, st), "multi")
            order.append({"what": "multi", "k": k})
        for _ in range(launches):
            dccl_amd.check(dccl_amd.local_reduce_chain(sends[:k], recv, recv, 7, n - 16, 0, st), "chain")
            order.append({"what": "chain", "k": k})
    torch.cuda.synchronize()
    print(json.dumps({"order": order, "bytes_per_operand": nbytes, "phase": phase}), flush=True)


def _load(pdir):
    ktr = glob.glob(os.path.join(pdir, "**", "*kernel_trace.csv"), recursive=True)
    ctr = glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True)
    order, nbytes = None, NBYTES
    for lg in glob.glob(os.path.join(pdir, "*.log")):
        for line in open(lg):
            if line.startswith('{"order"'):
                d = json.loads(line)
                order, nbytes = d["order"], d["bytes_per_operand"]
    if not ktr or not ctr or order is None:
        return None, nbytes
    dur, names = {}, {}
    with open(ktr[0]) as f:
        for row in csv.DictReader(f):
            nm = row.get("Kernel_Name", "")
            if "multi" in nm or "chain" in nm or "shift" in nm or "vec_kernel" in nm:
                d = int(row["Dispatch_Id"])
                dur[d] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
                names[d] = nm
    cnt = {}
    with open(ctr[0]) as f:
        for row in csv.DictReader(f):
            d = int(row["Dispatch_Id"])
            if d in dur:
                cnt.setdefault(d, {}).setdefault(row["Counter_Name"], 0.0)
                cnt[d][row["Counter_Name"]] += float(row["Counter_Value"])
    ids = sorted(dur)
    if len(ids) != len(order):
        raise SystemExit(f"{pdir}: {len(ids)} dispatches vs {len(order)} launches")
    out = {}
    for lab, d in zip(order, ids):
        e = out.setdefault((lab["what"], lab["k"]), {"ms": [], "counters": {}, "kernel": names[d].split("(")[0]})
        e["ms"].append(dur[d])
        for k, v in cnt.get(d, {}).items():
            e["counters"].setdefault(k, []).append(v)
    return out, nbytes


def parse(outdir: str, dst: str) -> None:
    fetch, nbytes = _load(os.path.join(outdir, "fetch"))
    write, _ = _load(os.path.join(outdir, "write"))
    rows = []
    for key in sorted(fetch or {}):
        what, k = key
        f = fetch[key]
        w = (write or {}).get(key, {"ms": [], "counters": {}})
        ms = statistics.median(f["ms"] + w["ms"])
        fs = statistics.median(f["counters"].get("FETCH_SIZE", [0]))
        ws = statistics.median(w["counters"].get("WRITE_SIZE", [0])) if w["counters"] else None
        rd = 2 * fs * 1024
        row = {"what": what, "k": k, "kernel": f["kernel"], "ms": round(ms, 4),
               "frac_of_peak": round((k + 2) * nbytes / (ms * 1e-3) / PEAK, 4),
               "read_bytes": rd, "read_over_algorithmic": round(rd / ((k + 1) * nbytes), 5)}
        if ws is not None:
            row["write_bytes"] = ws * 1024
            row["write_over_algorithmic"] = round(ws * 1024 / nbytes, 5)
            row["traffic_over_algorithmic"] = round((rd + ws * 1024) / ((k + 2) * nbytes), 5)
        rows.append(row)
    res = {"bytes_per_operand": nbytes, "layout": "staggered (one allocation, 4 KiB x (j+1) gaps)",
           "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950), write = WRITE_SIZE x 1024",
           "note": "durations from the profiled (serialised) dispatches of both passes", "rows": rows}
    txt = json.dumps(res, indent=1)
    if dst:
        with open(dst, "w") as fh:
            fh.write(txt)
    print(txt)


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--launches", type=int, default=2)
    p.add_argument("--mib", type=int, default=1024)
    p.add_argument("--phase", type=int, default=0, help="byte offset of every source (4: the phased kernels)")
    p.add_argument("--parse", default="")
    p.add_argument("--out", default="")
    a = p.parse_args()
    if a.parse:
        parse(a.parse, a.out)
    else:
        run(a.launches, a.mib, a.phase)
