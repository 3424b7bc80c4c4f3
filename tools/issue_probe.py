#!/usr/bin/env python3
"""Issue-side counters of the misaligned-operand combine classes beside their in-phase twins (VERDICT r2
"next" item 3): is the 4-8-point gap of these kernels on the issue side (the per-operand DPP + v_alignbyte
chain, lane 63's extra load) or in the memory system?  Tuning only.

Workload (run under rocprofv3 --pmc <counters> --kernel-trace): ten 1 GiB fp32 operands carved from one
allocation with a 4 KiB x (j+1) stagger (kway_pmc_probe.py's layout), sources ptrs[0..7], destination
ptrs[8]; each case --launches launches of N - 64 elements, in this order:

  pair          dccl_local_reduce, aligned                    reduce_vec_kernel                (k = 1)
  pair_dst+1    dccl_local_reduce, recv + 1 B                 reduce_unaligned_kernel          (k = 1)
  multi4        dccl_local_reduce_multi, k = 4, in phase      reduce_multi_vec_kernel
  multi4_dst+2  the same into recv + 2 B                      reduce_multi_unaligned_kernel
  multi6        k = 6, in phase                               reduce_multi_vec_kernel
  multi6_src+4  k = 6, every source + 4 B                     reduce_multi_phased_kernel (per operand)
  multi8        k = 8, in phase                               reduce_multi_vec_kernel
  multi8_strad  k = 8, source j + 16 (2j + 1) B (in phase, off recv's 128-B lines)  straddle launch

    rocprofv3 --pmc C1 C2 ... --kernel-trace --output-format csv -d OUT/<pass> -o p -- python3 tools/issue_probe.py
    python3 tools/issue_probe.py --parse OUT [--out profiles/x.json]
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 8e12
CASES = [("pair", 1), ("pair_dst+1", 1), ("multi4", 4), ("multi4_dst+2", 4), ("multi6", 6), ("multi6_src+4", 6),
         ("multi8", 8), ("multi8_strad", 8)]


def run(launches: int, mib: int, only: str) -> None:
    import torch
    sys.path.insert(0, ROOT)
    import dccl_amd
    nbytes = mib << 20
    n = nbytes // 4
    st = torch.cuda.current_stream().cuda_stream
    pool = torch.empty(10 * nbytes + 4096 * 55 + 1024, dtype=torch.uint8, device="cuda")
    ptrs, off = [], 0
    for j in range(10):
        ptrs.append(pool.data_ptr() + off)
        dccl_amd.check(dccl_amd.synth_fill(ptrs[-1], 7, n, 0, 0xDCC1, 10 + j, st), "synth")
        off += nbytes + 4096 * (j + 1)
    recv, cnt = ptrs[8], n - 64

    def multi(sends, dst):
        dccl_amd.check(dccl_amd.local_reduce_multi(sends, dst, 7, cnt, 0, st), "multi")

    calls = {
        "pair": lambda: dccl_amd.check(dccl_amd.local_reduce(ptrs[0], recv, 7, cnt, 0, st), "pair"),
        "pair_dst+1": lambda: dccl_amd.check(dccl_amd.local_reduce(ptrs[0], recv + 1, 7, cnt, 0, st), "pair"),
        "multi4": lambda: multi(ptrs[:4], recv),
        "multi4_dst+2": lambda: multi(ptrs[:4], recv + 2),
        "multi6": lambda: multi(ptrs[:6], recv),
        "multi6_src+4": lambda: multi([p + 4 for p in ptrs[:6]], recv),
        "multi8": lambda: multi(ptrs[:8], recv),
        "multi8_strad": lambda: multi([p + 16 * (2 * j + 1) for j, p in enumerate(ptrs[:8])], recv),
    }
    order = []
    torch.cuda.synchronize()
    for name, k in CASES:
        if only and name not in only.split(","):
            continue
        for _ in range(launches):
            calls[name]()
            order.append({"what": name, "k": k})
    torch.cuda.synchronize()
    print(json.dumps({"order": order, "bytes_per_operand": nbytes, "count": cnt}), flush=True)


def _load(pdir):
    ktr = glob.glob(os.path.join(pdir, "**", "*kernel_trace.csv"), recursive=True)
    ctr = glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True)
    order, count = None, None
    for lg in glob.glob(os.path.join(pdir, "*.log")):
        for line in open(lg):
            if line.startswith('{"order"'):
                d = json.loads(line)
                order, count = d["order"], d["count"]
    if not ktr or order is None:
        return None, count
    dur, names = {}, {}
    with open(ktr[0]) as f:
        for row in csv.DictReader(f):
            nm = row.get("Kernel_Name", "")
            if "reduce_" in nm and "synth" not in nm:
                d = int(row["Dispatch_Id"])
                dur[d] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
                names[d] = nm
    cnt = {}
    for path in ctr:
        with open(path) as f:
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
        e = out.setdefault(lab["what"], {"k": lab["k"], "ms": [], "counters": {}, "kernel": names[d].split("(")[0]})
        e["ms"].append(dur[d])
        for k, v in cnt.get(d, {}).items():
            e["counters"].setdefault(k, []).append(v)
    return out, count


def parse(outdir: str, dst: str) -> None:
    rows = {}
    count = None
    for pdir in sorted(glob.glob(os.path.join(outdir, "*"))):
        if not os.path.isdir(pdir):
            continue
        got, c = _load(pdir)
        count = c or count
        for name, e in (got or {}).items():
            r = rows.setdefault(name, {"k": e["k"], "kernel": e["kernel"], "ms": [], "counters": {}})
            r["ms"] += e["ms"]
            for k, v in e["counters"].items():
                r["counters"][k] = statistics.median(v)
    out = []
    for name, _ in CASES:
        if name not in rows:
            continue
        r = rows[name]
        ms = statistics.median(r["ms"])
        c = r["counters"]
        row = {"case": name, "k": r["k"], "kernel": r["kernel"], "ms": round(ms, 4),
               "frac_of_peak": round((r["k"] + 2) * count * 4 / (ms * 1e-3) / PEAK, 4), "counters": c}
        waves = c.get("SQ_WAVES")
        if waves:
            for key in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU",
                        "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY",
                        "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM"):
                if key in c:
                    row[key.lower() + "_per_wave"] = round(c[key] / waves, 2)
        if c.get("SQ_WAVE_CYCLES"):
            for key in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
                if key in c:
                    row[key.lower() + "_frac_of_wave_cycles"] = round(c[key] / c["SQ_WAVE_CYCLES"], 4)
        out.append(row)
    res = {"count": count, "layout": "one allocation, 4 KiB x (j+1) gaps, 1 GiB fp32 operands",
           "note": "durations from the profiled (serialised) dispatches of every pass; counters: median over "
                   "a case's dispatches, summed over the chip", "rows": out}
    txt = json.dumps(res, indent=1)
    if dst:
        with open(dst, "w") as fh:
            fh.write(txt)
    print(txt)


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--launches", type=int, default=3)
    p.add_argument("--mib", type=int, default=1024)
    p.add_argument("--only", default="", help="comma-separated case names")
    p.add_argument("--parse", default="")
    p.add_argument("--out", default="")
    a = p.parse_args()
    if a.parse:
        parse(a.parse, a.out)
    else:
        run(a.launches, a.mib, a.only)
