#!/usr/bin/env python3
"""Which counter separates the fast and slow placement modes of separately allocated operands?


Workload (run under rocprofv3 --pmc ... --kernel-trace): one pooled pair (bench.py's layout) and
--pairs separately allocated pairs of 1 GiB fp32 operands; each pair gets --launches combines of the
shipped kernel, in pair order.  Every dispatch then carries its duration (kernel trace) and the
counters of the pass, so fast and slow pairs of the same process can be compared counter by counter.

    rocprofv3 --pmc C1 C2 C3 C4 --kernel-trace --output-format csv -d OUT/pN -o p -- python3 tools/layout_pmc_probe.py
    python3 tools/layout_pmc_probe.py --parse OUT [--out profiles/x.json]
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "reduce_vec_kernel"
NBYTES = 1 << 30


def run(pairs: int, launches: int) -> None:
    import torch
    sys.path.insert(0, ROOT)
    import dccl_amd
    st = torch.cuda.current_stream().cuda_stream
    n = NBYTES // 4
    sets = []
    pool = torch.empty(2 * NBYTES + 4096, dtype=torch.uint8, device="cuda")
    sets.append(("pooled", pool[NBYTES + 4096:], pool[:NBYTES]))
    for i in range(pairs):
        s = torch.empty(NBYTES, dtype=torch.uint8, device="cuda")
        r = torch.empty(NBYTES, dtype=torch.uint8, device="cuda")
        sets.append((f"separate{i}", s, r))
    for i, (_, s, r) in enumerate(sets):
        dccl_amd.check(dccl_amd.synth_fill(s.data_ptr(), 7, n, 0, 0xDCC1, 2 * i, st), "synth")
        dccl_amd.check(dccl_amd.synth_fill(r.data_ptr(), 7, n, 0, 0xDCC1, 2 * i + 1, st), "synth")
    torch.cuda.synchronize()
    order = []
    for name, s, r in sets:
        for _ in range(launches):
            dccl_amd.check(dccl_amd.local_reduce(s.data_ptr(), r.data_ptr(), 7, n, 0, st), "combine")
            order.append({"set": name, "send": s.data_ptr(), "recv": r.data_ptr()})
    torch.cuda.synchronize()
    print(json.dumps({"order": order}), flush=True)


def _rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def parse(outdir: str, dst: str) -> None:
    passes = []
    for pdir in sorted(glob.glob(os.path.join(outdir, "p*"))):
        ktr = glob.glob(os.path.join(pdir, "**", "*kernel_trace.csv"), recursive=True)
        ctr = glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True)
        logs = glob.glob(os.path.join(pdir, "*.log"))
        if not ktr or not ctr:
            continue
        order = None
        for lg in logs:
            for line in open(lg):
                if line.startswith('{"order"'):
                    order = json.loads(line)["order"]
        dur = {}
        for row in _rows(ktr[0]):
            if KERNEL in row.get("Kernel_Name", ""):
                dur[int(row["Dispatch_Id"])] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
        cnt = {}
        for row in _rows(ctr[0]):
            if KERNEL not in row.get("Kernel_Name", ""):
                continue
            d = int(row["Dispatch_Id"])
            cnt.setdefault(d, {}).setdefault(row["Counter_Name"], 0.0)
            cnt[d][row["Counter_Name"]] += float(row["Counter_Value"])
        ids = sorted(set(dur) & set(cnt))
        if order is not None and len(order) == len(ids):
            for k, d in enumerate(ids):
                cnt[d]["_set"] = order[k]["set"]
        per_set = {}
        for d in ids:
            s = cnt[d].get("_set", "?")
            e = per_set.setdefault(s, {"ms": [], "counters": {}})
            e["ms"].append(dur[d])
            for k, v in cnt[d].items():
                if not k.startswith("_"):
                    e["counters"].setdefault(k, []).append(v)
        summary = []
        for s, e in per_set.items():
            ms = statistics.median(e["ms"])
            row = {"set": s, "ms": round(ms, 4), "frac": round(3 * NBYTES / (ms * 1e-3) / 8e12, 4)}
            for k, v in e["counters"].items():
                row[k] = statistics.median(v)
            # derived: average EA read / write latency in cycles (LEVEL / requests)
            if "TCC_EA0_RDREQ_LEVEL" in row and row.get("TCC_EA0_RDREQ"):
                row["rd_latency_cyc"] = round(row["TCC_EA0_RDREQ_LEVEL"] / row["TCC_EA0_RDREQ"], 1)
            if "TCC_EA0_WRREQ_LEVEL" in row and row.get("TCC_EA0_WRREQ"):
                row["wr_latency_cyc"] = round(row["TCC_EA0_WRREQ_LEVEL"] / row["TCC_EA0_WRREQ"], 1)
            summary.append(row)
        summary.sort(key=lambda r: r["ms"])
        passes.append({"pass": os.path.basename(pdir), "sets": summary})
    out = {"kernel": KERNEL, "bytes_per_operand": NBYTES, "passes": passes}
    txt = json.dumps(out, indent=1)
    if dst:
        with open(dst, "w") as f:
            f.write(txt)
    print(txt)


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--pairs", type=int, default=8)
    p.add_argument("--launches", type=int, default=3)
    p.add_argument("--parse", default="")
    p.add_argument("--out", default="")
    a = p.parse_args()
    if a.parse:
        parse(a.parse, a.out)
    else:
        run(a.pairs, a.launches)
