#!/usr/bin/env python3
"""Split a `rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py` run into the headline's own
dispatches: the kernel trace holds every launch of the bench (C3, C4, ring-step, other-layout, host-staged ... legs
use the same kernel symbol), so the headline is identified as the first warmup + steps launches, in time order,
of `reduce_vec_kernel<float, 0, ...>` at the headline's grid (1 GiB fp32 per operand: 2^20 one-wave blocks).
Prints one JSON object: the per-grid split of that symbol and the headline's average duration over the timed
steps, against 8 TB/s.

    python tools/rocprof_headline.py DIR [--mib 1024] [--warmup 5] [--steps 100]
"""
import argparse
import csv
import glob
import json
import os
import statistics

PEAK = 8e12


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--mib", type=int, default=1024)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--steps", type=int, default=100)
    a = p.parse_args()
    traces = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for t in traces:
        with open(t) as f:
            rows += list(csv.DictReader(f))
    sym = "reduce_vec_kernel<float, 0, dccl_amd::VecCfg<64, 1, 7, false"
    mine = [r for r in rows if sym in r["Kernel_Name"]]
    by_grid = {}
    for r in mine:
        g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)))
        by_grid.setdefault(g, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    split = [{"grid_x_threads": g, "calls": len(v), "avg_ns": round(statistics.mean(v), 1), "min_ns": min(v),
              "max_ns": max(v)} for g, v in sorted(by_grid.items(), key=lambda kv: -len(kv[1]))]
    nbytes = a.mib << 20
    grid = nbytes // 16 * 1  # one 16-B vector per lane: threads = vectors
    head = sorted((r for r in mine if int(r.get("Grid_Size_X", r.get("Grid_Size", 0))) == grid),
                  key=lambda r: int(r["Start_Timestamp"]))[: a.warmup + a.steps]
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in head]
    timed = durs[a.warmup:]
    out = {"source": f"rocprofv3 --kernel-trace --stats kernel trace under {a.dir}", "kernel_symbol_prefix": sym,
           "split": split,
           "headline_timed": {"what": f"the first {a.warmup + a.steps} launches of the {grid}-thread grid in time order: "
                                      f"the bench's {a.warmup} warmup + {a.steps} timed headline steps",
                              "launches": len(durs), "avg_ns_timed": round(statistics.mean(timed), 1) if timed else None,
                              "min_ns": min(timed) if timed else None, "max_ns": max(timed) if timed else None,
                              "frac_of_8TBps": round(3 * nbytes / (statistics.mean(timed) * 1e-9) / PEAK, 4)
                              if timed else None}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
