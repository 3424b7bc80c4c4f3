#!/usr/bin/env python3
"""Issue-side counters per kernel from a rocprofv3 --pmc run: per kernel name, the mean over
its dispatches of SALU and VALU instructions per wave and of the issue-stall share SQ_WAIT_INST_ANY /
SQ_WAVE_CYCLES.  Collect with, e.g.,

    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VALU \\
        SQ_BUSY_CYCLES -d OUT -o p --output-format csv -- python tools/ab_cases.py OLD.so NEW.so \\
        --cases multi4_dst+2,multi8_dst+2 --rounds 1 --launches 3
    python tools/issue_counters.py OUT [--match reduce_]
"""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="reduce_")
    a = ap.parse_args()
    per = collections.defaultdict(dict)  # (kernel, dispatch) -> counter -> value
    for path in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                if a.match not in name:
                    continue
                key = (name, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                per[key][row["Counter_Name"]] = per[key].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    agg = collections.defaultdict(list)
    for (name, _), c in per.items():
        waves = c.get("SQ_WAVES", 0.0)
        cycles = c.get("SQ_WAVE_CYCLES", 0.0)
        if waves <= 0:
            continue
        agg[name].append({"salu_per_wave": c.get("SQ_INSTS_SALU", 0.0) / waves,
                          "valu_per_wave": c.get("SQ_INSTS_VALU", 0.0) / waves,
                          "wait_inst_any_frac": c.get("SQ_WAIT_INST_ANY", 0.0) / cycles if cycles else None,
                          "waves": waves})
    out = {}
    for name, rows in sorted(agg.items()):
        mean = lambda k: round(sum(r[k] for r in rows if r[k] is not None) / len(rows), 4)  # noqa: E731
        out[name] = {"dispatches": len(rows), "salu_per_wave": mean("salu_per_wave"),
                     "valu_per_wave": mean("valu_per_wave"), "wait_inst_any_frac": mean("wait_inst_any_frac"),
                     "waves": mean("waves")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
