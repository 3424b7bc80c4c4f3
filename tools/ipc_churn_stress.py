#!/usr/bin/env python3
"""Churn stress of the IPC transport's peer-mapping cache: tests/test_direct.py's
re-allocation rank body (all-gathers over buffers freed back to the driver and re-allocated every round, every
round's data checked) run `--runs` times at W ranks on the box's one GPU.  One JSON line on stdout: runs, runs
with a wrong slice or an error, and the first few reports.

    python tools/ipc_churn_stress.py [--runs 20] [--world 2] [--mib 1] [--rounds 140] [--grow] [--two] [--register]

With --register every round registers its buffers and deregisters them before the free (tracked only since
round 5: peers read the scratch either way); a wrong slice is reported with whether its exporter's input sat at
the same address as the round before (`va_reused`).
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from tests.test_direct import _ipc_realloc_rank
    p = argparse.ArgumentParser()
    p.add_argument("--runs", type=int, default=20)
    p.add_argument("--world", type=int, default=2)
    p.add_argument("--mib", type=int, default=1)
    p.add_argument("--rounds", type=int, default=140)
    p.add_argument("--grow", action="store_true")
    p.add_argument("--two", action="store_true")
    p.add_argument("--register", action="store_true")
    p.add_argument("--trace", default="", help="directory: DCCL_IPC_DEBUG=1, every rank's stderr kept per run "
                                               "(runs without a wrong slice are deleted)")
    a = p.parse_args()
    # a rank that fails leaves its peers at a barrier: let them give up well before a pool's silence limit
    os.environ.setdefault("DCCL_IPC_TIMEOUT_S", "60")
    ctx = mp.get_context("spawn")
    failed, reports = 0, []
    import shutil
    for run in range(a.runs):
        run_dir = ""
        if a.trace:
            run_dir = os.path.join(a.trace, f"run{run}")
            os.makedirs(run_dir, exist_ok=True)
            os.environ.update({"DCCL_IPC_DEBUG": "1", "DCCL_STRESS_LOG_DIR": run_dir})
        q = ctx.Queue()
        tag = "stress_" + uuid.uuid4().hex[:10]
        ps = [ctx.Process(target=_ipc_realloc_rank,
                          args=(r, a.world, a.mib << 20, a.rounds, a.grow, tag, q, a.two, False, a.register))
              for r in range(a.world)]
        for x in ps:
            x.start()
        bad, results = [], {}
        for _ in range(a.world):
            r, res, err = q.get(timeout=150)
            if err is not None:
                bad.append((r, err))
            else:
                results[r] = res
        for r, res in results.items():
            if res[0] or res[1] != 0:
                rep = []
                for k, peer, what in res[0][:4]:
                    pp = results.get(peer, (None, None, None, []))[3] if peer >= 0 else []
                    reused = bool(k > 0 and len(pp) > k and pp[k] == pp[k - 1])
                    rep.append((k, peer, what, {"va_reused": reused}))
                bad.append((r, rep, res[1], {k: v for k, v in res[2].items() if v}))
        for x in ps:
            x.join(60)
            if x.is_alive():
                x.kill()
        if bad:
            failed += 1
            reports.append({"run": run, "bad": bad})
        elif run_dir:
            shutil.rmtree(run_dir, ignore_errors=True)
        print(f"run {run}: {'FAILED ' + repr(bad) if bad else 'ok'}", file=sys.stderr, flush=True)
    print(json.dumps({"runs": a.runs, "world": a.world, "mib": a.mib, "rounds": a.rounds, "grow": a.grow,
                      "two": a.two, "register": a.register, "failed_runs": failed, "reports": reports[:5]}, default=str), flush=True)


if __name__ == "__main__":
    main()
