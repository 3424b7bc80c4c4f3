#!/usr/bin/env python3
"""Secondary measurements of the combine on one MI355X (BASELINE.json configs C2-C4 and §8(f)).

  c3     every op x {fp16, bf16, fp32, int32, int64} (+ the other dtypes) at 1 GiB per operand
  c4     size sweep 4 KiB - 4 GiB, fp32 Sum, GiB/s vs the HBM roofline; points whose working set
         (send + recv) fits the 256 MiB Infinity Cache are labelled "mall"
  c2     256 MiB fp32 Sum
  kway   dccl_local_reduce_multi, k = 1..8 sends at 256 MiB per operand: (k+2)N bytes
  host   host-resident operands (pinned and pageable): H2D + combine + D2H rate

All device timings are HIP events on the launch stream around back-to-back launches
(median of rounds); operands rotate over enough buffer sets that each launch reads cold data
when the working set is below 512 MiB.  Writes one JSON document (--out) and prints a summary.

    python tools/bench_suite.py [--parts c3,c4,c2,kway,host] [--out file.json]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccl_amd  # noqa: E402

PEAK = 8000.0  # GB/s
MALL = 256 << 20
NAMES = {0: "int8", 1: "uint8", 2: "int32", 3: "uint32", 4: "int64", 5: "uint64", 6: "float16",
         7: "float32", 8: "float64", 9: "bfloat16"}
OPS = {0: "sum", 1: "prod", 2: "max", 3: "min"}


def fill(nbytes, dt, op, buffer_id):
    """Device-generated synthetic operand (include/dccl/dccl_synth.h)."""
    t = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    n = nbytes // dccl_amd.size_of_type(dt)
    dccl_amd.check(dccl_amd.synth_fill(t.data_ptr(), dt, n, op, 0xDCC1, buffer_id,
                                       torch.cuda.current_stream().cuda_stream), "synth_fill")
    return t


def time_launches(fns, rounds=7, min_ms=20.0):
    """Median per-launch ms of cycling through fns back to back."""
    st = torch.cuda.current_stream()
    for f in fns:
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    fns[0]()
    e1.record(st)
    e1.synchronize()
    one = max(e0.elapsed_time(e1), 1e-3)
    reps = max(len(fns), int(min_ms / one) // len(fns) * len(fns))
    res = []
    for _ in range(rounds):
        e0.record(st)
        for i in range(reps):
            fns[i % len(fns)]()
        e1.record(st)
        e1.synchronize()
        res.append(e0.elapsed_time(e1) / reps)
    return statistics.median(res), min(res)


def pooled(nbytes, dt, op, seed):
    """send/recv carved from one allocation (recv, then send 4 KiB past it): bench.py's layout."""
    pool = torch.empty(2 * nbytes + 4096, dtype=torch.uint8, device="cuda")
    pool[:nbytes].copy_(fill(nbytes, dt, op, seed))
    pool[nbytes + 4096:].copy_(fill(nbytes, dt, op, seed + 1))
    return pool[nbytes + 4096:], pool[:nbytes]


def c3(results, mib=1024):
    st = torch.cuda.current_stream().cuda_stream
    nbytes = mib << 20
    rows = []
    for dt in [7, 6, 9, 2, 4, 0, 1, 3, 5, 8]:
        n = nbytes // dccl_amd.size_of_type(dt)
        for op in range(4):
            s, r = pooled(nbytes, dt, op, 1)
            fn = lambda: dccl_amd.check(dccl_amd.local_reduce(s.data_ptr(), r.data_ptr(), dt, n, op, st))
            med, mn = time_launches([fn], rounds=5)
            gbs = 3 * nbytes / (med * 1e-3) / 1e9
            rows.append({"dtype": NAMES[dt], "op": OPS[op], "ms": round(med, 4), "gb_s": round(gbs, 1),
                         "gib_s_traffic": round(3 * nbytes / (med * 1e-3) / 2**30, 1), "frac": round(gbs / PEAK, 4)})
            del s, r
        print("c3", NAMES[dt], [x["gb_s"] for x in rows[-4:]], flush=True)
    results["c3"] = {"bytes_per_operand": nbytes, "layout": "pooled (bench.py)", "rows": rows}


def c4(results):
    st = torch.cuda.current_stream().cuda_stream
    rows = []
    for lg in range(12, 33):
        nbytes = 1 << lg
        n = nbytes // 4
        sets = max(1, min(64, (512 << 20) // (2 * nbytes)))  # rotate so launches read cold lines
        if nbytes >= 1 << 32:
            sets = 1
        row = {"bytes_per_operand": nbytes, "buffer_sets": sets, "regime": "mall" if 2 * nbytes * sets <= MALL else "hbm"}
        # bench.py's pooled pair first (the headline layout), then separately allocated operands
        for layout in ("pooled", "separate"):
            if layout == "pooled":
                bufs = [pooled(nbytes, 7, 0, 2 * i) for i in range(sets)]
            else:
                bufs = [(fill(nbytes, 7, 0, 2 * i), fill(nbytes, 7, 0, 2 * i + 1)) for i in range(sets)]
            fns = [lambda s=s, r=r: dccl_amd.local_reduce(s.data_ptr(), r.data_ptr(), 7, n, 0, st) for s, r in bufs]
            med, mn = time_launches(fns)
            gbs = 3 * nbytes / (med * 1e-3) / 1e9
            key = "" if layout == "pooled" else "separate_"
            row.update({f"{key}ms": round(med, 5), f"{key}gb_s": round(gbs, 1), f"{key}frac": round(gbs / PEAK, 4)})
            if layout == "pooled":
                row["gib_s_traffic"] = round(3 * nbytes / (med * 1e-3) / 2**30, 1)
            del bufs, fns
            torch.cuda.empty_cache()
        rows.append(row)
        print("c4", nbytes, row["gb_s"], row["separate_gb_s"], row["regime"], flush=True)
    results["c4"] = rows


def c4_graph(results):
    """The small end of the sweep with launch overhead removed: 50 back-to-back combines captured in
    one HIP graph and replayed (torch.cuda.graph), so the per-combine time is the kernel's own."""
    rows = []
    for lg in range(12, 25):
        nbytes = 1 << lg
        n = nbytes // 4
        s, r = fill(nbytes, 7, 0, 1), fill(nbytes, 7, 0, 2)
        st = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=st):
            for _ in range(50):
                dccl_amd.local_reduce(s.data_ptr(), r.data_ptr(), 7, n, 0, st.cuda_stream)
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 50)
        med = statistics.median(ts)
        rows.append({"bytes_per_operand": nbytes, "us_per_combine": round(med * 1e3, 3),
                     "gb_s": round(3 * nbytes / (med * 1e-3) / 1e9, 1), "regime": "mall (L2/MALL-resident)"})
        print("c4_graph", rows[-1], flush=True)
    results["c4_graph"] = rows


def c2(results):
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 256 << 20
    n = nbytes // 4
    res = {"bytes_per_operand": nbytes, "note": "2 buffer sets rotated (1 GiB working set); pooled = bench.py's "
                                                 "layout, separate = separately allocated operands"}
    for layout in ("pooled", "separate"):
        sets = [pooled(nbytes, 7, 0, 2 * i) if layout == "pooled" else (fill(nbytes, 7, 0, 2 * i + 1),
                                                                        fill(nbytes, 7, 0, 2 * i + 2))
                for i in range(2)]
        fns = [lambda s=s, r=r: dccl_amd.local_reduce(s.data_ptr(), r.data_ptr(), 7, n, 0, st) for s, r in sets]
        med, mn = time_launches(fns)
        gbs = 3 * nbytes / (med * 1e-3) / 1e9
        key = "" if layout == "pooled" else "separate_"
        res.update({f"{key}ms": round(med, 4), f"{key}gb_s": round(gbs, 1), f"{key}frac": round(gbs / PEAK, 4)})
        del sets, fns
        torch.cuda.empty_cache()
    results["c2"] = res
    print("c2", results["c2"], flush=True)


def kway(results, mib=256):
    """k-way combine, k = 1..8: separately allocated operands, and the nine operands carved from one
    allocation with a 4 KiB x (j+1) stagger between operand j and j+1 (bench.py's pooled layout
    generalised, as tools/tune_multi.py's "staggered")."""
    st = torch.cuda.current_stream().cuda_stream
    nbytes = mib << 20
    n = nbytes // 4
    out = {"bytes_per_operand": nbytes}
    for layout in ("separate", "staggered"):
        if layout == "separate":
            keep = [fill(nbytes, 7, 0, 10 + k) for k in range(8)] + [fill(nbytes, 7, 0, 99)]
            ptrs_all = [x.data_ptr() for x in keep]
        else:
            pool = torch.empty(9 * nbytes + 4096 * 45, dtype=torch.uint8, device="cuda")
            keep, ptrs_all, off = [pool], [], 0
            for j in range(9):
                ptrs_all.append(pool.data_ptr() + off)
                dccl_amd.check(dccl_amd.synth_fill(ptrs_all[-1], 7, n, 0, 0xDCC1, 10 + j, st), "synth")
                off += nbytes + 4096 * (j + 1)
        sends, r = ptrs_all[:8], ptrs_all[8]
        rows = []
        for k in range(1, 9):
            ptrs = sends[:k]
            fn = lambda ptrs=ptrs: dccl_amd.local_reduce_multi(ptrs, r, 7, n, 0, st)
            med, _ = time_launches([fn])
            seq = lambda ptrs=ptrs: [dccl_amd.local_reduce(p, r, 7, n, 0, st) for p in ptrs]
            med_seq, _ = time_launches([seq])
            gbs = (k + 2) * nbytes / (med * 1e-3) / 1e9
            rows.append({"k": k, "ms": round(med, 4), "gb_s": round(gbs, 1), "frac": round(gbs / PEAK, 4),
                         "ms_k_single_launches": round(med_seq, 4), "speedup": round(med_seq / med, 2)})
            print("kway", layout, rows[-1], flush=True)
        out["rows" if layout == "separate" else "staggered_rows"] = rows
        del keep
        torch.cuda.empty_cache()
    results["kway"] = out


def host(results):
    import numpy as np
    rows = []
    for nbytes in (4 << 10, 64 << 10, 256 << 10, 1 << 20, 16 << 20, 256 << 20, 1 << 30):
        n = nbytes // 4
        for pinned in (True, False):
            if pinned:
                s = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
                r = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
                ps, pr = s.data_ptr(), r.data_ptr()
            else:
                s = np.ones(n, np.float32)
                r = np.zeros(n, np.float32)
                ps, pr = s.ctypes.data, r.ctypes.data
            dccl_amd.check(dccl_amd.local_reduce_host(ps, pr, 7, n, 0))
            reps, t0 = 0, time.perf_counter()
            while reps < 5 or time.perf_counter() - t0 < 0.3:
                dccl_amd.check(dccl_amd.local_reduce_host(ps, pr, 7, n, 0))
                reps += 1
            t = (time.perf_counter() - t0) / reps
            rows.append({"bytes_per_operand": nbytes, "pinned": pinned, "ms": round(t * 1e3, 3),
                         "payload_gib_s": round(nbytes / t / 2**30, 2)})
            print("host", rows[-1], flush=True)
    results["host_staged"] = {"zero_copy_max": os.environ.get("DCCL_HOST_ZEROCOPY_MAX", "default (unlimited)"),
                              "copy_threads": os.environ.get("DCCL_HOST_COPY_THREADS", "default (4)"),
                              "rows": rows}


def c1(results):
    """BASELINE C1 through the C++ API: dccl_cli all_reduce fp32 count 1024, 4 ranks (threads),
    1000 timed repeats after 10 warm-ups (scratchpad allocation and registration happen in the first call),
    host buffers and device buffers; plus a 64 MiB all_reduce on device buffers.  The known answer after
    1,010 all-reduces is still +inf (0x7f800000), as after the reference's 1,000."""
    import subprocess
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dccl_amd", "bin", "dccl_cli")
    rows = []
    for args in (["-c", "1024", "-r", "1000", "-w", "10", "-g", "-1"], ["-c", "1024", "-r", "1000", "-w", "10", "-g", "0"],
                 ["-c", str(16 << 20), "-r", "20", "-w", "2", "-g", "0"]):
        p = subprocess.run([cli, "-a", "all_reduce", "-t", "float32", "-n", "4", *args], capture_output=True,
                           text=True, timeout=600)
        ranks = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
        rows.append({"args": " ".join(args), "rc": p.returncode,
                     "us_per_call_max": max(r["us_per_call"] for r in ranks) if ranks else None,
                     "first": ranks[0]["first"] if ranks else None})
        print("c1", rows[-1], flush=True)
    results["c1"] = rows


def misaligned(results, mib=1024):
    """Operands off their 128-B lines (vector kernel), off the 16-B phase of each other (shifted vector
    kernel), a send off element alignment (shifted kernel, byte phase) or a recv off element alignment
    (reduce_unaligned_kernel), fp32 Sum, 1 GiB."""
    st = torch.cuda.current_stream().cuda_stream
    nbytes = mib << 20
    n = nbytes // 4 - 4
    s = fill(nbytes, 7, 0, 1)
    r = fill(nbytes, 7, 0, 2)
    rows = []
    for soff, roff, what in ((0, 0, "aligned (vector path)"),
                             (16, 0, "same 16-B phase, send off its lines (vector, send cached)"),
                             (0, 16, "same 16-B phase, recv off its lines (vector, recv realigned by the head)"),
                             (4, 0, "4-B phase mismatch (shifted vector kernel)"),
                             (8, 4, "8/4-B offsets (shifted vector kernel, recv realigned)"),
                             (1, 0, "send at a byte offset, recv aligned (shifted vector kernel, byte phase)"),
                             (3, 0, "send at a byte offset, recv aligned (shifted vector kernel, byte phase)"),
                             (1, 1, "byte offsets, recv element-misaligned (reduce_unaligned_kernel: 16-B accesses at the displaced addresses)"),
                             (0, 2, "recv element-misaligned (reduce_unaligned_kernel: 16-B accesses at the displaced addresses)")):
        fn = lambda soff=soff, roff=roff: dccl_amd.local_reduce(s.data_ptr() + soff, r.data_ptr() + roff, 7, n, 0, st)
        med, _ = time_launches([fn], rounds=5)
        gbs = 3 * n * 4 / (med * 1e-3) / 1e9
        rows.append({"send_offset": soff, "recv_offset": roff, "path": what, "ms": round(med, 4),
                     "gb_s": round(gbs, 1), "frac": round(gbs / PEAK, 4)})
        print("misaligned", rows[-1], flush=True)
    results["misaligned"] = rows


def phased(results, mib=256):
    """k-way and chain combines with sources off the destination's 16-B phase (phased kernels) beside
    the same launch with every operand in phase, fp32 Sum, separately allocated operands."""
    st = torch.cuda.current_stream().cuda_stream
    nbytes = mib << 20
    n = nbytes // 4 - 64
    keep = [fill(nbytes, 7, 0, 20 + k) for k in range(9)]
    base = [x.data_ptr() for x in keep]
    rows = []
    for k in (1, 2, 4, 7):
        for what, offs in (("in phase", [0] * k), ("all sources +4 B", [4] * k),
                           ("alternate sources +8 B", [8 * (j % 2) for j in range(k)]),
                           ("sources +16 B (cached loads)", [16] * k), ("sources +20 B", [20] * k)):
            ptrs = [base[j] + offs[j] for j in range(k)]
            r = base[8]
            fm = lambda ptrs=ptrs: dccl_amd.local_reduce_multi(ptrs, r, 7, n, 0, st)
            fc = lambda ptrs=ptrs: dccl_amd.local_reduce_chain(ptrs, r, r, 7, n, 0, st)
            row = {"k": k, "sources": what}
            for name, fn in (("multi", fm), ("chain", fc)):
                med, _ = time_launches([fn], rounds=5)
                gbs = (k + 2) * n * 4 / (med * 1e-3) / 1e9
                row[name] = {"ms": round(med, 4), "gb_s": round(gbs, 1), "frac": round(gbs / PEAK, 4)}
            rows.append(row)
            print("phased", row, flush=True)
    results["phased"] = {"bytes_per_operand": n * 4, "rows": rows}
    del keep
    torch.cuda.empty_cache()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--parts", default="c3,c4,c2,kway,host,c1,misaligned")
    p.add_argument("--out", default="")
    a = p.parse_args()
    results = {"device": torch.cuda.get_device_name(0), "peak_gb_s": PEAK}
    for part in a.parts.split(","):
        {"c3": c3, "c4": c4, "c2": c2, "kway": kway, "host": host, "c1": c1, "misaligned": misaligned,
         "c4_graph": c4_graph, "phased": phased}[part](results)
        if a.out:
            with open(a.out, "w") as f:
                json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
