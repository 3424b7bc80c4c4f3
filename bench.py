#!/usr/bin/env python3
"""bench.py — device-resident DCCL local combine on MI355X (BASELINE.json metric).

One "step" = one pass of the combine ``recv[i] = recv[i] + send[i]`` over 1 GiB fp32
operands resident in HBM (BASELINE.json metric: ncclSum fp32, 1 GiB).  Each rank owns its
own 1 GiB shard pair (the combine is element-wise: no data-path collective), so the
aggregate is weak scaling.  Operands are carved from one HBM allocation (recv, then send 4 KiB
past its end); the separately allocated layout is timed too and reported as `other_layout`
(separate 1 GiB allocations land in one of two physical placement modes).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mib 1024] [--dtype float32] [--op sum]

Rank 0 prints ONE JSON line:
  value            whole-job HBM traffic rate, GiB/s = N * 3 * bytes_per_operand / t_step
                   (3 = read send + read recv + write recv; BASELINE.md §2 roofline basis)
  roofline         dominant kernel (the combine): algorithmic bytes per launch / average
                   launch duration (HIP events around the timed region on the launch stream,
                   divided by the steps), vs 8.0 TB/s HBM peak;
                   `traffic` = HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
                   run during the bench (N=1) over the same kernel and layout (measured_traffic)
  cpu_baseline     the build's C restatement of the reference loop (oracle/host_reduce.c, Release flags)
                   on the headline's own 1 GiB operands in host memory: 1 core and every core this
                   process may use (rank 0, N=1); nproc and the CPU model are stated
Extra keys: c3 (BASELINE C3: 4 ops x fp16/bf16/fp32/int32/int64 at 1 GiB, timed and sample-verified) and
c4 (BASELINE C4: fp32 Sum size sweep 4 KiB - 4 GiB, 21 points, operand sets rotated below a 512 MiB working
set, per-launch duration eager from Python and from a C++ loop, and graph-replayed, fraction of HBM peak), rank 0 at N=1; payload_gib_s, host_staged (H2D+combine+D2H rate for host-resident operands,
rank 0, N=1), allgather (RCCL all-gather of the shards over xGMI, N>1, reported separately),
c5 (BASELINE config C5 on every run: --c5-gib GiB per operand sharded over the N GPUs, strong scaling,
combine time and, N>1, the RCCL all-gather of the reduced shards),
dccl_allreduce (N>1: the namespace-dccl ncclAllReduce over RCCL (the ring step loop, and the grouped form:
one RCCL group per phase and one chain combine) and over the direct IPC peer-read transport (inputs through
the communicator's scratch), checked against each other and RCCL's own all_reduce, timed beside it, plus
the namespace-dccl all_gather of each transport against RCCL's all_gather (`dccl_allgather`), and the
direct all_gather at C5's size beside RCCL's (`c5_allgather`);
in a child process per rank, so a fault or hang there cannot take the bench line with it).
Progress goes to stderr, one line per phase.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# The HIP library is loaded by _native() in the rank processes only: with --gpus N and no WORLD_SIZE the
# parent spawns the N ranks before anything touches the GPU (launch_ranks), and never loads it itself.
dccl_amd = None


def _native():
    """Load the dccl_amd package (fails loudly when the HIP library is missing: there is no CPU path)."""
    global dccl_amd
    if dccl_amd is None:
        import dccl_amd as m
        dccl_amd = m
    return dccl_amd


# ncclDataType_t / ncclRedOp_t names (include/dccl/dccl.hpp; the same tables as dccl_amd.DTYPE_NAMES /
# OP_NAMES, checked by tests/test_bench_launcher.py), kept here so that parsing needs no native library
DTYPE_NAMES = {"int8": 0, "uint8": 1, "int32": 2, "uint32": 3, "int64": 4, "uint64": 5,
               "float16": 6, "float32": 7, "float64": 8, "bfloat16": 9}
OP_NAMES = {"sum": 0, "prod": 1, "max": 2, "min": 3}

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
GIB = float(1 << 30)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="ranks, one process per GPU: without WORLD_SIZE in the environment bench.py spawns them "
                        "itself; under torch.distributed.run it must equal WORLD_SIZE")
    p.add_argument("--rank-timeout", type=float, default=1800.0,
                   help="seconds the self-launching parent waits for its ranks before killing them")
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--mib", type=int, default=1024, help="MiB per operand per GPU (weak scaling)")
    p.add_argument("--total-gib", type=float, default=0.0,
                   help="BASELINE C5: one buffer of this many GiB per operand sharded over the GPUs (strong)")
    p.add_argument("--dtype", default="float32", choices=list(DTYPE_NAMES))
    p.add_argument("--op", default="sum", choices=["sum", "prod", "max", "min"])
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (rank 0, N=1)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-host-staged", action="store_true")
    p.add_argument("--c5-gib", type=float, default=16.0,
                   help="BASELINE C5 extra on every run: one buffer of this many GiB per operand sharded over "
                        "the N GPUs, combine + RCCL all-gather, reported as `c5` (0 disables)")
    p.add_argument("--no-pmc", action="store_true",
                   help="skip the rocprofv3 --pmc passes that measure roofline.traffic (N=1)")
    p.add_argument("--no-other-layout", action="store_true",
                   help="skip timing the other operand layout (profiling runs: one layout per kernel average)")
    p.add_argument("--no-configs", action="store_true",
                   help="skip the C3 (ops x dtypes, 1 GiB) and C4 (size sweep 4 KiB - 4 GiB) legs (rank 0, N=1)")
    p.add_argument("--layout", default="pooled", choices=["pooled", "separate"],
                   help="operand placement in HBM (see operand_pair); the other layout is also timed briefly")
    p.add_argument("--launcher-selftest", action="store_true",
                   help="test aid: each rank joins a gloo group and rank 0 prints the world it saw (no GPU)")
    p.add_argument("--other-pairs", type=int, default=4,
                   help="separately allocated operand pairs timed for `other_layout` (median reported)")
    return p.parse_args(argv)


def synth_into(t: torch.Tensor, n: int, dt: int, op: int, buffer_id: int) -> None:
    """Counter-based synthetic operand written on the device (include/dccl/dccl_synth.h):
    uniform [-1,1) for Sum/Max/Min, [0.5,2) for Prod, integers full range; seed 0xDCC1."""
    dccl_amd.check(dccl_amd.synth_fill(t.data_ptr(), dt, n, op, SEED, buffer_id,
                                       torch.cuda.current_stream().cuda_stream), "synth_fill")


SEED = 0xDCC1
PAIR_GAP = 4096  # bytes between the end of recv and the start of send in the pooled layout


def operand_pair(n: int, dt: int, op: int, buffer_id: int, device, layout: str, keep: list | None = None):
    """(send, recv) synthetic operands.  "pooled": both carved from ONE HBM allocation, recv first
    and send PAIR_GAP bytes past its end; "separate": two allocations (DCCL's own shape: scratchpad
    + user chunk).  Separately allocated 1 GiB operands land in one of two physical placement modes
    (0.476 vs 0.508 ms on MI355X); the pooled layout is consistently in the fast one."""
    nbytes = n * dccl_amd.size_of_type(dt)
    tdt = dccl_amd.TORCH_DTYPES[dt]
    if layout == "separate":
        send = torch.empty(nbytes, dtype=torch.uint8, device=device).view(tdt)
        recv = torch.empty(nbytes, dtype=torch.uint8, device=device).view(tdt)
    else:
        pool = torch.empty(2 * nbytes + PAIR_GAP, dtype=torch.uint8, device=device)
        recv = pool[:nbytes].view(tdt)
        send = pool[nbytes + PAIR_GAP:].view(tdt)
        if keep is not None:  # the caller keeps the allocation for later legs (C3)
            keep.append(pool)
    synth_into(send, n, dt, op, buffer_id)
    synth_into(recv, n, dt, op, buffer_id + 1)
    return send, recv


def verify_sample(recv: torch.Tensor, n: int, dt: int, op: int, send_id: int, recv_id: int, applications: int,
                  width: int = 1 << 16) -> bool | None:
    """Check sampled slices of a combined operand: the first and last `width` elements and four seeded
    random slices.  Their inputs are regenerated on the device (dccl_synth_fill_range, the same counter-based
    values at the same indices), the combine is applied `applications` times in order by plain torch ops
    (IEEE arithmetic and compare-select, as the reference's do_host_reduce applies them,
    internal_common.hpp:546-549), and the result must match the HIP kernel's bit for bit.
    None when torch lacks the dtype's ops."""
    import random
    tdt = dccl_amd.TORCH_DTYPES.get(dt)
    if tdt is None or dt in (3, 5):
        return None
    ops = {0: lambda r, s: r + s, 1: lambda r, s: r * s,
           2: lambda r, s: torch.where(r < s, s, r), 3: lambda r, s: torch.where(r > s, s, r)}
    width = min(width, n)
    rnd = random.Random(0xDCC1 + recv_id)
    starts = sorted({0, n - width, *(rnd.randrange(0, n - width + 1) for _ in range(4))})
    st = torch.cuda.current_stream(recv.device).cuda_stream
    for a0 in starts:
        sv = torch.empty(width, dtype=tdt, device=recv.device)
        want = torch.empty(width, dtype=tdt, device=recv.device)
        dccl_amd.check(dccl_amd.synth_fill_range(sv.data_ptr(), dt, width, op, SEED, send_id, a0, st), "synth")
        dccl_amd.check(dccl_amd.synth_fill_range(want.data_ptr(), dt, width, op, SEED, recv_id, a0, st), "synth")
        for _ in range(applications):
            want = ops[op](want, sv)
        got = recv[a0:a0 + width]
        if got.view(torch.uint8).cpu().numpy().tobytes() != want.view(torch.uint8).cpu().numpy().tobytes():
            return False
    return True


def time_kernel(ps: int, pr: int, dt: int, n: int, op: int, stream, steps: int) -> float:
    """Average launch duration (ms) over `steps` back-to-back launches, HIP events on `stream`."""
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        dccl_amd.check(dccl_amd.local_reduce(ps, pr, dt, n, op, stream.cuda_stream))
    ev0.record(stream)
    for _ in range(steps):
        dccl_amd.check(dccl_amd.local_reduce(ps, pr, dt, n, op, stream.cuda_stream))
    ev1.record(stream)
    ev1.synchronize()
    return ev0.elapsed_time(ev1) / steps


_BENCHFLAGS_CHILD = r"""
import json, sys, time
sys.path.insert(0, sys.argv[1])
import oracle
path, n, budget = sys.argv[2], int(sys.argv[3]), float(sys.argv[4])
nat = oracle.restatement_benchflags(path)
s = oracle.synth(n, 7, 0, 0xDCC1, 0); r = oracle.synth(n, 7, 0, 0xDCC1, 1)
nat.oracle_host_reduce(s.ctypes.data, r.ctypes.data, n, 7, 0)
reps, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < budget or reps < 2:
    nat.oracle_host_reduce(s.ctypes.data, r.ctypes.data, n, 7, 0); reps += 1
print(json.dumps({"seconds_per_pass": (time.perf_counter() - t0) / reps, "passes": reps}))
"""


def benchflags_variant(budget_s: float, n: int) -> dict | None:
    """The restatement with the reference's Benchmark flags (-Ofast -march=native, CMakeLists.txt:26), a
    labelled 1-core variant, compiled at run time on THIS host so that -march=native means this host's CPU
    (the prebuilt -march=x86-64-v4 library is the fallback).  It runs in a child process: an instruction
    the CPU lacks ends the child, not the bench."""
    import subprocess
    import tempfile
    import oracle
    with tempfile.TemporaryDirectory(prefix="dccl_benchflags_") as d:
        path, flags = oracle.compile_benchflags(d), "-Ofast -march=native (compiled on this host at run time)"
        if path is None:
            path, flags = oracle.benchflags_fallback(), "-Ofast -march=x86-64-v4 (prebuilt; no compiler on this host)"
        if path is None:
            return None
        try:
            p = subprocess.run([sys.executable, "-c", _BENCHFLAGS_CHILD, ROOT, path, str(n), str(budget_s)],
                               capture_output=True, text=True, timeout=budget_s + 120)
            if p.returncode != 0:
                return {"error": f"child exited with {p.returncode}", "flags": flags}
            res = json.loads(p.stdout.strip().splitlines()[-1])
        except Exception as e:  # reported, never fatal
            return {"error": repr(e), "flags": flags}
    t = res["seconds_per_pass"]
    return {"value": round(3 * n * 4 / t / GIB, 2), "payload_gib_s": round(n * 4 / t / GIB, 2), "cores": 1,
            "passes": res["passes"], "flags": flags + " -mprefer-vector-width=512"}


def cgroup_cpu_quota() -> float | None:
    """CPUs granted by the cgroup v2 quota (cpu.max) of this process, None when unlimited or unreadable."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if quota == "max" else round(int(quota) / int(period), 2)
    except Exception:
        return None


def cpu_baseline(budget_s: float, nbytes: int) -> dict | None:
    """the build's C restatement of the reference loop (oracle/host_reduce.c, the combine
    of internal_common.hpp:496-586 with its head/pack/tail split) compiled with the reference's Release
    flags (-O3 -mprefer-vector-width=512, CMakeLists.txt:25), on the headline's own operands: the same
    counter-based fp32 values, 1 GiB per operand, in host memory.  Timed (i) on 1 core, as the reference
    runs its combine (one thread per rank), (ii) on all the cores this process is granted (`all_cores`: the
    cgroup CPU quota, 16 on the GPU box, or the affinity mask when there is no quota), and (iii) when the
    affinity mask is wider than the quota, on one thread per CPU of the mask (`affinity_threads`, throttled by
    the quota), the buffer split into 64-B aligned contiguous slices, one persistent thread each (ctypes drops
    the GIL)."""
    try:
        import oracle  # test infrastructure: the CPU baseline leg only
    except Exception:
        return None
    lib = oracle.restatement()
    fn = lambda s, r, n: lib.oracle_host_reduce(s, r, n, 7, 0)  # noqa: E731
    n = nbytes // 4
    affinity = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    granted = granted_cpus()

    def slices(nthr):
        per = (n // nthr) // 16 * 16
        return [(i * per, n if i == nthr - 1 else (i + 1) * per) for i in range(nthr)]

    s = oracle.aligned_empty(n, np.float32)
    r = oracle.aligned_empty(n, np.float32)

    def gen(b):  # the device generator's values, regenerated on the host in parallel slices
        for arr, bid in ((s, 0), (r, 1)):
            rc = lib.oracle_synth_fill(arr.ctypes.data + 4 * b[0], 7, b[1] - b[0], 0, SEED, bid, b[0])
            assert rc == 0

    with ThreadPoolExecutor(max_workers=min(affinity, 64)) as pool:
        list(pool.map(gen, slices(min(affinity, 64))))
    ps, pr = s.ctypes.data, r.ctypes.data
    fn(ps, pr, n)  # page in
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s * 0.35 or reps < 2:
        fn(ps, pr, n)
        reps += 1
    t1 = (time.perf_counter() - t0) / reps

    def threaded(nthr, budget):
        bounds = slices(nthr)

        def work(b):
            fn(ps + 4 * b[0], pr + 4 * b[0], b[1] - b[0])

        reps_mt = 0
        with ThreadPoolExecutor(max_workers=nthr) as pool:
            list(pool.map(work, bounds))  # warm the threads
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < budget or reps_mt < 2:
                list(pool.map(work, bounds))
                reps_mt += 1
            tmt = (time.perf_counter() - t0) / reps_mt
        return {"value": round(3 * nbytes / tmt / GIB, 2), "cores": nthr, "passes": reps_mt,
                "payload_gib_s": round(nbytes / tmt / GIB, 2), "ms_per_pass": round(tmt * 1e3, 2),
                "slices": "64-B aligned contiguous, one thread each"}

    every = threaded(granted, budget_s * 0.2)
    wide = threaded(affinity, budget_s * 0.15) if affinity > granted else None
    del s, r
    variant = benchflags_variant(budget_s * 0.3, n)
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {
        "value": round(3 * nbytes / t1 / GIB, 2), "unit": "GiB/s (HBM-traffic basis 3*N*4 B, fp32 Sum)",
        "cores": 1, "kind": "port",
        "sample": f"fp32 Sum, 1 GiB per operand in host memory (the headline's operands: splitmix64, seed 0xDCC1, "
                  f"64-B aligned), {reps} passes in {t1 * reps:.1f}s; oracle/host_reduce.c (restatement of "
                  f"internal_common.hpp:496-586) with the Release flags -O3 -mprefer-vector-width=512",
        "payload_gib_s": round(nbytes / t1 / GIB, 2),
        "ms_per_pass": round(t1 * 1e3, 2),
        "all_cores": every, "affinity_threads": wide,
        "affinity_cpus": affinity, "machine_cpus": os.cpu_count(), "cgroup_cpu_quota": quota,
        "cores_note": (f"all_cores = the {granted} CPUs this process is granted "
                       + (f"(cgroup quota {quota} CPUs of time); affinity_threads = one thread per CPU of the "
                          f"{affinity}-CPU affinity mask, throttled by that quota" if quota and affinity > granted
                          else "(its affinity mask; no narrower cgroup quota)")),
        "benchmark_flags_variant": variant,
        "cpu_model": cpu_model,
    }


def measured_traffic(nbytes: int, dt: int, op: int, launches: int = 5) -> dict:
    """roofline.traffic, measured in this run: two rocprofv3 --pmc passes (FETCH_SIZE, then WRITE_SIZE: they
    do not fit one pass on gfx950) over dccl_amd/bin/pmc_combine, which runs the same kernel on operands of
    the same size and layout.  Per launch, read = 2 x FETCH_SIZE (gfx950 reports half the bytes of 16-B-per-
    lane streaming reads) and write = WRITE_SIZE (exact for 16-B stores), both in KiB
    (MI355X_MICROARCH.md §HBM).  Any failure is reported, never fatal."""
    import glob
    import shutil
    import statistics
    import subprocess
    import tempfile
    if any(k.startswith("ROCPROF") for k in os.environ):
        return {"skipped": "bench.py itself runs under rocprofv3"}
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    binary = os.path.join(ROOT, "dccl_amd", "bin", "pmc_combine")
    if not (os.path.exists(prof) and os.path.exists(binary)):
        return {"error": "rocprofv3 or dccl_amd/bin/pmc_combine missing"}
    vals = {}
    with tempfile.TemporaryDirectory(prefix="dccl_pmc_") as d:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            cmd = ["timeout", "-s", "KILL", "90", prof, "--pmc", counter, "--output-format", "csv",
                   "-d", os.path.join(d, counter), "-o", "p", "--", binary, str(nbytes), str(launches), str(dt),
                   str(op)]
            try:
                p = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
            except subprocess.TimeoutExpired:
                return {"error": f"{counter} pass timed out"}
            if p.returncode != 0:
                return {"error": f"{counter} pass exited with {p.returncode}", "stderr": p.stderr[-300:]}
            rows = []
            for path in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
                with open(path) as f:
                    rows += [float(r["Counter_Value"]) for r in csv.DictReader(f)
                             if "reduce_vec_kernel" in r.get("Kernel_Name", "") and r["Counter_Name"] == counter]
            if len(rows) != launches:
                return {"error": f"{counter}: {len(rows)} dispatches found, {launches} expected"}
            vals[counter] = statistics.median(rows)
    read_b, write_b = 2 * vals["FETCH_SIZE"] * 1024, vals["WRITE_SIZE"] * 1024
    return {"hbm_bytes_per_launch": read_b + write_b, "read_bytes": read_b, "write_bytes": write_b,
            "over_algorithmic": round((read_b + write_b) / (3 * nbytes), 6), "launches": launches,
            "FETCH_SIZE_kb": vals["FETCH_SIZE"], "WRITE_SIZE_kb": vals["WRITE_SIZE"],
            "how": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) during this run over "
                   "dccl_amd/bin/pmc_combine (same kernel, operand size and pooled layout); "
                   "read = 2 x FETCH_SIZE x 1024 (gfx950 halving), write = WRITE_SIZE x 1024"}


HOST_SIZES = [4 << 10, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20, 1 << 30]
HOST_ROTATE_BYTES = 1 << 30  # per operand: operand pairs rotated over this much memory, so no call finds its operands
#                              in a cache (the L3 is 32 MiB per CCD, 512 MiB over a 2-socket EPYC 9575F host's 16 CCDs,
#                              which a 16-thread leg spread over both sockets can fill), as a chunk that just arrived
#                              by RDMA


def granted_cpus() -> int:
    """CPUs this process may use: the cgroup quota (16 on the GPU box) capped by the affinity mask."""
    affinity = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    return max(1, min(affinity, int(quota))) if quota else affinity


def _gpu_host_us(ps: int, pr: int, n: int, nsets: int, stride: int, dt: int, op: int, min_s: float) -> tuple:
    """Microseconds per dccl_local_reduce_host call (synchronous: staging, PCIe both ways, the combine), the
    operand pairs rotated as in the CPU legs; the loop is Python over the ctypes entry point (its own cost,
    well under a microsecond per call, is included)."""
    f = dccl_amd.lib.dccl_local_reduce_host
    for k in range(min(nsets, 3)):
        dccl_amd.check(f(ps + k * stride, pr + k * stride, dt, n, op), "dccl_local_reduce_host")
    reps, t0 = 0, time.perf_counter()
    while True:
        k = reps % nsets
        rc = f(ps + k * stride, pr + k * stride, dt, n, op)
        if rc:
            raise dccl_amd.DcclError(rc, "dccl_local_reduce_host")
        reps += 1
        if reps >= 3 and (reps & 7 == 0 or n >= 1 << 18):
            el = time.perf_counter() - t0
            if el >= min_s:
                return el / reps * 1e6, reps


def numa_nodes_of(addr: int) -> dict | None:
    """Pages per NUMA node of the mapping that holds `addr` (/proc/self/numa_maps), None when unreadable."""
    try:
        for line in open("/proc/self/numa_maps"):
            parts = line.split()
            start = int(parts[0], 16)
            if start <= addr and any(p.startswith("N") and "=" in p for p in parts):
                nodes = {p.split("=")[0]: int(p.split("=")[1]) for p in parts if p[0] == "N" and p[1:2].isdigit()}
                kb = next((int(p.split("=")[1]) for p in parts if p.startswith("kernelpagesize_kB=")), 4)
                if start + sum(nodes.values()) * kb * 1024 > addr:
                    return nodes
    except Exception:
        return None
    return None


def node_cpus() -> dict:
    """{NUMA node: CPUs of this process's affinity mask on it}, from /sys (empty when unreadable)."""
    allowed, out = os.sched_getaffinity(0), {}
    base = "/sys/devices/system/node"
    try:
        for d in sorted(os.listdir(base)):
            if not (d.startswith("node") and d[4:].isdigit()):
                continue
            cpus = set()
            for part in open(os.path.join(base, d, "cpulist")).read().strip().split(","):
                if part:
                    lo, _, hi = part.partition("-")
                    cpus.update(range(int(lo), int(hi or lo) + 1))
            if cpus & allowed:
                out[int(d[4:])] = sorted(cpus & allowed)
    except Exception:
        return {}
    return out


def host_crossover(dt: int = 7, op: int = 0, min_s: float = 0.25) -> dict:
    """Where the host-resident GPU path pays.  For each payload size 4 KiB - 1 GiB, on three
    kinds of host operands, on the SAME buffers: dccl_local_reduce_host (the product: H2D,
    combine, D2H) against the oracle restatement of the reference's loop do_host_reduce
    (internal_common.hpp:496-586, oracle/host_reduce.c, Release flags; timed in C by oracle/cpu_timing.c) on
    1 core, as the reference runs it (one thread per rank), and on every core this process is granted.
    Kinds: `registered` = ordinary malloc'ed memory page-locked in place by dccl_register_host_memory (DCCL's
    configuration: Derecho's RDMA buffers registered through dcclRegisterCacheMemory, dccl.cpp:503-549),
    `pinned` = hipHostMalloc memory (torch pin_memory), `pageable` = malloc'ed memory (bounced by the GPU path).
    The 1-core legs run on a CPU of the NUMA node that holds the buffer (`cpu1_us`, the CPU's best case: a rank
    thread placed by its memory) and on a CPU of another node (`cpu1_remote_us`): an unpinned thread lands on
    either, and the remote socket's rate is ~1.6x lower.
    Operand pairs rotate over HOST_ROTATE_BYTES so every call starts cold; `cpu1_hot_us` repeats one pair
    (cache-resident up to tens of MiB) as the CPU's best case.  Every size's GPU result is checked bit for bit
    against the oracle on the same inputs.  `crossover` = the smallest size from which the GPU path is faster
    at that size and every larger one (null: never).  The oracle is the CPU baseline here, never the product."""
    import oracle  # test infrastructure: the CPU baseline legs only
    cores = granted_cpus()
    esz = dccl_amd.size_of_type(dt)
    top = HOST_SIZES[-1]
    pin_s = torch.empty(top, dtype=torch.uint8).pin_memory()
    pin_r = torch.empty(top, dtype=torch.uint8).pin_memory()
    pin_s.view(torch.float32).uniform_(-1, 1)
    pin_r.view(torch.float32).uniform_(-1, 1)
    pag_s = oracle.aligned_empty(top, np.uint8, align=4096)
    pag_r = oracle.aligned_empty(top, np.uint8, align=4096)
    reg_s = oracle.aligned_empty(top, np.uint8, align=4096)
    reg_r = oracle.aligned_empty(top, np.uint8, align=4096)
    for dst, src in ((pag_s, pin_s), (pag_r, pin_r), (reg_s, pin_s), (reg_r, pin_r)):
        np.copyto(dst, src.numpy())
    for b in (reg_s, reg_r):
        dccl_amd.check(dccl_amd.register_host_memory(b.ctypes.data, top), "dccl_register_host_memory")
    bufs = {"registered": (reg_s, reg_r), "pinned": (pin_s.numpy(), pin_r.numpy()), "pageable": (pag_s, pag_r)}
    placement = {kind: numa_nodes_of(s.ctypes.data) for kind, (s, _) in bufs.items()}
    nodes = node_cpus()
    full_affinity = os.sched_getaffinity(0)

    def cpu_pick(kind, local):  # a CPU on (local) or off (remote) the node holding the buffer, None if unknown
        pages = placement.get(kind) or {}
        if not pages or len(nodes) < (1 if local else 2):
            return None
        home = int(max(pages, key=pages.get)[1:])
        cands = [c for nd, cs in nodes.items() if (nd == home) == local for c in cs]
        return cands[len(cands) // 2] if cands else None

    def time_cpu1(kind, local, ps, pr, n, nsets, stride, budget):
        cpu = cpu_pick(kind, local)
        if cpu is None and not local:
            return None
        try:
            if cpu is not None:
                os.sched_setaffinity(0, {cpu})
            return oracle.time_host_reduce(ps, pr, n, dt, op, 1, nsets, stride, budget)[0]
        finally:
            os.sched_setaffinity(0, full_affinity)
    npd = oracle.NP_DTYPES[dt]
    rows = []
    for size in HOST_SIZES:
        n = size // esz
        nsets = max(1, min(HOST_ROTATE_BYTES, top) // size)
        row = {"bytes": size, "operand_pairs_rotated": nsets}
        for kind, (s, r) in bufs.items():
            ps, pr = s.ctypes.data, r.ctypes.data
            want = r[:size].view(npd).copy()  # pair 0, checked bit for bit against the oracle
            dccl_amd.check(dccl_amd.local_reduce_host(ps, pr, dt, n, op), "dccl_local_reduce_host")
            oracle.expected_reduce(s[:size].view(npd), want, dt, op)
            exact = r[:size].tobytes() == want.tobytes()
            del want
            # every leg three times, interleaved, each trial a third of the budget; the fastest trial of each leg
            # is kept (the host's CPUs and memory are shared with the node's other GPUs' jobs)
            legs = {"gpu_us": lambda: _gpu_host_us(ps, pr, n, nsets, size, dt, op, min_s / 3)[0] * 1e-6,
                    "cpu1_us": lambda: time_cpu1(kind, True, ps, pr, n, nsets, size, min_s / 3),
                    "cpu1_remote_us": lambda: time_cpu1(kind, False, ps, pr, n, nsets, size, min_s / 3),
                    "cpu_all_us": lambda: oracle.time_host_reduce(ps, pr, n, dt, op, cores, nsets, size,
                                                                  min_s / 3)[0]}
            if kind == "registered" and size <= 64 << 20:
                legs["cpu1_hot_us"] = lambda: time_cpu1(kind, True, ps, pr, n, 1, 0, min_s / 3)
            trials = {k: [] for k in legs}
            for _ in range(3):
                for k, fn in legs.items():
                    trials[k].append(fn())
            rec = {k: round(min(v) * 1e6, 2) for k, v in trials.items() if None not in v}
            rec["spread"] = {k: round(max(v) / min(v), 3) for k, v in trials.items() if None not in v}
            rec.update(gpu_payload_gib_s=round(size / (rec["gpu_us"] * 1e-6) / GIB, 2), bit_exact=exact)
            row[kind] = rec
        rows.append(row)
        progress(f"host crossover {size >> 10} KiB, registered: GPU {row['registered']['gpu_us']} us, "
                 f"CPU 1 core {row['registered']['cpu1_us']} us (other node "
                 f"{row['registered'].get('cpu1_remote_us')} us), {cores} cores {row['registered']['cpu_all_us']} us")
    kinds = list(bufs)
    for b in (reg_s, reg_r):
        dccl_amd.check(dccl_amd.deregister_host_memory(b.ctypes.data), "dccl_deregister_host_memory")
    del pin_s, pin_r, pag_s, pag_r, reg_s, reg_r, bufs

    def crossover(kind, key):
        win = None
        for row in reversed(rows):
            if key not in row[kind]:  # cpu1_hot_us: only up to 64 MiB (larger pairs do not stay in a cache)
                continue
            if not row[kind]["gpu_us"] < row[kind][key]:
                break
            win = row["bytes"]
        return win

    f, reps, t0 = dccl_amd.lib.dccl_size_of_type, 0, time.perf_counter()
    while reps < 200000:  # the Python loop's own cost per ctypes call, included in every gpu_us
        f(dt)
        reps += 1
    call_us = (time.perf_counter() - t0) / reps * 1e6
    return {
        "python_call_overhead_us": round(call_us, 3),
        "crossover": {kind: {"vs_1_core": crossover(kind, "cpu1_us"), "vs_1_core_hot": crossover(kind, "cpu1_hot_us"),
                             "vs_1_core_remote_node": crossover(kind, "cpu1_remote_us"),
                             f"vs_{cores}_cores": crossover(kind, "cpu_all_us")} for kind in kinds},
        "cores": cores, "dtype": dt, "op": op, "numa_pages_by_kind": placement,
        "cpu1_cpus": {kind: {"local": cpu_pick(kind, True), "remote": cpu_pick(kind, False)} for kind in kinds},
        "all_bit_exact": all(row[k]["bit_exact"] for row in rows for k in kinds),
        "product_default_gpu_min_bytes": dccl_amd.host_reduce_gpu_min_bytes(dt),
        "rows": rows,
        "how": "same host buffers for every leg; GPU = dccl_local_reduce_host per call (synchronous); CPU = "
               "oracle/host_reduce.c (restatement of internal_common.hpp:496-586, -O3 -mprefer-vector-width=512) "
               "timed in C, 1 thread and `cores` threads (64-B aligned slices, spinning team); pairs rotated over "
               f"{HOST_ROTATE_BYTES >> 20} MiB per operand (cold), cpu1_hot_us = one pair repeated (registered "
               "kind, up to 64 MiB)",
    }


def config_c3(dev, stream, nbytes: int = 1 << 30, launches: int = 20, pool: torch.Tensor | None = None) -> list:
    """BASELINE config C3: every ncclRedOp_t x {fp16, bf16, fp32, int32, int64} on 1 GiB operands (pooled
    layout), each timed over `launches` back-to-back launches (HIP events on the launch stream) and its
    result checked by verify_sample (3 + launches applications).  `pool`: the headline's own allocation
    (recv, then send PAIR_GAP bytes past it), so every dtype and op runs on the same buffers as the headline;
    a re-allocated pool lands in another physical placement and runs ~1 point slower."""
    out = []
    if pool is None or pool.numel() < 2 * nbytes + PAIR_GAP:
        pool = torch.empty(2 * nbytes + PAIR_GAP, dtype=torch.uint8, device=dev)
    names = {6: "f16", 9: "bf16", 7: "f32", 2: "i32", 4: "i64"}
    for dt in (6, 9, 7, 2, 4):
        esz = dccl_amd.size_of_type(dt)
        n = nbytes // esz
        tdt = dccl_amd.TORCH_DTYPES[dt]
        recv = pool[:nbytes].view(tdt)
        send = pool[nbytes + PAIR_GAP:].view(tdt)
        for op, oname in enumerate(("sum", "prod", "max", "min")):
            synth_into(send, n, dt, op, 20)
            synth_into(recv, n, dt, op, 21)
            k = time_kernel(send.data_ptr(), recv.data_ptr(), dt, n, op, stream, launches)
            ok = verify_sample(recv, n, dt, op, 20, 21, 3 + launches)
            out.append({"dtype": names[dt], "op": oname, "kernel_ms_avg": round(k, 4),
                        "frac": round(3 * nbytes / (k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "verified": ok})
    del pool
    torch.cuda.empty_cache()
    return out


def _time_pairs(pairs, n: int, stream, launches: int) -> float:
    """Average duration (ms) of `launches` back-to-back fp32 Sum combines cycling over the (send, recv)
    pointer pairs, HIP events on `stream`."""
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    sh = stream.cuda_stream
    for ps, pr in pairs[:3]:
        dccl_amd.check(dccl_amd.local_reduce(ps, pr, 7, n, 0, sh))
    ev0.record(stream)
    for i in range(launches):
        ps, pr = pairs[i % len(pairs)]
        dccl_amd.check(dccl_amd.local_reduce(ps, pr, 7, n, 0, sh))
    ev1.record(stream)
    ev1.synchronize()
    return ev0.elapsed_time(ev1) / launches


def graph_us_per_launch(pairs, n: int, dev, per_graph: int = 200, replays: int = 10) -> float:
    """Average duration (us) of one fp32 Sum combine of n elements when `per_graph` launches (cycling over
    the pointer pairs) are captured in one HIP graph (torch.cuda.CUDAGraph over dccl_local_reduce on the
    capture stream) and the graph is replayed `replays` times, in three timed windows (median): the device-side
    cost per launch without the host's issue rate."""
    side = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        dccl_amd.check(dccl_amd.local_reduce(pairs[0][0], pairs[0][1], 7, n, 0, side.cuda_stream), "warm")
        side.synchronize()
        with torch.cuda.graph(g, stream=side):
            for i in range(per_graph):
                ps, pr = pairs[i % len(pairs)]
                dccl_amd.check(dccl_amd.local_reduce(ps, pr, 7, n, 0, side.cuda_stream), "capture")
    g.replay()
    torch.cuda.synchronize(dev)
    cur = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    runs = []
    for _ in range(3):  # the median of three timed windows: one disturbed window does not set the point
        ev0.record(cur)
        for _ in range(replays):
            g.replay()
        ev1.record(cur)
        ev1.synchronize()
        runs.append(ev0.elapsed_time(ev1))
    del g
    return sorted(runs)[1] * 1e3 / (replays * per_graph)


MALL_BYTES = 256 << 20  # MI355X Infinity Cache


def config_c4(dev, stream) -> list:
    """BASELINE config C4: 2^12 ... 2^32 bytes per operand, powers of 2 (21 points), ncclSum
    fp32, pooled layout.  Below a 512 MiB working set the launches rotate over `sets` operand pairs spread
    over 8 GiB, so the 256 MiB Infinity Cache does not hold the operands from one launch to the next; points
    whose single-pair working set (3 x bytes) fits that cache are labelled `mall`.  Per size: the average
    duration of back-to-back launches (HIP events on the launch stream, >= ~20 ms of launches), the HBM rate
    3*bytes/t against the 8 TB/s roofline and the payload GiB/s; up to 64 MiB eager launches are
    host-issue-bound, so the same rotation is also replayed from a HIP graph (graph_us_per_launch,
    graph_frac) and issued eagerly from a C++ loop (native_c4: native_eager_us_per_launch, native_eager_frac)."""
    out = []
    top = 4 << 30
    pool = torch.empty(2 * top + PAIR_GAP, dtype=torch.uint8, device=dev)
    synth_into(pool[:top].view(torch.float32), top // 4, 7, 0, 30)
    synth_into(pool[top + PAIR_GAP:].view(torch.float32), top // 4, 7, 0, 31)
    pr0, ps0 = pool.data_ptr(), pool.data_ptr() + top + PAIR_GAP
    for e in range(12, 33):
        nb = 1 << e
        n = nb // 4
        sets = 1 if 2 * nb >= (512 << 20) else min(top // nb, max(2, -(-(512 << 20) // (2 * nb))))
        stride = top // sets // 4096 * 4096 if sets > 1 else 0
        pairs = [(ps0 + j * stride, pr0 + j * stride) for j in range(sets)]
        k = _time_pairs(pairs, n, stream, 5)
        launches = int(min(20000, max(10, 20.0 / max(k, 1e-4))))
        k = _time_pairs(pairs, n, stream, launches)
        row = {"bytes_per_operand": nb, "sets": sets, "mall": 3 * nb <= MALL_BYTES, "launches": launches,
               "us_per_launch": round(k * 1e3, 2), "hbm_gb_s": round(3 * nb / (k * 1e-3) / 1e9, 1),
               "frac": round(3 * nb / (k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
               "payload_gib_s": round(nb / (k * 1e-3) / GIB, 2)}
        if nb <= (64 << 20):
            g = graph_us_per_launch(pairs, n, dev)
            row["graph_us_per_launch"] = round(g, 2)
            row["graph_frac"] = round(3 * nb / (g * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
        out.append(row)
    del pool
    torch.cuda.empty_cache()
    native = native_c4()
    for row in out:
        row.update(native.get(row["bytes_per_operand"], {}))
    if "error" in native and out:
        out[0]["native_eager_error"] = native["error"]
    return out


def ring_step(dev, stream, sizes_mib=(512, 256, 128, 64, 32, 8)) -> dict:
    """DCCL's own ring-step operand shape (reduce_scatter_ring.cpp:64-67, 84-94): `send` is the library's
    scratchpad (one separate allocation, dccl.cpp:170-237) and `recv` is chunk k of the user's all-reduce
    buffer, count/W elements.  Sizes are the chunks of a 1 GiB all-reduce at W = 2, 4, 8 (512, 256, 128 MiB)
    and of a 256 MiB one (128, 64, 32 MiB), plus 8 MiB.  Below a 512 MiB working set the launches rotate
    over `sets` scratch slots and user chunks (as in C4), so the Infinity Cache does not hold the operands.
    Per size: eager (Python-issued, back-to-back) and graph-replayed time per combine and their fraction of
    the HBM roofline (3 * bytes per combine).  Reporting only."""
    user_bytes = 2 << 30
    user = torch.empty(user_bytes, dtype=torch.uint8, device=dev)
    synth_into(user.view(torch.float32), user_bytes // 4, 7, 0, 40)
    points = []
    for mib in sizes_mib:
        nb = mib << 20
        n = nb // 4
        sets = 1 if 2 * nb >= (512 << 20) else max(2, -(-(512 << 20) // (2 * nb)))
        scratch = torch.empty(sets * nb, dtype=torch.uint8, device=dev)  # the library's scratchpad
        synth_into(scratch.view(torch.float32), sets * n, 7, 0, 41)
        pairs = [(scratch.data_ptr() + j * nb, user.data_ptr() + ((2 * j + 1) * nb) % user_bytes) for j in range(sets)]
        k = _time_pairs(pairs, n, stream, 5)
        k = _time_pairs(pairs, n, stream, int(min(2000, max(10, 20.0 / max(k, 1e-4)))))
        g = graph_us_per_launch(pairs, n, dev, per_graph=min(200, max(20, int(20e3 / max(k * 1e3, 1.0)))))
        points.append({"mib": mib, "sets": sets, "eager_us": round(k * 1e3, 1),
                       "eager_frac": round(3 * nb / (k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                       "graph_us": round(g, 1), "graph_frac": round(3 * nb / (g * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)})
        del scratch
    del user
    torch.cuda.empty_cache()
    return {"shape": "send = separately allocated scratchpad slot, recv = chunk of a 2 GiB user buffer, fp32 Sum",
            "points": points}


def native_c4(max_log2: int = 26) -> dict:
    """C4 up to 2^max_log2 bytes per operand issued from a C++ loop (dccl_amd/bin/c4_native, the same rotation
    over operand sets): the eager per-launch time a native caller such as DCCL's ring step loop sees, without
    the Python/ctypes issue cost of the `us_per_launch` column.  Runs as a child process; any failure is
    reported, never fatal."""
    import subprocess
    binary = os.path.join(ROOT, "dccl_amd", "bin", "c4_native")
    if not os.path.exists(binary):
        return {"error": "dccl_amd/bin/c4_native missing"}
    try:
        p = subprocess.run([binary, str(max_log2)], capture_output=True, text=True, timeout=180)
    except subprocess.TimeoutExpired:
        return {"error": "c4_native timed out"}
    res = {}
    for line in p.stdout.splitlines():
        if line.startswith("{"):
            d = json.loads(line)
            res[d["bytes_per_operand"]] = {k: d[k] for k in ("native_eager_us_per_launch", "native_eager_frac")}
    if p.returncode != 0:
        res["error"] = f"c4_native exited with {p.returncode}: {p.stderr[-200:]}"
    return res


def run_with_watchdog(fn, seconds: float):
    """Run fn() in a daemon thread; (result, finished).  A collective that hangs must not take the
    bench line with it: the caller reports the timeout and exits without joining the thread."""
    box = {}
    done = threading.Event()

    def target():
        try:
            box["value"] = fn()
        except Exception as e:  # reported in the JSON line
            box["value"] = {"error": repr(e)}
        finally:
            done.set()

    threading.Thread(target=target, daemon=True).start()
    if not done.wait(seconds):
        return {"error": f"timed out after {seconds:.0f}s"}, False
    return box["value"], True


def dccl_allreduce_multi(world: int, rank: int, dev, count: int, iters: int = 5) -> dict:
    """the namespace-dccl ncclAllReduce end to end on one node, one process per GPU,
    through both cross-process transports:
      ring    ring RS with the gfx950 combine + ring AG, chunks moved by RCCL send/recv;
      direct  each GPU reduces its chunk from all peers' buffers at once over xGMI (IPC-mapped,
              dccl_local_reduce_chain in the ring's order) and pulls the other chunks.
    Both are checked against RCCL's own all_reduce (int32: bit-exact; fp32: |d| <= (W-1) eps sum|x|, a
    different association order) and against each other (fp32: bit-exact, same order), and timed."""
    _native()
    os.environ.setdefault("DCCL_IPC_TIMEOUT_S", "60")
    transports = os.environ.get("DCCL_BENCH_AR_TRANSPORTS", "ring,direct").split(",")
    # wall seconds per phase: returned as `phase_s`, and rewritten after every phase to
    # DCCL_BENCH_PHASE_FILE by rank 0, so a child the watchdog kills still says how far it got
    phases, last = {}, [time.perf_counter()]

    def mark(name):
        now = time.perf_counter()
        phases[name] = round(now - last[0], 2)
        last[0] = now
        path = os.environ.get("DCCL_BENCH_PHASE_FILE")
        if path and rank == 0:
            with open(path, "w") as f:
                json.dump(phases, f)

    uid = None
    if rank == 0 and "ring" in transports:
        try:
            uid = dccl_amd.Comm.unique_id()
        except Exception:  # every rank must still reach the broadcast below
            uid = None
    obj = [uid]
    dist.broadcast_object_list(obj, src=0)
    comms = {}
    if obj[0] is not None:
        # one RCCL communicator, two algorithms: the reference's ring step loop (the default), and the grouped
        # form (one RCCL group per phase, one chain combine, DCCL_ALLREDUCE_ALGORITHM=grouped, algorithms.hpp)
        comms["ring"] = dccl_amd.Comm.rccl(world, rank, obj[0])
        comms["grouped"] = comms["ring"]
    if "direct" in transports:
        comms["direct"] = dccl_amd.Comm.ipc(world, rank)
    algo_env = {"ring": "ring", "grouped": "grouped", "direct": "auto"}
    out = {"count": count, "world": world, "bytes": count * 4, "phase_s": phases}
    mark("init")
    try:
        st = torch.cuda.current_stream(dev)
        g = torch.Generator(device=dev).manual_seed(1234 + rank)
        xi = torch.randint(-2**20, 2**20, (count,), device=dev, generator=g, dtype=torch.int32)
        xf = torch.rand(count, device=dev, generator=g).mul_(2).sub_(1)
        ri, rf = xi.clone(), xf.clone()
        dist.all_reduce(ri)
        dist.all_reduce(rf)
        yf_by = {}
        for name, comm in comms.items():
            if rank == 0:
                progress(f"child: all_reduce over {name}, {count * 4 >> 20} MiB, W = {world}")
            os.environ["DCCL_ALLREDUCE_ALGORITHM"] = algo_env[name]
            yi = xi.clone()
            yf = xf.clone()
            torch.cuda.synchronize(dev)
            dccl_amd.check(comm.all_reduce(yi.data_ptr(), yi.data_ptr(), count, 2, 0, st.cuda_stream), name)
            dccl_amd.check(comm.all_reduce(yf.data_ptr(), yf.data_ptr(), count, 7, 0, st.cuda_stream), name)
            torch.cuda.synchronize(dev)
            bound = (world - 1) * 1.2e-7 * world  # |x| < 1
            diff = float((yf - rf).abs().max())
            res = {"int32_sum_bit_exact_vs_rccl": bool(torch.equal(yi, ri)),
                   "fp32_max_abs_diff_vs_rccl": diff, "fp32_within_bound": diff <= bound}
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                dccl_amd.check(comm.all_reduce(yf.data_ptr(), yf.data_ptr(), count, 7, 0, st.cuda_stream), name)
            torch.cuda.synchronize(dev)
            t = (time.perf_counter() - t0) / iters
            res.update({"ms": round(t * 1e3, 3), "busbw_gb_s": round(2 * (world - 1) / world * count * 4 / t / 1e9, 1)})
            if name != "grouped":  # broadcast / reduce do not depend on the all-reduce algorithm
                res.update(root_ops(comm, world, rank, dev, st, xi, ri, iters))
            out[name] = res
            yf_by[name] = yf
            mark(f"allreduce_{name}")
        # same association order: the first all_reduce of every path must agree with the ring's bit for bit
        if "ring" in yf_by:
            first = {}
            for name in ("ring", "grouped", "direct"):
                if name in comms:
                    os.environ["DCCL_ALLREDUCE_ALGORITHM"] = algo_env[name]
                    first[name] = xf.clone()
                    torch.cuda.synchronize(dev)
                    dccl_amd.check(comms[name].all_reduce(first[name].data_ptr(), first[name].data_ptr(), count, 7,
                                                          0, st.cuda_stream), name)
                    torch.cuda.synchronize(dev)
            for name in ("grouped", "direct"):
                if name in first:
                    out[f"fp32_{name}_bit_exact_vs_ring"] = bool(torch.equal(first["ring"].view(torch.int32),
                                                                             first[name].view(torch.int32)))
        os.environ["DCCL_ALLREDUCE_ALGORITHM"] = "auto"
        mark("bit_exact_vs_ring")
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(rf)
        torch.cuda.synchronize(dev)
        t = (time.perf_counter() - t0) / iters
        out["rccl_allreduce"] = {"ms": round(t * 1e3, 3),
                                 "busbw_gb_s": round(2 * (world - 1) / world * count * 4 / t / 1e9, 1),
                                 "backend": dist.get_backend(),
                                 "note": "the torch.distributed backend's own all_reduce (RCCL when the backend is "
                                         "nccl), informational: its combine is the backend's"}
        mark("rccl_allreduce")
        out["sweep_busbw_gb_s"] = allreduce_sweep(comms, algo_env, world, rank, dev, st, iters)
        mark("sweep")
        if rank == 0:
            progress("child: all_gather of every transport")
        out["dccl_allgather"] = allgather_compare({k: v for k, v in comms.items() if k != "grouped"}, world, rank,
                                                  dev, st, count, iters)
        mark("allgather")
        # BASELINE C5's exchange step at its own size (the reduced shards of DCCL_BENCH_C5_GIB GiB of fp32,
        # moved as int32): the direct IPC all-gather beside RCCL's (the single-link ring is left out here)
        c5_gib = float(os.environ.get("DCCL_BENCH_C5_GIB", "0") or 0)
        if c5_gib > 0 and "direct" in comms:
            c5_count = int(c5_gib * GIB) // 4 // world * world
            if rank == 0:
                progress(f"child: C5's all_gather, {c5_gib:g} GiB")
            torch.cuda.empty_cache()
            out["c5_allgather"] = allgather_compare({"direct": comms["direct"]}, world, rank, dev, st, c5_count, 3)
            mark("c5_allgather")
    finally:
        for comm in {id(c): c for c in comms.values()}.values():
            comm.finalize()
    mark("finalize")
    if "direct" in comms:  # the IPC transport's counters, summed over the ranks (alias_errors must be 0)
        every = [None] * world
        dist.all_gather_object(every, dccl_amd.ipc_stats())
        out["ipc_stats"] = {k: sum(d[k] for d in every) for k in every[0]}
    return out


def allreduce_sweep(comms: dict, algo_env: dict, world: int, rank: int, dev, st, iters: int) -> dict:
    """fp32 Sum all-reduce bus bandwidth (GB/s, 2 (W-1)/W x bytes / time) per size for every namespace-dccl
    algorithm and the torch.distributed backend's own all_reduce, timing only (the 256 MiB collective above is
    the checked one): the data the first xGMI run decides the RCCL default by, per size.
    Sizes from DCCL_BENCH_AR_SWEEP_MIB (the parent passes 1,16,64,256; 1,4 in a socket rehearsal)."""
    sizes = [int(x) for x in os.environ.get("DCCL_BENCH_AR_SWEEP_MIB", "1,16,64,256").split(",") if x.strip()]
    out = {}
    for mib in sizes:
        cnt = (mib << 20) // 4 // world * world
        if cnt == 0:
            continue
        if rank == 0:
            progress(f"child: all_reduce sweep, {mib} MiB")
        buf = torch.rand(cnt, device=dev)
        row = {}

        def timed(call):
            call()  # warm (first use of a size may map or grow a scratch)
            torch.cuda.synchronize(dev)
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                call()
            torch.cuda.synchronize(dev)
            return (time.perf_counter() - t0) / iters

        for name, comm in comms.items():
            os.environ["DCCL_ALLREDUCE_ALGORITHM"] = algo_env[name]
            t = timed(lambda: dccl_amd.check(comm.all_reduce(buf.data_ptr(), buf.data_ptr(), cnt, 7, 0,
                                                             st.cuda_stream), name))
            row[name] = float(f"{2 * (world - 1) / world * cnt * 4 / t / 1e9:.3g}")
        os.environ["DCCL_ALLREDUCE_ALGORITHM"] = "auto"
        t = timed(lambda: dist.all_reduce(buf))
        row["rccl"] = float(f"{2 * (world - 1) / world * cnt * 4 / t / 1e9:.3g}")
        out[str(mib)] = row
        del buf
    return out


def root_ops(comm, world: int, rank: int, dev, st, xi, ri, iters: int) -> dict:
    """ncclBroadcast and ncclReduce (root 0, int32) through the namespace-dccl API of this transport: the
    broadcast must deliver rank 0's input bit for bit (regenerated from its seed), the reduce must leave
    RCCL's own all_reduce sum at the root; each is timed.  On the RCCL transport the root's W - 1 transfers
    run in one group (rccl_fan)."""
    count = xi.numel()
    want0 = torch.randint(-2**20, 2**20, (count,), device=dev, dtype=torch.int32,
                          generator=torch.Generator(device=dev).manual_seed(1234))
    y = torch.empty_like(xi)
    z = torch.zeros_like(xi)
    out = {}
    for what in ("broadcast", "reduce"):
        def call():
            if what == "broadcast":
                return comm.broadcast(xi.data_ptr(), y.data_ptr(), count, 2, 0, st.cuda_stream)
            return comm.reduce(xi.data_ptr(), z.data_ptr(), count, 2, 0, 0, st.cuda_stream)
        dccl_amd.check(call(), what)
        torch.cuda.synchronize(dev)
        ok = bool(torch.equal(y, want0)) if what == "broadcast" else (rank != 0 or bool(torch.equal(z, ri)))
        flag = torch.tensor([int(ok)], dtype=torch.int32, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            dccl_amd.check(call(), what)
        torch.cuda.synchronize(dev)
        out[f"{what}_bit_exact"] = bool(flag[0])
        out[f"{what}_ms"] = round((time.perf_counter() - t0) / iters * 1e3, 3)
    return out


def allgather_compare(comms: dict, world: int, rank: int, dev, st, count: int, iters: int) -> dict:
    """The exchange step of C5 (and the second half of the direct all-reduce) through the namespace-dccl
    ncclAllGather of each transport, int32, count/world elements per rank: checked bit for bit against
    the concatenation of every rank's slice (each rank regenerates all slices from their seeds), timed,
    and beside RCCL's all_gather_into_tensor when torch.distributed runs on RCCL."""
    per = count // world

    def slice_of(p):  # rank p's input, regenerated anywhere from its seed
        return torch.randint(-2**31, 2**31 - 1, (per,), device=dev, dtype=torch.int32,
                             generator=torch.Generator(device=dev).manual_seed(777 + p))

    mine = slice_of(rank)
    res = {"bytes_per_rank": per * 4}
    y = torch.empty(per * world, dtype=torch.int32, device=dev)
    for name, comm in comms.items():
        y.zero_()
        torch.cuda.synchronize(dev)
        dccl_amd.check(comm.all_gather(mine.data_ptr(), y.data_ptr(), per, 2, st.cuda_stream), name)
        torch.cuda.synchronize(dev)
        wrong = {}
        for p in range(world):  # per peer slice: the fraction of elements that differ, and of 128-B lines
            d = y[p * per:(p + 1) * per] != slice_of(p)
            if bool(d.any()):
                lines = d[:per // 32 * 32].view(-1, 32).any(dim=1)
                wrong[p] = {"elems": round(float(d.float().mean()), 6), "lines": round(float(lines.float().mean()), 6)}
        # every rank checked its own copy: agree on the result and count the wrong slices over all ranks
        nwrong = torch.tensor([len(wrong)], dtype=torch.int64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(nwrong)
        ok = int(nwrong[0]) == 0
        dist.barrier()
        each = []
        t0 = time.perf_counter()
        for _ in range(iters):
            t1 = time.perf_counter()
            dccl_amd.check(comm.all_gather(mine.data_ptr(), y.data_ptr(), per, 2, st.cuda_stream), name)
            torch.cuda.synchronize(dev)
            each.append((time.perf_counter() - t1) * 1e3)
        t = (time.perf_counter() - t0) / iters
        res[name] = {"bit_exact": ok, "wrong_slices_all_ranks": int(nwrong[0]), "ms": round(t * 1e3, 3),
                     "ms_each": [round(x, 3) for x in each], "busbw_gb_s": round((world - 1) * per * 4 / t / 1e9, 1)}
        if wrong:
            res[name]["wrong_slices"] = wrong
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(y, mine)
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_gather_into_tensor(y, mine)
        torch.cuda.synchronize(dev)
        t = (time.perf_counter() - t0) / iters
        res["rccl"] = {"ms": round(t * 1e3, 3), "busbw_gb_s": round((world - 1) * per * 4 / t / 1e9, 1)}
    return res


def c5_extra(a, world: int, rank: int, dev, backend: str, coll_dev) -> dict:
    """BASELINE config C5 measured inside every bench run, so the driver's 1/2/4/8-GPU runs report it too:
    one buffer of a.c5_gib GiB per operand (fp32 Sum) split into contiguous 256-B aligned shards
    (dccl_amd/shard.py), each GPU combining its shard (strong scaling: fixed total work), then the one
    exchange step, an RCCL all-gather of the reduced shards over xGMI (every GPU ends with the whole
    result).  Timings are barrier-bracketed and max-over-ranks, like the headline."""
    from dccl_amd.shard import all_bounds
    esz, dt, op = 4, 7, 0
    total = int(a.c5_gib * GIB) // esz
    bounds = all_bounds(total, esz, world)
    n = bounds[rank][1] - bounds[rank][0]
    send, recv = operand_pair(n, dt, op, 2 * rank, dev, "pooled")
    stream = torch.cuda.current_stream(dev)
    steps = 10
    for _ in range(2):
        dccl_amd.check(dccl_amd.local_reduce(send.data_ptr(), recv.data_ptr(), dt, n, op, stream.cuda_stream))

    def bracket(fn, iters):
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64, device=coll_dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    tc = bracket(lambda: dccl_amd.check(dccl_amd.local_reduce(send.data_ptr(), recv.data_ptr(), dt, n, op,
                                                               stream.cuda_stream)), steps)
    # every rank checks sampled slices of its combined shard (2 + steps applications), then all agree
    ok = verify_sample(recv, n, dt, op, 2 * rank, 2 * rank + 1, 2 + steps)
    if world > 1:
        flag = torch.tensor([int(bool(ok))], dtype=torch.int32, device=coll_dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = bool(flag[0])
    out = {"total_gib_per_operand": a.c5_gib, "shard_bytes_per_operand_max": max(b - a_ for a_, b in bounds) * esz,
           "steps": steps, "combine_ms": round(tc * 1e3, 4),
           "value": round(3 * total * esz / tc / GIB, 2), "unit": "GiB/s (3*N*4 B over all GPUs)",
           "frac_of_n_hbm_peaks": round(3 * total * esz / tc / 1e9 / (HBM_PEAK_GBS * world), 4),
           "scaling": "strong", "verified": ok,
           "verification": "every rank: first, last and 4 random 64 Ki-element slices of its shard, inputs "
                           "regenerated on the device, 12 sequential torch fp32 adds, bit-exact"}
    del send
    if world > 1:
        width = max(b - a_ for a_, b in bounds)
        src = recv if width == n else torch.cat([recv, recv.new_zeros(width - n)])
        src = src.to(coll_dev)
        del recv
        gathered = torch.empty(world * width, dtype=src.dtype, device=coll_dev)
        dist.all_gather_into_tensor(gathered, src)
        tg = bracket(lambda: dist.all_gather_into_tensor(gathered, src), 3)
        out["allgather"] = {"ms": round(tg * 1e3, 3), "backend": backend,
                            "algbw_gb_s": round(total * esz / tg / 1e9, 1),
                            "busbw_gb_s": round((world - 1) * width * esz / tg / 1e9, 1)}
        out["combine_plus_allgather_ms"] = round((tc + tg) * 1e3, 3)
        del gathered, src
    torch.cuda.empty_cache()
    progress(f"C5 ({a.c5_gib:g} GiB sharded): combine {tc * 1e3:.3f} ms" +
             (f", all-gather {out['allgather']['ms']} ms" if world > 1 else ""))
    return out


def progress(msg: str) -> None:
    """One line on stderr per phase, so a long multi-GPU run is never silent (the JSON line is stdout)."""
    print(f"[bench] rank {os.environ.get('RANK', '0')}: {msg}", file=sys.stderr, flush=True)


CHILD_TIMEOUT_S = 150.0
# DCCL_BENCH_RCCL_REHEARSAL=1 with more ranks than GPUs: RCCL runs over loopback sockets, ~100x slower than
# xGMI, so the child's collectives are sized down (the paths are the same) and given longer
REHEARSAL_CHILD_TIMEOUT_S = 420.0
REHEARSAL_AR_MIB = 32
REHEARSAL_C5_GIB = 1.0


def socket_rehearsal(world: int, backend: str) -> bool:
    """N RCCL ranks sharing fewer GPUs over loopback sockets (DCCL_BENCH_RCCL_REHEARSAL=1)."""
    return (backend == "nccl" and os.environ.get("DCCL_BENCH_RCCL_REHEARSAL") == "1"
            and world > torch.cuda.device_count())


def collective_in_child(world: int, rank: int, local: int, backend: str, c5_gib: float = 0.0) -> dict:
    """Run dccl_allreduce_multi in a child process per rank, with its own process group on a fresh port.
    The namespace-dccl collectives (RCCL p2p ring, IPC peer reads) are reported extras, never `value`: a
    fault or hang inside them ends the child, which is killed after CHILD_TIMEOUT_S, while this process,
    its measurement and the JSON line survive.  Every parent waits at most that long and joins no
    collective of the child, so no rank can be left behind."""
    import socket
    import subprocess
    port = [0]
    if rank == 0:
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port[0] = sk.getsockname()[1]
    dist.broadcast_object_list(port, src=0)
    # not the launcher's agent store (torchrun exports TORCHELASTIC_USE_AGENT_STORE): the child's rank 0
    # hosts its own store on the fresh port
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    import tempfile
    phase_file = os.path.join(tempfile.gettempdir(), f"dccl_bench_phases_{os.getpid()}.json")
    rehearsal = socket_rehearsal(world, backend)
    timeout = REHEARSAL_CHILD_TIMEOUT_S if rehearsal else CHILD_TIMEOUT_S
    env = {**env, "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port[0]), "RANK": str(rank),
           "WORLD_SIZE": str(world), "LOCAL_RANK": str(local), "DCCL_BENCH_BACKEND": backend,
           "DCCL_BOOTSTRAP_TAG": f"bench_child_{port[0]}",
           "DCCL_BENCH_C5_GIB": str(min(c5_gib, REHEARSAL_C5_GIB) if rehearsal else c5_gib),
           "DCCL_BENCH_AR_MIB": str(REHEARSAL_AR_MIB if rehearsal else 256),
           "DCCL_BENCH_AR_SWEEP_MIB": "1,4" if rehearsal else "1,16,64,256",
           "DCCL_BENCH_CHILD_TIMEOUT_S": str(timeout), "DCCL_BENCH_PHASE_FILE": phase_file}
    torch.cuda.synchronize()
    progress(f"namespace-dccl all_reduce extras in a child process (port {port[0]}"
             + (f", socket rehearsal: {REHEARSAL_AR_MIB} MiB all-reduces, timeout {timeout:.0f}s)" if rehearsal else ")"))
    t0 = time.perf_counter()

    def phases_so_far():
        try:
            with open(phase_file) as f:
                return json.load(f)
        except Exception:
            return None
        finally:
            if os.path.exists(phase_file):
                os.remove(phase_file)

    try:
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--collective-child"], env=env,
                           stdout=subprocess.PIPE, stderr=None, text=True, timeout=timeout)
    except subprocess.TimeoutExpired:
        return {"error": f"child timed out after {timeout:.0f}s and was killed", "child_timeout_s": timeout,
                "phase_s": phases_so_far()}
    wall = time.perf_counter() - t0
    progress(f"child exited with {p.returncode} after {wall:.1f}s")
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    res = json.loads(lines[-1]) if lines else {}
    res.update(child_wall_s=round(wall, 1), child_timeout_s=timeout)
    if "phase_s" not in res:
        res["phase_s"] = phases_so_far()
    else:
        phases_so_far()  # remove the file
    if p.returncode != 0:
        res = {**res, "error": res.get("error", f"child exited with {p.returncode}")}
    return res


def collective_child() -> None:
    """Entry point of the child process started by collective_in_child."""
    _native()
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    backend = os.environ.get("DCCL_BENCH_BACKEND", "nccl")
    local = int(os.environ["LOCAL_RANK"]) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    import datetime
    limit = datetime.timedelta(seconds=60)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev, timeout=limit)
    else:
        dist.init_process_group(backend, timeout=limit)
    count = (int(os.environ.get("DCCL_BENCH_AR_MIB", "256")) << 20) // 4 // world * world
    limit_s = float(os.environ.get("DCCL_BENCH_CHILD_TIMEOUT_S", str(CHILD_TIMEOUT_S)))
    res, finished = run_with_watchdog(lambda: dccl_allreduce_multi(world, rank, dev, count), limit_s - 30)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if not finished or "error" in res:
        os._exit(3)  # a rank may be stuck inside a collective: never wait for it at teardown
    dist.barrier()
    dist.destroy_process_group()


def launch_ranks(a, argv) -> int:
    """`--gpus N` with no WORLD_SIZE in the environment: start N rank processes, one per GPU, as the
    reference's harness runs one process per rank (/root/reference/README.md:74-101,
    src/application/cli.cpp:360-381), each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
    MASTER_PORT set as torch.distributed.run sets them.  This process never touches the GPU (it only
    counts devices, which does not initialise one on this image), relays rank 0's JSON line, and exits
    non-zero if any rank fails or outlives --rank-timeout (the others are then terminated: a rank left
    alone would wait in a collective forever).  Returns the exit code."""
    import signal
    import socket
    import subprocess
    n = a.gpus
    backend = os.environ.get("DCCL_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    # DCCL_BENCH_RCCL_REHEARSAL=1: N RCCL ranks on fewer GPUs.  RCCL refuses two ranks on one device of one
    # host, so each rank gets its own NCCL_HOSTID: RCCL then sees N hosts and joins them over its socket
    # transport on loopback (every RCCL call of the bench, the namespace-dccl ring over RCCL included, runs
    # for real; the rates are not xGMI rates)
    rehearse_rccl = backend == "nccl" and os.environ.get("DCCL_BENCH_RCCL_REHEARSAL") == "1"
    if backend == "nccl" and ndev < n and not rehearse_rccl:
        print(f"bench.py: --gpus {n} needs {n} GPUs, {ndev} visible (DCCL_BENCH_BACKEND=gloo or "
              f"DCCL_BENCH_RCCL_REHEARSAL=1 rehearse N ranks on fewer GPUs)", file=sys.stderr)
        return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    # a SIGTERM from whoever runs the bench ends the ranks too (the finally below)
    signal.signal(signal.SIGTERM, lambda *_: sys.exit(143))
    procs, out = [], {}
    progress(f"launching {n} rank processes (backend {backend}, {ndev} GPU(s) visible, port {port})")
    try:
        for r in range(n):
            env = {**os.environ, "RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                   "LOCAL_WORLD_SIZE": str(n), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                   "MASTER_PORT": str(port)}
            if rehearse_rccl:
                env.update({"NCCL_HOSTID": f"dccl-rehearsal-{port}-{r}", "NCCL_SOCKET_IFNAME": "lo",
                            "NCCL_IB_DISABLE": "1"})
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                          stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True))
        reader = threading.Thread(target=lambda: out.setdefault("stdout", procs[0].stdout.read()), daemon=True)
        reader.start()
        deadline, failed_at = time.monotonic() + a.rank_timeout, None
        while any(p.poll() is None for p in procs):
            now = time.monotonic()
            if failed_at is None and any(p.poll() not in (None, 0) for p in procs):
                failed_at = now
            if now > deadline or (failed_at is not None and now - failed_at > 30):
                break
            time.sleep(0.25)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(15)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    reader.join(15)
    codes = [p.returncode for p in procs]
    for line in out.get("stdout", "").splitlines():
        if line.startswith("{"):
            print(line, flush=True)
    if any(codes):
        print(f"bench.py: rank exit codes {codes}", file=sys.stderr)
        return next(c for c in codes if c) if all(c >= 0 for c in codes) else 1
    return 0


def other_layout_median(n: int, dt: int, op: int, rank: int, dev, stream, layout: str, pairs: int,
                        launches: int) -> dict:
    """The other operand layout, timed on `pairs` operand pairs allocated side by side (each separately
    allocated pair lands in its own physical placement; the pooled layout has one), every
    pair `launches` back-to-back launches; the median pair is reported (DCCL's own operand shape is the
    separate one: scratchpad + user chunk)."""
    import statistics
    nbytes = n * dccl_amd.size_of_type(dt)
    pairs = 1 if layout == "pooled" else max(1, min(pairs, (64 << 30) // (2 * nbytes)))
    ops = [operand_pair(n, dt, op, 2 * rank, dev, layout) for _ in range(pairs)]
    ks = sorted(time_kernel(sv.data_ptr(), rv.data_ptr(), dt, n, op, stream, launches) for sv, rv in ops)
    del ops
    torch.cuda.empty_cache()
    frac = lambda k: round(3 * nbytes / (k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)  # noqa: E731
    med = statistics.median(ks)
    return {"layout": layout, "pairs": pairs, "kernel_ms_median": round(med, 4), "frac": frac(med),
            "frac_min": frac(ks[-1]), "frac_max": frac(ks[0]), "launches_per_pair": launches}


def allreduce_summary(ar) -> dict:
    """The bit-exactness flags and rates of dccl_allreduce (N > 1), small enough for the line's tail."""
    if not isinstance(ar, dict):
        return {"error": repr(ar)}
    out = {k: ar[k] for k in ("error", "fp32_direct_bit_exact_vs_ring", "fp32_grouped_bit_exact_vs_ring", "child_wall_s",
                              "child_timeout_s", "phase_s") if k in ar}
    for name in ("ring", "grouped", "direct"):
        if isinstance(ar.get(name), dict):
            out[name] = {k: ar[name][k] for k in ("int32_sum_bit_exact_vs_rccl", "fp32_within_bound", "ms",
                                                  "busbw_gb_s", "broadcast_bit_exact",
                                                  "broadcast_ms", "reduce_bit_exact", "reduce_ms") if k in ar[name]}
    if isinstance(ar.get("rccl_allreduce"), dict):
        out["rccl"] = {k: ar["rccl_allreduce"][k] for k in ("ms", "busbw_gb_s")}
    if isinstance(ar.get("sweep_busbw_gb_s"), dict):
        out["sweep_busbw_gb_s"] = ar["sweep_busbw_gb_s"]
    for key in ("dccl_allgather", "c5_allgather"):
        ag = ar.get(key)
        if isinstance(ag, dict):
            out[key] = {name: {k: v[k] for k in ("bit_exact", "wrong_slices_all_ranks", "ms", "busbw_gb_s",
                                                 "wrong_slices") if k in v}
                        for name, v in ag.items() if isinstance(v, dict)}
    if isinstance(ar.get("ipc_stats"), dict):
        out["ipc_stats"] = {k: ar["ipc_stats"][k] for k in (
            "alias_errors", "alias_evictions", "mappings_retired", "retire_log_overflows", "open_retries",
            "size_mismatches", "scratch_copies", "verify_failures",
            "exports_made") if k in ar["ipc_stats"]}
    return out


def run_rank(a):
    """One rank: the timed combine on this rank's operands, then the reported extras."""
    _native()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; DCCL_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (CPU collectives)
    backend = os.environ.get("DCCL_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    dt = DTYPE_NAMES[a.dtype]
    op = OP_NAMES[a.op]
    esz = dccl_amd.size_of_type(dt)
    strong = a.total_gib > 0
    if strong:  # C5: contiguous 256-B aligned shards of one buffer (dccl_amd/shard.py)
        from dccl_amd.shard import all_bounds
        total_count = int(a.total_gib * GIB) // esz
        bounds = all_bounds(total_count, esz, world)
        n = bounds[rank][1] - bounds[rank][0]
        total_bytes = total_count * esz
    else:
        n = (a.mib << 20) // esz
        total_bytes = world * n * esz
    nbytes = n * esz

    progress(f"world {world}, backend {backend}, {nbytes >> 20} MiB per operand on {dev}")
    headline_pool = []
    send, recv = operand_pair(n, dt, op, 2 * rank, dev, a.layout, keep=headline_pool)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    ps, pr = send.data_ptr(), recv.data_ptr()

    def step():
        rc = dccl_amd.local_reduce(ps, pr, dt, n, op, sh)
        if rc:
            raise dccl_amd.DcclError(rc, "dccl_local_reduce")

    for _ in range(a.warmup):
        step()
    # HIP events over the timed region, on the stream the kernel is launched on: the average
    # launch duration of the dominant kernel (back-to-back launches, as rocprofv3 sees them).
    # The region is bracketed by a barrier + synchronize on both sides; each rank's clock runs from the
    # opening barrier to its own synchronize, so the closing barrier's cost is not charged to the combine,
    # and the job's time is the max over ranks.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(a.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    kern_ms = ev0.elapsed_time(ev1) / a.steps
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms_max = float(t[0]), float(t[1])
    else:
        kern_ms_max = kern_ms
    ms_per_step = elapsed / a.steps * 1e3
    progress(f"timed region done: {ms_per_step:.4f} ms per step, kernel {kern_ms:.4f} ms")
    # the timed combines' result, sampled: warmup + steps applications of the op on this rank's operands
    ok = verify_sample(recv, n, dt, op, 2 * rank, 2 * rank + 1, a.warmup + a.steps)
    if world > 1:
        flag = torch.tensor([-1 if ok is None else int(ok)], dtype=torch.int32, device=coll_dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = None if int(flag[0]) < 0 else bool(flag[0])

    extra = {}
    if world > 1:  # the exchange step: RCCL all-gather of the reduced shards (reported separately)
        width = max(b - a_ for a_, b in bounds) if strong else n
        src = recv if width == n else torch.cat([recv, recv.new_zeros(width - n)])
        src = src.to(coll_dev)
        gathered = torch.empty(world * width, dtype=recv.dtype, device=coll_dev)
        dist.all_gather_into_tensor(gathered, src)
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        iters = 3
        for _ in range(iters):
            dist.all_gather_into_tensor(gathered, src)
        torch.cuda.synchronize(dev)
        dist.barrier()
        tag = (time.perf_counter() - t0) / iters
        extra["allgather"] = {"ms": round(tag * 1e3, 3),
                              "busbw_gb_s": round((world - 1) * width * esz / tag / 1e9, 1),
                              "combine_plus_allgather_ms": round(ms_per_step + tag * 1e3, 3),
                              "backend": backend,
                              "note": "RCCL all_gather_into_tensor of the reduced shards over xGMI "
                                      "(every GPU ends with the full result); not in value"}
        del gathered, src
        progress(f"all-gather done: {tag * 1e3:.3f} ms")
    # C3 runs here, on the headline's own pooled allocation (same buffers, every dtype and op; N = 1 only),
    # before anything else is allocated: the pool is freed before the other-layout and C4 legs
    c3 = None
    if world == 1 and headline_pool and nbytes == 1 << 30 and not a.no_configs:
        progress("C3: ops x dtypes at 1 GiB")
        c3 = config_c3(dev, stream, pool=headline_pool[0])
    headline_pool.clear()
    # the other operand layout, timed briefly on every rank (reported, never in `value`)
    del send, recv
    send = recv = None
    torch.cuda.empty_cache()
    if not a.no_other_layout:
        other = "separate" if a.layout == "pooled" else "pooled"
        extra["other_layout"] = other_layout_median(n, dt, op, rank, dev, stream, other, a.other_pairs,
                                                    max(10, a.steps // 4))
        progress(f"other layout ({other}): median {extra['other_layout']['frac']:.4f} of peak")
    if a.c5_gib > 0 and not strong:
        extra["c5"] = c5_extra(a, world, rank, dev, backend, coll_dev)
    if world > 1:
        # DCCL_BENCH_AR_TRANSPORTS=direct with the gloo backend rehearses the direct path with several
        # processes on one GPU (RCCL refuses two ranks on one device)
        rehearse = backend == "gloo" and os.environ.get("DCCL_BENCH_AR_TRANSPORTS") == "direct"
        if (backend == "nccl" or rehearse) and os.environ.get("DCCL_BENCH_NO_COLLECTIVE", "0") != "1":
            torch.cuda.empty_cache()
            extra["dccl_allreduce"] = collective_in_child(world, rank, local, backend,
                                                          a.c5_gib if backend == "nccl" else min(a.c5_gib, 1.0))

    if rank == 0:
        traffic, traffic_detail = None, None
        if world == 1 and not a.no_pmc:
            progress("rocprofv3 --pmc passes for roofline.traffic")
            traffic_detail = measured_traffic(nbytes, dt, op)
            traffic = traffic_detail.get("hbm_bytes_per_launch")
        achieved = 3 * nbytes / (kern_ms * 1e-3) / 1e9
        # Key order: the contract keys, then the bulky legs (c4, c3, host_staged, the full collective
        # record), then the compact evidence LAST, so that a reader that keeps only the line's tail still
        # sees roofline, cpu_baseline, other_layout, c5, the collective flags and `verified`.
        res = {
            "metric": "device-resident reduce GiB/s (ncclSum fp32, 1 GiB) at 1/2/4/8 GPU vs HBM peak",
            "value": round(3 * total_bytes / (ms_per_step * 1e-3) / GIB, 2),
            "unit": "GiB/s (HBM traffic 3*N*sizeof per combine, summed over GPUs)",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
            "dtype": {0: "i8", 1: "u8", 2: "i32", 3: "u32", 4: "i64", 5: "u64", 6: "f16", 7: "f32", 8: "f64",
                      9: "bf16"}[dt],
            "data": f"synthetic (device splitmix64 counter generator, seed 0xDCC1, uniform [-1,1) operands resident in HBM, {a.layout} layout)",
            "config": {"workload": (f"C5: {a.total_gib:g} GiB per operand sharded over {world} GPU(s), "
                                    f"in-place combine recv=op(recv,send), {a.op}") if strong else
                                   (f"in-place two-buffer combine recv=op(recv,send), {a.op}, "
                                    f"{a.mib} MiB per operand per GPU (BASELINE metric / config C3)"),
                       "bytes_per_operand_per_gpu": nbytes, "bytes_per_operand_total": total_bytes,
                       "op": a.op, "parallelism": f"shard x{world}"},
            "payload_gib_s": round(total_bytes / (ms_per_step * 1e-3) / GIB, 2),
        }
        if world > torch.cuda.device_count():
            res["rehearsal"] = (f"{world} ranks on {torch.cuda.device_count()} GPU(s), torch.distributed backend "
                                f"{backend}: a functional rehearsal, the rates are not scaling numbers")
        if world == 1 and not a.no_configs:
            progress("C4: size sweep 4 KiB - 4 GiB")
            res["c4"] = config_c4(dev, stream)
            if c3 is None:
                progress("C3: ops x dtypes at 1 GiB")
                c3 = config_c3(dev, stream)
            res["c3"] = c3
            progress("ring step: scratchpad + user chunk, 512 MiB - 8 MiB")
            extra["ring_step"] = ring_step(dev, stream)
        if world == 1 and not a.no_host_staged:
            progress("host-resident operands: GPU path vs the CPU loop, 4 KiB - 1 GiB")
            try:
                hc = host_crossover()
            except Exception as e:  # reported, never fatal to the line
                hc = {"error": repr(e)}
            top = hc["rows"][-1] if "rows" in hc else {"bytes": None, "pinned": {}, "pageable": {}, "registered": {}}
            res["host_staged"] = {"payload_gib_s": top["pinned"].get("gpu_payload_gib_s"),
                                  "ms": round(top["pinned"].get("gpu_us", 0) / 1e3, 3), "bytes_per_operand": top["bytes"],
                                  "pageable_payload_gib_s": top["pageable"].get("gpu_payload_gib_s"),
                                  "registered_payload_gib_s": top["registered"].get("gpu_payload_gib_s"),
                                  "note": "fp32 Sum, pinned host operands; PCIe H2D 2N + D2H N bytes "
                                          "(the 1 GiB row of host_crossover)"}
            res["host_crossover"] = hc
        if "allgather" in extra:
            res["allgather"] = extra["allgather"]
        if "dccl_allreduce" in extra:
            res["dccl_allreduce"] = extra["dccl_allreduce"]
        res["traffic_measurement"] = traffic_detail
        res["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                           "kernel": "reduce_vec_kernel (dccl_local_reduce)",
                           "kernel_ms_avg": round(kern_ms, 4), "kernel_ms_max_rank": round(kern_ms_max, 4),
                           "bytes_per_launch": 3 * nbytes, "operand_layout": a.layout}
        if world == 1 and not a.no_cpu:
            progress("CPU baseline")
            res["cpu_baseline"] = cpu_baseline(a.cpu_seconds, nbytes)
        for key in ("other_layout", "ring_step", "c5"):
            if key in extra:
                res[key] = extra[key]
        if "dccl_allreduce" in extra:
            res["dccl_allreduce_summary"] = allreduce_summary(extra["dccl_allreduce"])
        res["verified"] = ok
        print(json.dumps(res), flush=True)
    if world > 1:
        try:
            dist.barrier()
            dist.destroy_process_group()
        except Exception:  # a peer left early after printing its part; the line is out
            os._exit(0)


def launcher_selftest() -> None:
    """Test aid (tests/test_bench_launcher.py): what a rank started by launch_ranks sees, over gloo on the
    CPU, without touching the GPU or the HIP library."""
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([rank], dtype=torch.int64)
    hostids = [os.environ.get("NCCL_HOSTID")]
    if world > 1:
        dist.all_reduce(t)
        hostids = [None] * world
        dist.all_gather_object(hostids, os.environ.get("NCCL_HOSTID"))
    if rank == 0:
        print(json.dumps({"n_gpus": world, "rank_sum": int(t[0]), "local_rank": os.environ.get("LOCAL_RANK"),
                          "nccl_hostids": hostids,
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if os.environ.get("DCCL_BENCH_SELFTEST_FAIL_RANK") == str(rank):
        sys.exit(7)


def main():
    if "--collective-child" in sys.argv:
        collective_child()
        return
    argv = sys.argv[1:]
    a = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if a.gpus > 1:
            sys.exit(launch_ranks(a, argv))
        if a.gpus < 1:
            print(f"bench.py: --gpus {a.gpus} must be >= 1", file=sys.stderr)
            sys.exit(2)
    elif int(env_world) != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={env_world} (one process per GPU: launch "
              f"--nproc-per-node {a.gpus}, or run without a launcher and let bench.py start the ranks)",
              file=sys.stderr)
        sys.exit(2)
    if a.launcher_selftest:
        launcher_selftest()
        return
    run_rank(a)


if __name__ == "__main__":
    main()
