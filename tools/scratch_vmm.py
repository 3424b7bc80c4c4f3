#!/usr/bin/env python3
"""Tuning only: does the way the library allocates its device scratchpad move DCCL's ring-step
combine between the DRAM's fast and slow modes?  bench.py's `ring_step` shape (send = a library scratch slot,
recv = chunk (2j+1) of a separately allocated 2 GiB user buffer, fp32 Sum), eager back-to-back launches, HIP
events, at 512 / 256 / 128 MiB per operand, on three separate user buffers, with the scratch from:
  hipmalloc    torch.empty (hipMalloc through torch's allocator: today's library scratch)
  vmm_seq      HIP VMM (hipMemAddressReserve + hipMemCreate + hipMemMap) in 2 MiB granules, mapped in creation order
  vmm_rev      the same granules mapped in reverse order
  vmm_inter    created in order, mapped as two interleaved halves (even slots, then odd slots)
  vmm_single   one physical allocation of the whole scratch
A fresh scratch of every variant per user buffer; variants interleaved within each of --rounds rounds; the median
per (variant, size, user buffer) is reported, then the median over user buffers.

    python tools/scratch_vmm.py [--rounds 5] [--out gpurun_out/scratch_vmm.json]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import dccl_amd  # noqa: E402

LIB = os.path.join(ROOT, "tools", "lib", "libscratch_vmm.so")
VARIANTS = {"hipmalloc": None, "vmm_seq": 0, "vmm_rev": 1, "vmm_inter": 2, "vmm_single": 3}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--users", type=int, default=3)
    p.add_argument("--sizes", default="512,256,128")
    p.add_argument("--out", default="")
    a = p.parse_args()
    bench._native()
    vmm = ctypes.CDLL(LIB)
    vmm.vmm_alloc.argtypes = [ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    vmm.vmm_free.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    user_bytes = 2 << 30
    users, fillers = [], []
    for u in range(a.users):  # separate allocations with different neighbours
        fillers.append(torch.empty((u + 1) * (96 << 20), dtype=torch.uint8, device=dev))
        t = torch.empty(user_bytes, dtype=torch.uint8, device=dev)
        bench.synth_into(t.view(torch.float32), user_bytes // 4, 7, 0, 40 + u)
        users.append(t)
    res = {"shape": "send = scratch slot, recv = chunk (2j+1) of a separate 2 GiB user buffer, fp32 Sum, eager",
           "rounds": a.rounds, "users": a.users, "points": []}
    for mib in [int(x) for x in a.sizes.split(",")]:
        nb = mib << 20
        n = nb // 4
        sets = 1 if 2 * nb >= (512 << 20) else max(2, -(-(512 << 20) // (2 * nb)))
        per_user = []
        for u, user in enumerate(users):
            scratches, keep = {}, []
            for name, order in VARIANTS.items():
                if order is None:
                    t = torch.empty(sets * nb, dtype=torch.uint8, device=dev)
                    keep.append(t)
                    base = t.data_ptr()
                else:
                    ptr = ctypes.c_void_p()
                    rc = vmm.vmm_alloc(sets * nb, 2 << 20, order, ctypes.byref(ptr))
                    assert rc == 0, (name, rc)
                    base = ptr.value
                dccl_amd.check(dccl_amd.synth_fill(base, 7, sets * n, 0, bench.SEED, 41,
                                                   stream.cuda_stream), "synth")
                scratches[name] = (base, order)
            pairs = {name: [(b + j * nb, user.data_ptr() + ((2 * j + 1) * nb) % user_bytes) for j in range(sets)]
                     for name, (b, _) in scratches.items()}
            times = {name: [] for name in scratches}
            k0 = bench._time_pairs(pairs["hipmalloc"], n, stream, 5)
            launches = int(min(400, max(10, 20.0 / max(k0, 1e-4))))
            for _ in range(a.rounds):
                for name in scratches:
                    times[name].append(bench._time_pairs(pairs[name], n, stream, launches))
            row = {name: round(3 * nb / (statistics.median(v) * 1e-3) / 1e9 / bench.HBM_PEAK_GBS, 4)
                   for name, v in times.items()}
            per_user.append(row)
            print(f"{mib} MiB user {u}: " + "  ".join(f"{k} {100 * v:.1f}%" for k, v in row.items()), flush=True)
            torch.cuda.synchronize()
            for name, (b, order) in scratches.items():
                if order is not None:
                    assert vmm.vmm_free(ctypes.c_void_p(b)) == 0
            del keep
            torch.cuda.empty_cache()
        med = {name: round(statistics.median(r[name] for r in per_user), 4) for name in VARIANTS}
        res["points"].append({"mib": mib, "sets": sets, "per_user": per_user, "median_over_users": med,
                              "gain_points_vs_hipmalloc": {k: round(100 * (v - med["hipmalloc"]), 2)
                                                           for k, v in med.items()}})
        print(f"{mib} MiB median: " + "  ".join(f"{k} {100 * v:.1f}%" for k, v in med.items()), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
