#!/usr/bin/env python3
"""Tuning only: does the allocation call decide the DRAM placement mode of the 1 GiB fp32 Sum combine?
Two shapes, fresh allocations per sample, variants interleaved within each round, HIP events:
  pooled    recv, then send 4 KiB past its end, in ONE allocation of 2 GiB + 4 KiB (the bench's headline)
  separate  send and recv in two allocations of 1 GiB (DCCL's scratchpad + user chunk)
allocated by:
  torch      torch.empty (hipMalloc through torch's caching allocator)
  hipmalloc  hipExtMallocWithFlags(flags 0) directly
  contig     hipExtMallocWithFlags(hipDeviceMallocContiguous)
  vmm1       one HIP VMM physical allocation (hipMemCreate) mapped whole
    python tools/alloc_probe.py [--samples 3] [--rounds 5] [--out f.json]
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

LIB = os.path.join(ROOT, "tools", "lib", "libscratch_vmm.so")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--samples", type=int, default=3)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--launches", type=int, default=20)
    p.add_argument("--out", default="")
    a = p.parse_args()
    dccl = bench._native()
    lib = ctypes.CDLL(LIB)
    lib.ext_alloc.argtypes = [ctypes.c_size_t, ctypes.c_uint, ctypes.POINTER(ctypes.c_void_p)]
    lib.ext_free.argtypes = [ctypes.c_void_p]
    lib.vmm_alloc.argtypes = [ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    lib.vmm_free.argtypes = [ctypes.c_void_p]
    stream = torch.cuda.current_stream()
    nb = 1 << 30
    n = nb // 4
    keep = []

    def alloc(kind, size):
        if kind == "torch":
            t = torch.empty(size, dtype=torch.uint8, device="cuda")
            keep.append(t)
            return t.data_ptr(), None
        ptr = ctypes.c_void_p()
        if kind == "vmm1":
            assert lib.vmm_alloc(size, 2 << 20, 3, ctypes.byref(ptr)) == 0
            return ptr.value, lambda: lib.vmm_free(ptr)
        flags = {"hipmalloc": 0, "contig": 4}[kind]
        rc = lib.ext_alloc(size, flags, ctypes.byref(ptr))
        assert rc == 0, (kind, rc)
        return ptr.value, lambda: lib.ext_free(ptr)

    kinds = ["torch", "hipmalloc", "contig", "vmm1"]
    res = {"bytes_per_operand": nb, "samples": a.samples, "rounds": a.rounds, "launches": a.launches, "shapes": {}}
    for shape in ("pooled", "separate"):
        per = {k: [] for k in kinds}
        for smp in range(a.samples):
            pairs, frees = {}, []
            for k in kinds:
                if shape == "pooled":
                    base, f = alloc(k, 2 * nb + 4096)
                    frees.append(f)
                    pr, ps = base, base + nb + 4096
                else:
                    ps, f1 = alloc(k, nb)
                    pr, f2 = alloc(k, nb)
                    frees += [f1, f2]
                dccl.check(dccl.synth_fill(ps, 7, n, 0, bench.SEED, 0, stream.cuda_stream), "synth")
                dccl.check(dccl.synth_fill(pr, 7, n, 0, bench.SEED, 1, stream.cuda_stream), "synth")
                pairs[k] = [(ps, pr)]
            t = {k: [] for k in kinds}
            for _ in range(a.rounds):
                for k in kinds:
                    t[k].append(bench._time_pairs(pairs[k], n, stream, a.launches))
            for k in kinds:
                per[k].append(round(3 * nb / (statistics.median(t[k]) * 1e-3) / 1e9 / bench.HBM_PEAK_GBS, 4))
            print(f"{shape} sample {smp}: " + "  ".join(f"{k} {100 * per[k][-1]:.2f}%" for k in kinds), flush=True)
            torch.cuda.synchronize()
            for f in frees:
                if f is not None:
                    assert f() == 0
            keep.clear()
            torch.cuda.empty_cache()
        res["shapes"][shape] = {k: {"per_sample": v, "median": statistics.median(v), "min": min(v), "max": max(v)}
                                for k, v in per.items()}
        print(shape + " median: " + "  ".join(f"{k} {100 * statistics.median(v):.2f}%" for k, v in per.items()),
              flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
