#!/usr/bin/env python3
"""Host-operand combine, two staging strategies side by side (tuning only): dccl_local_reduce_host (zero-copy
up to 16 MiB, then the 3-stream DMA pipeline with bounced pageable chunks) against
dccl_local_reduce_chain_host with one send (zero-copy kernels over double-buffered pinned staging),
pageable and page-locked fp32 operands, payload GiB/s.
    python tools/host_path_probe.py [--out f.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (initialises HIP the way the other tools do)
import dccl_amd  # noqa: E402


def rate(fn, nbytes, budget=1.0):
    fn()
    reps, t0 = 0, time.perf_counter()
    while reps < 3 or time.perf_counter() - t0 < budget:
        assert fn() == 0
        reps += 1
    t = (time.perf_counter() - t0) / reps
    return round(nbytes / t / 2**30, 2), round(t * 1e3, 3)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--out", default="")
    a = p.parse_args()
    rows = []
    for mib in (16, 64, 256, 1024):
        n = (mib << 20) // 4
        s = np.random.default_rng(1).standard_normal(n).astype(np.float32)
        r = np.zeros(n, np.float32)
        for pinned in (False, True):
            if pinned:
                for x in (s, r):
                    assert dccl_amd.register_host_memory(x.ctypes.data, x.nbytes) == 0
            for name, fn in (("local_reduce_host", lambda: dccl_amd.local_reduce_host(s.ctypes.data, r.ctypes.data, 7, n, 0)),
                             ("chain_host_1", lambda: dccl_amd.local_reduce_chain_host([s.ctypes.data], r.ctypes.data,
                                                                                       r.ctypes.data, 7, n, 0))):
                gib, ms = rate(fn, n * 4)
                rows.append({"mib": mib, "pinned": pinned, "path": name, "payload_gib_s": gib, "ms": ms})
                print(json.dumps(rows[-1]), flush=True)
            if pinned:
                for x in (s, r):
                    dccl_amd.deregister_host_memory(x.ctypes.data)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
