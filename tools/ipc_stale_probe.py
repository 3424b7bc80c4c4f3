#!/usr/bin/env python3
"""Does a peer read through a fresh IPC mapping ever see an earlier allocation's data?

Two processes on one GPU.  Every round the exporter allocates S bytes (hipMalloc), fills them with the round's
pattern (hipMemsetD32), synchronises and sends the IPC handle; the importer opens it, copies the bytes out
with this build's copy kernel (dccl_copy_multi, the kernel of the direct all-gather), closes the mapping and
checks every 128-B line against the round's pattern; then the exporter frees the allocation, so the next
round's allocation usually lands on the same physical pages.  Reported: rounds, rounds with any wrong line,
wrong lines, and for wrong lines whether they hold an earlier round's pattern.  One JSON line on stdout.

    python tools/ipc_stale_probe.py [--rounds 2000] [--mib 2] [--keep-mapping]

--keep-mapping: the importer closes round k's mapping only after opening round k+1's (the cache's order).
"""
import argparse
import ctypes
import json
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class Handle(ctypes.Structure):  # hipIpcMemHandle_t, passed BY VALUE to hipIpcOpenMemHandle
    _fields_ = [("reserved", ctypes.c_char * 64)]


def _hip():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), Handle, ctypes.c_uint]
    return hip


def exporter(a, conn):
    hip = _hip()
    nbytes = a.mib << 20
    for k in range(a.rounds):
        x = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(x), ctypes.c_size_t(nbytes)) == 0
        assert hip.hipMemsetD32(x, ctypes.c_int(0x5A000000 + k), ctypes.c_size_t(nbytes // 4)) == 0
        assert hip.hipDeviceSynchronize() == 0
        h = ctypes.create_string_buffer(64)
        assert hip.hipIpcGetMemHandle(h, x) == 0
        conn.send(h.raw)
        conn.recv()  # the importer has read it
        assert hip.hipFree(x) == 0
    conn.send(None)


def importer(a, conn, q):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    import dccl_amd
    hip = _hip()
    nbytes = a.mib << 20
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    bad_rounds, bad_lines, old_lines, k, prev = 0, 0, 0, 0, None
    while True:
        raw = conn.recv()
        if raw is None:
            break
        h = Handle()
        ctypes.memmove(ctypes.addressof(h), raw, 64)
        p = ctypes.c_void_p()
        assert hip.hipIpcOpenMemHandle(ctypes.byref(p), h, 1) == 0
        if prev is not None:
            assert hip.hipIpcCloseMemHandle(prev) == 0
            prev = None
        dst.zero_()
        torch.cuda.synchronize()
        assert dccl_amd.copy_multi([p.value], [dst.data_ptr()], nbytes, st) == 0
        torch.cuda.synchronize()
        if a.keep_mapping:
            prev = p
        else:
            assert hip.hipIpcCloseMemHandle(p) == 0
        conn.send(True)
        words = dst.view(torch.int32).cpu().numpy().reshape(-1, 32)  # 128-B lines
        wrong = np.any(words != np.int32(0x5A000000 + k), axis=1)
        if wrong.any():
            bad_rounds += 1
            bad_lines += int(wrong.sum())
            vals = words[wrong][:, 0]
            old_lines += int(np.sum((vals >= 0x5A000000) & (vals < 0x5A000000 + k)))
        k += 1
    if prev is not None:
        hip.hipIpcCloseMemHandle(prev)
    q.put({"rounds": k, "mib": a.mib, "keep_mapping": a.keep_mapping, "rounds_with_wrong_lines": bad_rounds,
           "wrong_lines": bad_lines, "wrong_lines_with_an_earlier_rounds_pattern": old_lines,
           "lines_per_round": nbytes // 128})


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=2000)
    p.add_argument("--mib", type=int, default=2)
    p.add_argument("--keep-mapping", action="store_true")
    a = p.parse_args()
    ctx = mp.get_context("spawn")
    c1, c2 = ctx.Pipe()
    q = ctx.Queue()
    pe = ctx.Process(target=exporter, args=(a, c1))
    pi = ctx.Process(target=importer, args=(a, c2, q))
    pe.start()
    pi.start()
    res = q.get(timeout=600)
    pe.join(60)
    pi.join(60)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
