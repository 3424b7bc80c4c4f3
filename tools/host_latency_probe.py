#!/usr/bin/env python3
"""Host-path latency pieces (tuning only): hipPointerGetAttributes on pageable memory, one host combine, one
host chain combine (3 sends), one device combine + synchronise; 1 KiB fp32 operands, microseconds per call."""
import ctypes, time, sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch, dccl_amd
torch.cuda.init()
hip = ctypes.CDLL("libamdhip64.so.7")
n = 256
a = [np.ones(n, np.float32) for _ in range(4)]
def t(fn, reps=2000):
    for _ in range(50): fn()
    t0 = time.perf_counter()
    for _ in range(reps): fn()
    return (time.perf_counter() - t0) / reps * 1e6
attr = (ctypes.c_char * 256)()
print("hipPointerGetAttributes pageable us", t(lambda: hip.hipPointerGetAttributes(attr, ctypes.c_void_p(a[0].ctypes.data))))
print("hipGetLastError us", t(lambda: hip.hipGetLastError()))
print("local_reduce_host 1KiB us", t(lambda: dccl_amd.local_reduce_host(a[0].ctypes.data, a[1].ctypes.data, 7, n, 0)))
print("chain_host 3 sends 1KiB us", t(lambda: dccl_amd.local_reduce_chain_host([x.ctypes.data for x in a[:3]], a[3].ctypes.data, a[3].ctypes.data, 7, n, 0)))
d = torch.ones(n, device="cuda"); e = torch.ones(n, device="cuda")
st = torch.cuda.current_stream().cuda_stream
def dev_sync():
    dccl_amd.local_reduce(d.data_ptr(), e.data_ptr(), 7, n, 0, st); torch.cuda.synchronize()
print("device combine + sync us", t(dev_sync))
