#!/usr/bin/env python3
"""Can an allocation be exported while a peer still maps a freed allocation at the same address?

Two processes on one GPU, HIP runtime calls through ctypes:
  A: hipMalloc X, hipIpcGetMemHandle(X) -> B opens it (hipIpcOpenMemHandle) and keeps it open.
  A: hipFree X, hipMalloc Y of the same size (the same address in practice), hipIpcGetMemHandle(Y)
     -> reported: its result, whether Y's handle bytes equal X's, whether Y has X's address.
  B: hipIpcCloseMemHandle(X's mapping);  A: hipIpcGetMemHandle(Y) again -> reported.
  B: opens Y's handle, reads it back (hipMemcpy D2H) and checks A's fill pattern.
One JSON line on stdout.

    python tools/ipc_reexport_probe.py [MiB]
"""
import ctypes
import json
import multiprocessing as mp
import sys


class Handle(ctypes.Structure):  # hipIpcMemHandle_t, passed BY VALUE to hipIpcOpenMemHandle
    _fields_ = [("reserved", ctypes.c_char * 64)]


def _hip():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), Handle, ctypes.c_uint]
    return hip


def _open(hip, raw, out):
    h = Handle()
    ctypes.memmove(ctypes.addressof(h), raw, 64)
    return hip.hipIpcOpenMemHandle(ctypes.byref(out), h, 1)  # hipIpcMemLazyEnablePeerAccess


def _handle(hip, p):
    h = ctypes.create_string_buffer(64)
    rc = hip.hipIpcGetMemHandle(h, p)
    return rc, h.raw


def exporter(nbytes, conn):
    hip = _hip()
    x = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(x), ctypes.c_size_t(nbytes)) == 0
    assert hip.hipMemset(x, 1, ctypes.c_size_t(nbytes)) == 0
    rc, hx = _handle(hip, x)
    conn.send(("X", rc, hx))
    conn.recv()  # B mapped X
    assert hip.hipFree(x) == 0
    y = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(y), ctypes.c_size_t(nbytes)) == 0
    assert hip.hipMemset(y, 7, ctypes.c_size_t(nbytes)) == 0
    assert hip.hipDeviceSynchronize() == 0
    rc1, hy1 = _handle(hip, y)
    out = {"x_addr": hex(x.value), "y_addr": hex(y.value), "same_address": x.value == y.value,
           "export_while_peer_maps_old_rc": rc1, "handle_bytes_equal_old": hy1 == hx}
    conn.send(("ask_close", None, None))
    conn.recv()  # B closed X's mapping
    rc2, hy2 = _handle(hip, y)
    out["export_after_peer_closed_rc"] = rc2
    out["handle_after_close_equal_old"] = hy2 == hx
    conn.send(("Y", rc2, hy2 if rc2 == 0 else hy1))
    out["peer_read"] = conn.recv()
    conn.send(("done", None, out))
    conn.recv()
    hip.hipFree(y)


def importer(nbytes, conn):
    hip = _hip()
    _, rc, hx = conn.recv()
    px = ctypes.c_void_p()
    orc = _open(hip, hx, px) if rc == 0 else -1
    conn.send(orc)
    conn.recv()  # ask_close
    crc = hip.hipIpcCloseMemHandle(px) if orc == 0 else -1
    conn.send(crc)
    _, rc2, hy = conn.recv()
    py = ctypes.c_void_p()
    orc2 = _open(hip, hy, py)
    res = {"open_rc": orc2}
    if orc2 == 0:
        buf = (ctypes.c_ubyte * 4096)()
        res["memcpy_rc"] = hip.hipMemcpy(buf, py, ctypes.c_size_t(4096), 2)  # hipMemcpyDeviceToHost
        res["reads_new_fill"] = all(b == 7 for b in buf)
        res["reads_old_fill"] = all(b == 1 for b in buf)
        hip.hipIpcCloseMemHandle(py)
    conn.send(res)
    _, _, out = conn.recv()
    conn.send(None)
    print(json.dumps({"mib": nbytes >> 20, "close_old_rc": crc, **out}), flush=True)


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    ctx = mp.get_context("spawn")
    a, b = ctx.Pipe()
    pa = ctx.Process(target=exporter, args=(mib << 20, a))
    pb = ctx.Process(target=importer, args=(mib << 20, b))
    pa.start()
    pb.start()
    pa.join(120)
    pb.join(120)
    for p in (pa, pb):
        if p.is_alive():
            p.kill()
    sys.exit(0 if pa.exitcode == 0 and pb.exitcode == 0 else 1)


if __name__ == "__main__":
    main()
