#!/usr/bin/env python3
"""What a hipIpcMemHandle_t holds across free / re-allocation (the IPC mapping cache).

Allocates a buffer with hipMalloc, takes its IPC handle and buffer id, frees it, allocates another of the same
size (and one of another size) and prints, per allocation: the address, HIP_POINTER_ATTRIBUTE_BUFFER_ID and the
handle bytes, plus whether the handle bytes repeat.  One JSON line on stdout.

    python tools/ipc_handle_probe.py [MiB]
    python tools/ipc_handle_probe.py --torch     (torch allocations freed with empty_cache between rounds)
"""
import ctypes
import json
import sys

hip = ctypes.CDLL("libamdhip64.so")
HIP_POINTER_ATTRIBUTE_BUFFER_ID = 7  # driver_types.h: hipPointer_attribute


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with {rc}")


def alloc(nbytes):
    p = ctypes.c_void_p()
    check(hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes)), "hipMalloc")
    h = ctypes.create_string_buffer(64)
    check(hip.hipIpcGetMemHandle(h, p), "hipIpcGetMemHandle")
    bid = ctypes.c_uint64()
    check(hip.hipPointerGetAttribute(ctypes.byref(bid), HIP_POINTER_ATTRIBUTE_BUFFER_ID, p), "hipPointerGetAttribute")
    return p, {"addr": hex(p.value), "buffer_id": bid.value, "handle": h.raw.hex()}


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 256
    nb = mib << 20
    rows = []
    p, row = alloc(nb)
    rows.append({"what": f"first {mib} MiB", **row})
    check(hip.hipFree(p), "hipFree")
    p, row = alloc(nb)
    rows.append({"what": f"after free, {mib} MiB again", **row})
    q, row = alloc(nb)
    rows.append({"what": f"second live {mib} MiB", **row})
    check(hip.hipFree(p), "hipFree")
    r, row = alloc(2 * nb)
    rows.append({"what": f"after free, {2 * mib} MiB", **row})
    check(hip.hipFree(q), "hipFree")
    check(hip.hipFree(r), "hipFree")
    handles = [x["handle"] for x in rows]
    print(json.dumps({"rows": rows, "first_handle_repeats_after_free": handles[0] == handles[1],
                      "any_handle_repeats": len(set(handles)) < len(handles)}))


if __name__ == "__main__" and "--torch" not in sys.argv:
    main()


def torch_rounds(mib=64, rounds=6):
    """The same through torch's caching allocator, as tests/test_direct.py::test_ipc_reallocated_buffers
    allocates: per round an input of `mib` MiB and an output 4x that, both freed back to the driver
    (torch.cuda.empty_cache) before the next round."""
    import torch
    out_rows = []
    for k in range(rounds):
        a = torch.empty(mib << 20, dtype=torch.uint8, device="cuda")
        b = torch.empty(4 * mib << 20, dtype=torch.uint8, device="cuda")
        for name, t in (("in", a), ("out", b)):
            h = ctypes.create_string_buffer(64)
            check(hip.hipIpcGetMemHandle(h, ctypes.c_void_p(t.data_ptr())), "hipIpcGetMemHandle")
            bid = ctypes.c_uint64()
            check(hip.hipPointerGetAttribute(ctypes.byref(bid), HIP_POINTER_ATTRIBUTE_BUFFER_ID,
                                             ctypes.c_void_p(t.data_ptr())), "hipPointerGetAttribute")
            out_rows.append({"round": k, "buf": name, "addr": hex(t.data_ptr()), "buffer_id": bid.value,
                             "handle": h.raw.hex()})
        del a, b
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    hs = [r["handle"] for r in out_rows]
    return {"rows": out_rows, "distinct_handles": len(set(hs)), "handles": len(hs)}


if __name__ == "__main__" and "--torch" in sys.argv:
    print(json.dumps(torch_rounds()))
