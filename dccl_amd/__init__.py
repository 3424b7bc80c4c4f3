"""dccl_amd — MI355X-native DCCL local bucket-reduction combine.

Python binding of the C-ABI in ``include/dccl/dccl_reduce.h`` (ctypes; plain pointers,
sizes and enum integers).  The combine itself is hand-written HIP for gfx950 inside
``dccl_amd/lib/libdccl_amd.so``; there is no CPU fallback: if the shared library is
missing, importing this package raises.

Enum values are those of the reference's public header
(/root/reference/include/dccl/dccl.hpp:59-112), with ncclBfloat16 = 9 always present.
"""
from __future__ import annotations

import ctypes
import enum
import os

try:  # share torch's HIP runtime (same soname libamdhip64.so.7) when torch is around
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is plumbing only
    torch = None

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "lib", "libdccl_amd.so")


class ncclResult_t(enum.IntEnum):
    ncclSuccess = 0
    ncclUnhandledCudaError = 1
    ncclSystemError = 2
    ncclInternalError = 3
    ncclInvalidArgument = 4
    ncclInvalidUsage = 5
    ncclRemoteError = 6
    ncclInProgress = 7


class ncclDataType_t(enum.IntEnum):
    ncclInt8 = 0
    ncclUint8 = 1
    ncclInt32 = 2
    ncclUint32 = 3
    ncclInt64 = 4
    ncclUint64 = 5
    ncclFloat16 = 6
    ncclFloat32 = 7
    ncclFloat64 = 8
    ncclBfloat16 = 9


class ncclRedOp_t(enum.IntEnum):
    ncclSum = 0
    ncclProd = 1
    ncclMax = 2
    ncclMin = 3
    ncclAvg = 4


ALL_DTYPES = list(ncclDataType_t)
ALL_OPS = [ncclRedOp_t.ncclSum, ncclRedOp_t.ncclProd, ncclRedOp_t.ncclMax, ncclRedOp_t.ncclMin]

DTYPE_NAMES = {
    "int8": 0, "uint8": 1, "int32": 2, "uint32": 3, "int64": 4, "uint64": 5,
    "float16": 6, "float32": 7, "float64": 8, "bfloat16": 9,
}
OP_NAMES = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}


class DcclError(RuntimeError):
    def __init__(self, code: int, what: str):
        self.code = code
        super().__init__(f"{what} failed: {code} ({result_string(code)})")


#: dccl_p2p_exchange_fn of include/dccl/dccl_comm.h
P2P_EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                   ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p)


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"dccl_amd: native library {LIB_PATH} is missing; build it with "
            "`python dccl_amd/build.py` (hipcc, gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    c_int, c_size_t, c_void_p = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p
    sig = {
        "dccl_local_reduce": (c_int, [c_void_p, c_void_p, c_int, c_size_t, c_int, c_void_p]),
        "dccl_local_reduce_multi": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_int, c_size_t,
                                            c_int, c_void_p]),
        "dccl_local_reduce_host": (c_int, [c_void_p, c_void_p, c_int, c_size_t, c_int]),
        "dccl_local_reduce_chain": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_void_p, c_int, c_size_t,
                                            c_int, c_void_p]),
        "dccl_local_reduce_chain_host": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_void_p, c_int,
                                                 c_size_t, c_int]),
        "dccl_copy_multi": (c_int, [ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p), c_int, c_size_t, c_void_p]),
        "dccl_register_host_memory": (c_int, [c_void_p, c_size_t]),
        "dccl_deregister_host_memory": (c_int, [c_void_p]),
        "dccl_size_of_type": (c_size_t, [c_int]),
        "dccl_host_reduce_gpu_min_bytes": (c_size_t, [c_int]),
        "dccl_result_string": (ctypes.c_char_p, [c_int]),
        "dccl_version": (c_int, []),
    }
    sig.update({
        "dccl_comm_init_rank": (c_int, [ctypes.POINTER(c_void_p), ctypes.c_uint32, ctypes.c_uint32]),
        "dccl_get_unique_id": (c_int, [c_void_p]),
        "dccl_comm_init_rccl": (c_int, [ctypes.POINTER(c_void_p), ctypes.c_uint32, ctypes.c_uint32, c_void_p]),
        "dccl_comm_finalize": (c_int, [c_void_p]),
        "dccl_comm_init_ipc": (c_int, [ctypes.POINTER(c_void_p), ctypes.c_uint32, ctypes.c_uint32]),
        "dccl_comm_init_p2p": (c_int, [ctypes.POINTER(c_void_p), ctypes.c_uint32, ctypes.c_uint32, P2P_EXCHANGE_FN,
                                       c_void_p, c_int]),
        "dccl_reduce": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_int, c_int, c_void_p, c_void_p]),
        "dccl_broadcast": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_int, c_void_p, c_void_p]),
        "dccl_all_reduce": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_int, c_void_p, c_void_p]),
        "dccl_reduce_scatter": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_int, c_void_p, c_void_p]),
        "dccl_all_gather": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_void_p, c_void_p]),
        "dccl_rccl_available": (c_int, []),
        "dccl_bootstrap_unique_id": (c_int, [ctypes.c_uint32, ctypes.c_uint32, c_void_p]),
        "dccl_bootstrap_done": (c_int, [ctypes.c_uint32, ctypes.c_uint32]),
        "dccl_comm_register": (c_int, [c_void_p, c_void_p, c_size_t]),
        "dccl_comm_deregister": (c_int, [c_void_p, c_void_p]),
        "dccl_ipc_stats": (c_int, [ctypes.POINTER(ctypes.c_uint64), c_int]),
        "dccl_synth_fill": (c_int, [c_void_p, c_int, c_size_t, c_int, ctypes.c_uint64, ctypes.c_uint64, c_void_p]),
        "dccl_synth_fill_range": (c_int, [c_void_p, c_int, c_size_t, c_int, ctypes.c_uint64, ctypes.c_uint64,
                                          c_size_t, c_void_p]),
    })
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()

#: every symbol the C-ABI headers declare (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = [
    "dccl_local_reduce", "dccl_local_reduce_multi", "dccl_local_reduce_host",
    "dccl_register_host_memory", "dccl_deregister_host_memory", "dccl_size_of_type",
    "dccl_result_string", "dccl_version",
    "dccl_comm_init_rank", "dccl_get_unique_id", "dccl_comm_init_rccl", "dccl_comm_finalize", "dccl_all_reduce",
    "dccl_reduce_scatter", "dccl_all_gather", "dccl_rccl_available", "dccl_bootstrap_unique_id",
    "dccl_synth_fill", "dccl_synth_fill_range", "dccl_local_reduce_chain", "dccl_copy_multi",
    "dccl_comm_init_ipc", "dccl_reduce", "dccl_broadcast", "dccl_local_reduce_chain_host", "dccl_comm_init_p2p",
    "dccl_bootstrap_done", "dccl_comm_register", "dccl_comm_deregister", "dccl_ipc_stats",
    "dccl_host_reduce_gpu_min_bytes",
]

#: names of the dccl_ipc_stats counters, in order (include/dccl/dccl_comm.h); registered_hits,
#: stale_registrations and registered_fallbacks counted the registered in-place path removed in round 5 (always 0)
IPC_STAT_NAMES = [
    "exports_made", "exports_retired", "registered_hits", "scratch_copies", "scratch_bytes", "scratch_grows",
    "stale_registrations", "mappings_opened", "mappings_reused", "mappings_retired", "retire_log_overflows",
    "mappings_trimmed", "alias_evictions", "alias_errors", "open_retries", "size_mismatches", "mappings_open",
    "bytes_mapped", "recycled_handles", "registered_fallbacks", "verify_failures",
]


def ipc_stats() -> dict:
    """This process's IPC transport counters (dccl_ipc_stats) by name."""
    buf = (ctypes.c_uint64 * len(IPC_STAT_NAMES))()
    n = int(lib.dccl_ipc_stats(buf, len(IPC_STAT_NAMES)))
    assert n == len(IPC_STAT_NAMES), (n, len(IPC_STAT_NAMES))
    return dict(zip(IPC_STAT_NAMES, (int(v) for v in buf)))


def result_string(code: int) -> str:
    return lib.dccl_result_string(int(code)).decode()


def size_of_type(dtype: int) -> int:
    return int(lib.dccl_size_of_type(int(dtype)))


def version() -> int:
    return int(lib.dccl_version())


def local_reduce(send_ptr: int, recv_ptr: int, dtype: int, count: int, op: int, stream: int = 0) -> int:
    """Device combine recv = op(recv, send); returns the ncclResult_t code (no raise)."""
    return int(lib.dccl_local_reduce(send_ptr, recv_ptr, int(dtype), int(count), int(op), stream or None))


def local_reduce_multi(send_ptrs, recv_ptr: int, dtype: int, count: int, op: int, stream: int = 0) -> int:
    arr = (ctypes.c_void_p * len(send_ptrs))(*send_ptrs)
    return int(lib.dccl_local_reduce_multi(arr, len(send_ptrs), recv_ptr, int(dtype), int(count), int(op),
                                           stream or None))


def local_reduce_chain(send_ptrs, own_ptr: int, dst_ptr: int, dtype: int, count: int, op: int, stream: int = 0) -> int:
    """dst = op(own, op(s[k-1], ... op(s[1], s[0]))): the ring reduce-scatter's order for one chunk."""
    arr = (ctypes.c_void_p * max(1, len(send_ptrs)))(*send_ptrs)
    return int(lib.dccl_local_reduce_chain(arr, len(send_ptrs), own_ptr, dst_ptr, int(dtype), int(count), int(op),
                                           stream or None))


def local_reduce_chain_host(send_ptrs, own_ptr: int, dst_ptr: int, dtype: int, count: int, op: int) -> int:
    """The host twin of local_reduce_chain (synchronous, staged through the current GPU)."""
    arr = (ctypes.c_void_p * max(1, len(send_ptrs)))(*send_ptrs)
    return int(lib.dccl_local_reduce_chain_host(arr, len(send_ptrs), own_ptr, dst_ptr, int(dtype), int(count),
                                                int(op)))


def copy_multi(src_ptrs, dst_ptrs, nbytes: int, stream: int = 0) -> int:
    n = len(src_ptrs)
    s = (ctypes.c_void_p * max(1, n))(*src_ptrs)
    d = (ctypes.c_void_p * max(1, n))(*dst_ptrs)
    return int(lib.dccl_copy_multi(s, d, n, int(nbytes), stream or None))


def host_reduce_gpu_min_bytes(dtype: int) -> int:
    """Bytes per operand from which dccl_local_reduce_host beats the reference's one-thread CPU loop (0: the
    reference has no CPU loop for this dtype); a routing hint for callers that still hold that loop."""
    return int(lib.dccl_host_reduce_gpu_min_bytes(int(dtype)))


def local_reduce_host(send_ptr: int, recv_ptr: int, dtype: int, count: int, op: int) -> int:
    """Host-pointer combine (staged through the current GPU); synchronous."""
    return int(lib.dccl_local_reduce_host(send_ptr, recv_ptr, int(dtype), int(count), int(op)))


def synth_fill(ptr: int, dtype: int, count: int, op: int, seed: int, buffer_id: int, stream: int = 0) -> int:
    """Counter-based synthetic operand in device memory (include/dccl/dccl_synth.h)."""
    return int(lib.dccl_synth_fill(ptr, int(dtype), int(count), int(op), int(seed), int(buffer_id), stream or None))


def synth_fill_range(ptr: int, dtype: int, count: int, op: int, seed: int, buffer_id: int, first: int,
                     stream: int = 0) -> int:
    """Elements [first, first + count) of the same synthetic operand."""
    return int(lib.dccl_synth_fill_range(ptr, int(dtype), int(count), int(op), int(seed), int(buffer_id),
                                         int(first), stream or None))


def register_host_memory(ptr: int, size: int) -> int:
    return int(lib.dccl_register_host_memory(ptr, size))


def deregister_host_memory(ptr: int) -> int:
    return int(lib.dccl_deregister_host_memory(ptr))


class Comm:
    """A DCCL communicator (include/dccl/dccl_comm.h) — the namespace-dccl collectives over the
    in-process transport (``Comm.in_process(world, rank)``, one per thread) or the cross-process
    RCCL transport (``Comm.rccl(world, rank, unique_id)``) or IPC peer-read transport
    (``Comm.ipc(world, rank)``), one process per GPU."""

    def __init__(self, handle: int):
        self.handle = handle

    @classmethod
    def in_process(cls, world: int, rank: int) -> "Comm":
        h = ctypes.c_void_p()
        check(lib.dccl_comm_init_rank(ctypes.byref(h), world, rank), "dccl_comm_init_rank")
        return cls(h.value)

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        check(lib.dccl_get_unique_id(buf), "dccl_get_unique_id")
        return buf.raw

    @classmethod
    def rccl(cls, world: int, rank: int, unique_id: bytes) -> "Comm":
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(unique_id, 128)
        check(lib.dccl_comm_init_rccl(ctypes.byref(h), world, rank, buf), "dccl_comm_init_rccl")
        return cls(h.value)

    @classmethod
    def ipc(cls, world: int, rank: int) -> "Comm":
        """Cross-process IPC peer-read transport (one process per GPU); rendezvous through
        DCCL_BOOTSTRAP_DIR / DCCL_BOOTSTRAP_TAG (or MASTER_PORT)."""
        h = ctypes.c_void_p()
        check(lib.dccl_comm_init_ipc(ctypes.byref(h), world, rank), "dccl_comm_init_ipc")
        return cls(h.value)

    @classmethod
    def p2p(cls, world: int, rank: int, exchange, memory: int = 3) -> "Comm":
        """A group over a caller-supplied point-to-point transport (dccl_comm_init_p2p):
        ``exchange(send_ptr, send_bytes, to, recv_ptr, recv_bytes, frm, stream) -> int`` moves one buffer
        each way (a 0 pointer skips that side); ``memory`` 1 = host buffers, 2 = device, 3 = both."""
        def trampoline(ctx, sbuf, sn, to, rbuf, rn, frm, stream):
            try:
                return int(exchange(sbuf or 0, sn, to, rbuf or 0, rn, frm, stream or 0))
            except Exception:  # an exception must not cross the C frames
                return int(ncclResult_t.ncclSystemError)
        fn = P2P_EXCHANGE_FN(trampoline)
        h = ctypes.c_void_p()
        check(lib.dccl_comm_init_p2p(ctypes.byref(h), world, rank, fn, None, memory), "dccl_comm_init_p2p")
        c = cls(h.value)
        c._keep = fn  # the callback must outlive the communicator
        return c

    def all_reduce(self, send: int, recv: int, count: int, dtype: int, op: int, stream: int = 0) -> int:
        return int(lib.dccl_all_reduce(send, recv, count, dtype, op, self.handle, stream or None))

    def reduce_scatter(self, send: int, recv: int, recvcount: int, dtype: int, op: int, stream: int = 0) -> int:
        return int(lib.dccl_reduce_scatter(send, recv, recvcount, dtype, op, self.handle, stream or None))

    def all_gather(self, send: int, recv: int, sendcount: int, dtype: int, stream: int = 0) -> int:
        return int(lib.dccl_all_gather(send, recv, sendcount, dtype, self.handle, stream or None))

    def reduce(self, send: int, recv: int, count: int, dtype: int, op: int, root: int, stream: int = 0) -> int:
        return int(lib.dccl_reduce(send, recv, count, dtype, op, root, self.handle, stream or None))

    def broadcast(self, send: int, recv: int, count: int, dtype: int, root: int, stream: int = 0) -> int:
        return int(lib.dccl_broadcast(send, recv, count, dtype, root, self.handle, stream or None))

    def register(self, ptr: int, size: int) -> int:
        """dcclRegisterCacheMemory: host memory is page-locked; device memory is validated and tracked
        until deregister(ptr) (peers read inputs through the scratch); 64-byte aligned address and size."""
        return int(lib.dccl_comm_register(self.handle, ptr, size))

    def deregister(self, ptr: int) -> int:
        return int(lib.dccl_comm_deregister(self.handle, ptr))

    def finalize(self) -> int:
        h, self.handle = self.handle, None
        return int(lib.dccl_comm_finalize(h)) if h else 0


def check(code: int, what: str = "dccl") -> None:
    if code != 0:
        raise DcclError(code, what)


# --------------------------------------------------------------------------------------
# torch conveniences (device memory and streams are torch's; the compute is ours)
# --------------------------------------------------------------------------------------
if torch is not None:
    TORCH_DTYPES = {
        0: torch.int8, 1: torch.uint8, 2: torch.int32, 3: torch.uint32 if hasattr(torch, "uint32") else None,
        4: torch.int64, 5: torch.uint64 if hasattr(torch, "uint64") else None, 6: torch.float16,
        7: torch.float32, 8: torch.float64, 9: torch.bfloat16,
    }
    _TORCH_TO_DCCL = {v: k for k, v in TORCH_DTYPES.items() if v is not None}

    def dccl_dtype_of(t) -> int:
        return _TORCH_TO_DCCL[t.dtype]

    def reduce_(recv, send, op: int = 0, dtype: int | None = None, stream=None) -> None:
        """In place ``recv = op(recv, send)`` on CUDA tensors through the HIP kernel."""
        if not (recv.is_cuda and send.is_cuda):
            raise ValueError("reduce_ expects device tensors")
        if recv.numel() != send.numel() or not recv.is_contiguous() or not send.is_contiguous():
            raise ValueError("reduce_ expects contiguous tensors of equal numel")
        dt = dccl_dtype_of(recv) if dtype is None else dtype
        s = (stream or torch.cuda.current_stream(recv.device)).cuda_stream
        check(local_reduce(send.data_ptr(), recv.data_ptr(), dt, recv.numel(), op, s), "dccl_local_reduce")
