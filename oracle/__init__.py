"""TEST INFRASTRUCTURE ONLY — ctypes access to the CPU combine oracles.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg import this package, and only as the checker or the timed CPU baseline.
The product path (``dccl_amd``) never imports it.

* ``restatement()`` — ``oracle/liboracle_host_reduce.so``, the C restatement of
  ``do_host_reduce<DT>`` (/root/reference/src/core/internal_common.hpp:496-586),
  compiled with the reference's Release flags (CMakeLists.txt:25).
* ``restatement_benchflags(path)`` — the same source with the reference's Benchmark
  flags (-Ofast -march=native, CMakeLists.txt:26), a labelled CPU-baseline variant only.
  ``bench.py`` compiles it on the host it runs on (``compile_benchflags``); the prebuilt
  ``liboracle_host_reduce_v4.so`` (-march=x86-64-v4) is the fallback.

Parity unpinned: the reference's own combine is not built here (it needs its
CMake-generated config.h and spdlog, which the image lacks), and the reference
holds no test vectors.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_RESTATEMENT = os.path.join(HERE, "liboracle_host_reduce.so")
_V4 = os.path.join(HERE, "liboracle_host_reduce_v4.so")
SOURCE = os.path.join(HERE, "host_reduce.c")
BENCH_FLAGS = ["-std=c11", "-Ofast", "-march=native", "-mprefer-vector-width=512", "-fPIC", "-shared"]

# ncclDataType_t -> numpy dtype (fp16 / bf16 travel as raw uint16 bit patterns)
NP_DTYPES = {
    0: np.int8, 1: np.uint8, 2: np.int32, 3: np.uint32, 4: np.int64,
    5: np.uint64, 6: np.uint16, 7: np.float32, 8: np.float64, 9: np.uint16,
}

_cache: dict = {}


def build() -> None:
    """Compile the restatement (Release flags, plus the labelled -Ofast -march=x86-64-v4 variant)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _bind(path: str, names: list[str]):
    lib = ctypes.CDLL(path)
    for n in names:
        f = getattr(lib, n)
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
    return lib


def restatement():
    if "rs" not in _cache:
        if not os.path.exists(_RESTATEMENT):
            build()
        lib = _bind(_RESTATEMENT, ["oracle_host_reduce", "oracle_expected_reduce"])
        lib.oracle_float_to_half.restype = ctypes.c_uint16
        lib.oracle_float_to_half.argtypes = [ctypes.c_float]
        lib.oracle_half_to_float.restype = ctypes.c_float
        lib.oracle_half_to_float.argtypes = [ctypes.c_uint16]
        lib.oracle_float_to_bf16.restype = ctypes.c_uint16
        lib.oracle_float_to_bf16.argtypes = [ctypes.c_float]
        lib.oracle_bf16_to_float.restype = ctypes.c_float
        lib.oracle_bf16_to_float.argtypes = [ctypes.c_uint16]
        lib.oracle_synth_fill.restype = ctypes.c_int
        lib.oracle_synth_fill.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t]
        lib.oracle_time_host_reduce.restype = ctypes.c_double
        lib.oracle_time_host_reduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                                ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_double, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        _cache["rs"] = lib
    return _cache["rs"]


def time_host_reduce(send_ptr: int, recv_ptr: int, count: int, dtype: int, op: int, nthreads: int = 1,
                     nsets: int = 1, stride: int = 0, min_seconds: float = 0.25, min_reps: int = 3) -> tuple:
    """(seconds per combine, calls) of the restatement timed in C (cpu_timing.c): `nsets` operand pairs
    `stride` bytes apart in rotation, each combine split over `nthreads` threads.  Bench CPU baseline only."""
    reps = ctypes.c_size_t(0)
    t = restatement().oracle_time_host_reduce(send_ptr, recv_ptr, nsets, stride, count, dtype, op, nthreads,
                                              min_seconds, min_reps, ctypes.byref(reps))
    if t < 0:
        raise RuntimeError(f"oracle_time_host_reduce failed ({t})")
    return t, int(reps.value)


def compile_benchflags(outdir: str) -> str | None:
    """The restatement compiled with the reference's Benchmark flags for THIS host's CPU (-march=native,
    CMakeLists.txt:26) into `outdir`; None when no compiler is available."""
    out = os.path.join(outdir, "liboracle_host_reduce_benchflags.so")
    try:
        subprocess.run(["gcc", *BENCH_FLAGS, SOURCE, "-o", out], check=True, capture_output=True, timeout=120)
    except Exception:
        return None
    return out


def benchflags_fallback() -> str | None:
    """The prebuilt Benchmark-flags variant (-march=x86-64-v4), or None."""
    return _V4 if os.path.exists(_V4) else None


def restatement_benchflags(path: str):
    """The restatement built with the reference's Benchmark flags (a library from compile_benchflags or
    benchflags_fallback); only ever loaded in a child process (an unsupported instruction ends the child)."""
    return _bind(path, ["oracle_host_reduce"])


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def host_reduce(send: np.ndarray, recv: np.ndarray, dtype: int, op: int, count: int | None = None) -> int:
    """Faithful restatement (reference loop split) — in place on ``recv``."""
    n = recv.size if count is None else count
    return restatement().oracle_host_reduce(_ptr(send), _ptr(recv), n, dtype, op)


def expected_reduce(send: np.ndarray, recv: np.ndarray, dtype: int, op: int, count: int | None = None) -> int:
    """Intended semantics, plain pass — in place on ``recv``."""
    n = recv.size if count is None else count
    return restatement().oracle_expected_reduce(_ptr(send), _ptr(recv), n, dtype, op)


def synth(n: int, dtype: int, op: int, seed: int, buffer_id: int, first: int = 0) -> np.ndarray:
    """Elements [first, first+n) of the counter-based synthetic operand (include/dccl/dccl_synth.h)."""
    out = aligned_empty(n, NP_DTYPES[dtype])
    rc = restatement().oracle_synth_fill(_ptr(out), dtype, n, op, seed, buffer_id, first)
    if rc != 0:
        raise ValueError(f"oracle synth failed rc={rc}")
    return out


def combine(send: np.ndarray, recv: np.ndarray, dtype: int, op: int) -> np.ndarray:
    """Functional form: returns op(recv, send) without touching the inputs."""
    out = np.array(recv, copy=True)
    rc = expected_reduce(np.ascontiguousarray(send), out, dtype, op)
    if rc != 0:
        raise ValueError(f"oracle combine failed rc={rc}")
    return out


def aligned_empty(n: int, npdtype, align: int = 64, offset_bytes: int = 0, pad_elems: int = 0) -> np.ndarray:
    """1-D array whose first element sits ``offset_bytes`` past an ``align`` boundary.

    ``pad_elems`` extra elements of slack follow the view, so the faithful
    restatement / reference loop may overrun without corrupting
    the heap; the slack is reachable as ``arr.base``.
    """
    item = np.dtype(npdtype).itemsize
    raw = np.zeros((n + pad_elems) * item + align + offset_bytes + 64, dtype=np.uint8)
    start = (-raw.ctypes.data) % align + offset_bytes
    return raw[start:start + n * item].view(npdtype)
