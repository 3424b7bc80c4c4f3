"""TEST INFRASTRUCTURE ONLY — ctypes access to the CPU combine oracles.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg import this package, and only as the checker or the timed CPU baseline.
The product path (``dccl_amd``) never imports it.

* ``restatement()`` — ``oracle/liboracle_host_reduce.so``, the C restatement of
  ``do_host_reduce<DT>`` (/root/reference/src/core/internal_common.hpp:496-586),
  compiled with the reference's Release flags (CMakeLists.txt:25).
* ``restatement_native()`` — the same source with the reference's Benchmark flags
  (-Ofast -march=native, CMakeLists.txt:26), a labelled CPU-baseline variant only.

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
_NATIVE = os.path.join(HERE, "liboracle_host_reduce_native.so")

# ncclDataType_t -> numpy dtype (fp16 / bf16 travel as raw uint16 bit patterns)
NP_DTYPES = {
    0: np.int8, 1: np.uint8, 2: np.int32, 3: np.uint32, 4: np.int64,
    5: np.uint64, 6: np.uint16, 7: np.float32, 8: np.float64, 9: np.uint16,
}

_cache: dict = {}


def build() -> None:
    """Compile the restatement (Release flags, plus the labelled -Ofast -march=native variant)."""
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
        _cache["rs"] = lib
    return _cache["rs"]


def restatement_native():
    """The restatement built with the reference's Benchmark flags (-Ofast -march=native), or None."""
    if "native" not in _cache:
        _cache["native"] = _bind(_NATIVE, ["oracle_host_reduce"]) if os.path.exists(_NATIVE) else None
    return _cache["native"]


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
