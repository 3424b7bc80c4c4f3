"""CPU tests of the drop-in boundary: the C-ABI library loads and exports every symbol
include/dccl/*.h declares; argument validation answers without touching a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(ROOT, "include", "dccl")


def declared_c_symbols():
    syms = set()
    for h in os.listdir(INCLUDE):
        if not h.endswith(".h"):
            continue
        text = open(os.path.join(INCLUDE, h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(dccl_\w+)\s*\(", text, flags=re.M):
            syms.add(m.group(1))
    return syms


def test_library_exports_every_declared_symbol():
    import dccl_amd
    syms = declared_c_symbols()
    assert "dccl_local_reduce" in syms and "dccl_local_reduce_host" in syms
    out = subprocess.run(["nm", "-D", "--defined-only", dccl_amd.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = syms - exported
    assert not missing, missing
    assert set(dccl_amd.EXPORTED_SYMBOLS) == syms


def test_cpp_api_symbols_exported():
    """The C++ namespace-dccl surface of include/dccl/dccl.hpp is defined in the library."""
    import dccl_amd
    out = subprocess.run(["nm", "-D", "-C", "--defined-only", dccl_amd.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    for fn in ["dccl::ncclAllReduce(", "dccl::ncclReduceScatter(", "dccl::ncclCommInit(",
               "dccl::ncclCommFinalize(", "dccl::dcclGetMyRank(", "dccl::dcclGetWorldSize(",
               "dccl::dcclRegisterCacheMemory(", "dccl::dcclDeregisterCacheMemory(", "dccl::ncclAllGather(",
               "dccl::ncclReduce(", "dccl::ncclBroadcast(", "dccl::ncclBcast(", "dccl::ncclSend(",
               "dccl::ncclRecv("]:
        assert fn in out, fn


def test_validation_without_gpu():
    import dccl_amd as d
    assert d.size_of_type(7) == 4 and d.size_of_type(9) == 2 and d.size_of_type(6) == 2
    assert d.size_of_type(8) == 8 and d.size_of_type(0) == 1 and d.size_of_type(10) == 0
    assert d.version() >= 10000
    assert "InvalidUsage" in d.result_string(5)
    # dtype is checked before op (reference: type switch outside the op switch)
    assert d.local_reduce(0, 0, 10, 16, 0) == 4
    assert d.local_reduce(0, 0, 10, 16, 4) == 4
    assert d.local_reduce(0, 0, 7, 16, 4) == 5    # ncclAvg -> ncclInvalidUsage
    assert d.local_reduce(0, 0, 7, 16, 5) == 4    # beyond ncclNumOps -> ncclInvalidArgument
    assert d.local_reduce(0, 0, 7, 16, -1) == 4
    assert d.local_reduce(0, 0, 7, 0, 0) == 0     # empty combine
    assert d.local_reduce(0, 0, 7, 16, 0) == 4    # null operands
    assert d.local_reduce_host(0, 0, 7, 16, 4) == 5
    assert d.local_reduce_host(0, 0, 9, 0, 3) == 0
    assert d.local_reduce_multi([0] * 9, 0, 7, 16, 0) == 4
    assert d.local_reduce_multi([0], 0, 7, 16, 4) == 5
    assert d.local_reduce_chain_host([], 8, 8, 7, 16, 0) == 4        # nsend 0
    assert d.local_reduce_chain_host([8] * 9, 8, 8, 7, 16, 0) == 4   # nsend 9
    assert d.local_reduce_chain_host([8], 8, 8, 7, 16, 4) == 5       # Avg
    assert d.local_reduce_chain_host([8], 8, 8, 7, 0, 0) == 0        # count 0
    assert d.local_reduce_chain_host([0], 8, 8, 7, 16, 0) == 4       # NULL send


@pytest.mark.parametrize("dt", [0, 6, 7, 8])
def test_partial_overlap_rejected_without_gpu(dt):
    """The aliasing contract of include/dccl/dccl_reduce.h: an operand that shares bytes
    with the destination without starting at the same address returns ncclInvalidArgument at every combine
    entry point, before any HIP call (so it answers here, with no GPU).  Overlap by one element and by all
    but one, in both directions; sources only read may overlap each other."""
    import dccl_amd as d
    esz, n = d.size_of_type(dt), 64
    base = 1 << 40  # never dereferenced: the check is pointer arithmetic ahead of any launch
    dst = base + 4096
    shifts = [esz, -esz, (n - 1) * esz, -(n - 1) * esz]
    for sh in shifts:
        src = dst + sh
        assert d.local_reduce(src, dst, dt, n, 0) == 4, sh
        assert d.local_reduce_host(src, dst, dt, n, 0) == 4, sh
        far = base + (1 << 30)
        for k in (1, 3, 8):
            srcs = [far + j * n * esz for j in range(k - 1)] + [src]
            assert d.local_reduce_multi(srcs, dst, dt, n, 2) == 4, (sh, k)
            assert d.local_reduce_chain(srcs, far + (1 << 20), dst, dt, n, 3) == 4, (sh, k)
            assert d.local_reduce_chain_host(srcs, far + (1 << 20), dst, dt, n, 3) == 4, (sh, k)
        # own against dst
        assert d.local_reduce_chain([far], src, dst, dt, n, 0) == 4, sh
        assert d.local_reduce_chain_host([far], src, dst, dt, n, 0) == 4, sh
        # copy_multi: a dst overlapping its own src, another pair's src, or another pair's dst
        nb = n * esz
        assert d.copy_multi([src], [dst], nb) == 4, sh
        assert d.copy_multi([far, src], [dst, far + (1 << 20)], nb) == 4, sh
        assert d.copy_multi([far, far + (1 << 20)], [dst, src], nb) == 4, sh
    # validation order is unchanged: dtype and op first, then null pointers, then overlap
    assert d.local_reduce(dst + esz, dst, 10, n, 0) == 4
    assert d.local_reduce(dst + esz, dst, dt, n, 4) == 5
    assert d.local_reduce(dst + esz, dst, dt, 0, 0) == 0  # count 0: nothing overlaps
    # adjacent ranges (the bench's pooled layout, the ring's chunk k and k+1) pass validation: without a GPU
    # the launch itself then fails with a device error, not ncclInvalidArgument
    assert d.local_reduce(dst + n * esz, dst, dt, n, 0) not in (0, 4)
    assert d.local_reduce(dst - n * esz, dst, dt, n, 0) not in (0, 4)


def test_enum_values_match_reference_header():
    """Numeric enum values are the reference's (include/dccl/dccl.hpp:59-112)."""
    import dccl_amd as d
    assert [int(x) for x in d.ncclDataType_t] == list(range(10))
    assert int(d.ncclRedOp_t.ncclAvg) == 4 and int(d.ncclResult_t.ncclInvalidUsage) == 5
    hpp = open(os.path.join(INCLUDE, "dccl.hpp")).read()
    for name, val in [("ncclFloat32", 7), ("ncclBfloat16", 9), ("ncclAvg", 4), ("ncclInvalidArgument", 4),
                      ("ncclUnhandledCudaError", 1), ("ncclMin", 3)]:
        assert re.search(rf"\b{name}\s*=\s*{val}\b", hpp), name


def _c_check_binary():
    path = os.path.join(ROOT, "dccl_amd", "bin", "c_abi_check")
    if not os.path.exists(path):
        pytest.skip("c_abi_check not built (python dccl_amd/build.py)")
    return path


def test_plain_c_consumer_cpu():
    """tools/c_abi_check.c: the headers compile as C11 with -pedantic -Werror, the library links from C,
    and the validation contract answers from C without a GPU."""
    p = subprocess.run([_c_check_binary()], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "ok" in p.stdout, p.stdout + p.stderr


@pytest.mark.gpu
def test_plain_c_consumer_gpu(gpu):
    p = subprocess.run([_c_check_binary(), "gpu"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "ok" in p.stdout, p.stdout + p.stderr
