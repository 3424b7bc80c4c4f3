"""Build ``dccl_amd/lib/libdccl_amd.so`` in-tree with hipcc for gfx950.

One shared library holds the HIP kernels, the C-ABI (include/dccl/dccl_reduce.h) and the
C++ ``namespace dccl`` API (include/dccl/dccl.hpp).  Sources compile in parallel; the
link is a plain ``hipcc -shared``.  No fast-math / FTZ flags: the combine must keep
fp32/fp16 denormals (SURVEY.md §7 "Bit-exact semantics").

Tools-only artefacts, never linked into the product library: the dccl_cli harness and the plain-C ABI
check, the PMC and native C4 workloads of bench.py (dccl_amd/bin/).

    python dccl_amd/build.py [--force]      (by path: importing the package loads the library)
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OUT_DIR = os.path.join(PKG, "lib")
OBJ_DIR = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(OUT_DIR, "libdccl_amd.so")
BIN_DIR = os.path.join(PKG, "bin")
CLI_SRC = os.path.join(ROOT, "tools", "dccl_cli.cpp")
CLI = os.path.join(BIN_DIR, "dccl_cli")
C_CHECK_SRC = os.path.join(ROOT, "tools", "c_abi_check.c")
C_CHECK = os.path.join(BIN_DIR, "c_abi_check")
PMC_SRC = os.path.join(ROOT, "tools", "pmc_combine.cpp")
PMC_BIN = os.path.join(BIN_DIR, "pmc_combine")
C4_SRC = os.path.join(ROOT, "tools", "c4_native.cpp")
C4_BIN = os.path.join(BIN_DIR, "c4_native")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DCCL_OFFLOAD_ARCH", "gfx950")

COMMON = ["-std=c++17", "-O3", "-fPIC", "-Wall", "-Wno-unused-command-line-argument",
          f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}"]


def _sources() -> list[str]:
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _headers() -> list[str]:
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))]
    inc = os.path.join(ROOT, "include", "dccl")
    hs += [os.path.join(inc, f) for f in os.listdir(inc)]
    return hs


def _compile(src: str, extra_inc: tuple = ()) -> str:
    obj = os.path.join(OBJ_DIR, os.path.basename(src) + ".o")
    deps = _headers() + [src, __file__] + [os.path.join(d, f) for d in extra_inc for f in os.listdir(d)
                                          if f.endswith(".h")]
    newest_dep = max(os.path.getmtime(p) for p in deps)
    if os.path.exists(obj) and os.path.getmtime(obj) >= newest_dep:
        return obj
    cmd = [HIPCC, *COMMON, *[f"-I{d}" for d in extra_inc], f"--offload-arch={ARCH}", "-c", src, "-o", obj]
    if src.endswith(".hip"):
        cmd[1:1] = ["-x", "hip"]
    subprocess.run(cmd, check=True)
    return obj


def build(force: bool = False) -> str:
    os.makedirs(OUT_DIR, exist_ok=True)
    os.makedirs(OBJ_DIR, exist_ok=True)
    srcs = _sources()
    if force:
        for f in os.listdir(OBJ_DIR):
            os.remove(os.path.join(OBJ_DIR, f))
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        tmp = LIB + ".tmp"
        subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp,
                        "-Wl,-soname,libdccl_amd.so"], check=True)
        os.replace(tmp, LIB)
    # the dccl_cli harness (C++ on the namespace-dccl API), rpath'd to the in-tree library
    os.makedirs(BIN_DIR, exist_ok=True)
    if force or not os.path.exists(CLI) or os.path.getmtime(CLI) < max(os.path.getmtime(LIB),
                                                                          os.path.getmtime(CLI_SRC)):
        subprocess.run([HIPCC, *COMMON, CLI_SRC, "-o", CLI, f"-L{OUT_DIR}", "-ldccl_amd",
                        "-Wl,-rpath,$ORIGIN/../lib", "-pthread"], check=True)
    # the bench's combine as a bare process, for the rocprofv3 --pmc passes bench.py runs (roofline.traffic)
    if force or not os.path.exists(PMC_BIN) or os.path.getmtime(PMC_BIN) < max(os.path.getmtime(LIB),
                                                                                os.path.getmtime(PMC_SRC)):
        subprocess.run([HIPCC, *COMMON, PMC_SRC, "-o", PMC_BIN, f"-L{OUT_DIR}", "-ldccl_amd",
                        "-Wl,-rpath,$ORIGIN/../lib"], check=True)
    # BASELINE C4's small sizes issued from a native loop (bench.py's c4 leg, `native_eager_us_per_launch`)
    if force or not os.path.exists(C4_BIN) or os.path.getmtime(C4_BIN) < max(os.path.getmtime(LIB),
                                                                              os.path.getmtime(C4_SRC)):
        subprocess.run([HIPCC, *COMMON, C4_SRC, "-o", C4_BIN, f"-L{OUT_DIR}", "-ldccl_amd",
                        "-Wl,-rpath,$ORIGIN/../lib"], check=True)
    # a plain C11 consumer of the C-ABI headers (gcc, no C++ / HIP headers)
    if force or not os.path.exists(C_CHECK) or os.path.getmtime(C_CHECK) < max(
            [os.path.getmtime(LIB), os.path.getmtime(C_CHECK_SRC)] + [os.path.getmtime(h) for h in _headers()]):
        subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-pedantic", "-Werror",
                        f"-I{os.path.join(ROOT, 'include')}", C_CHECK_SRC, "-o", C_CHECK, f"-L{OUT_DIR}",
                        "-ldccl_amd", "-Wl,-rpath,$ORIGIN/../lib"], check=True)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
