"""ctypes binding of the tuning library tools/lib/libdccl_amd_tune.so (tools/tune/dccl_reduce_tuning.h).

The tuning variants are tools-only: dccl_amd/build.py builds them into their own library, so the
product library dccl_amd/lib/libdccl_amd.so exports none of them.
"""
import ctypes
import os

import dccl_amd  # noqa: F401  (loads the HIP runtime the tuning library shares)

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libdccl_amd_tune.so")


def _load():
    if not os.path.exists(PATH):
        raise ImportError(f"{PATH} is missing: run `python dccl_amd/build.py`")
    lib = ctypes.CDLL(PATH)
    c_int, c_size_t, c_void_p = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p
    sig = {
        "dccl_tune_reduce_f32_sum": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_size_t, c_void_p]),
        "dccl_tune_num_variants": (c_int, []),
        "dccl_tune_reduce_f32_sum_lds": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_size_t, c_size_t, c_void_p]),
        "dccl_tune_asm_f32_sum": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
        "dccl_tune_variant_info": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
        "dccl_tune_skew_f32_sum": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_int, c_void_p]),
        "dccl_tune_multi_f32_sum": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_size_t, c_int, c_size_t,
                                            c_void_p]),
        "dccl_tune_chain_f32_sum": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_void_p, c_size_t, c_size_t,
                                            c_void_p]),
        "dccl_tune_phased_f32_sum": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_size_t, c_int, c_size_t,
                                             c_void_p]),
        "dccl_tune_chain_phased_f32_sum": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_void_p, c_size_t,
                                                   c_int, c_void_p]),
        "dccl_tune_phased_walk_f32_sum": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_size_t, c_int,
                                                  c_void_p]),
        "dccl_tune_chain_policy_f32_sum": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_void_p, c_size_t,
                                                   c_size_t, c_int, c_void_p]),
        "dccl_tune_phased_prod_f32_sum": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_void_p, c_size_t,
                                                  c_int, c_int, c_size_t, c_void_p]),
        "dccl_tune_shift_caps_f32_sum": (c_int, [c_void_p, c_void_p, c_size_t, c_size_t, c_void_p]),
        "dccl_tune_group_f32_sum": (c_int, [c_void_p, c_void_p, c_size_t, c_size_t, c_void_p]),
        "dccl_tune_unaligned_kway_f32_sum": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_void_p, c_size_t,
                                                     c_size_t, c_int, c_void_p]),
        "dccl_tune_phased_run_f32_sum": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_size_t, c_size_t, c_int,
                                                 ctypes.c_uint, c_void_p]),
        "dccl_tune_runs_f32_sum": (c_int, [c_int, ctypes.POINTER(c_void_p), c_int, c_void_p, c_void_p, c_size_t,
                                           c_size_t, c_int, c_int, c_void_p]),
        "dccl_tune_pair_run_f32_sum": (c_int, [c_void_p, c_void_p, c_size_t, c_size_t, c_int, c_void_p]),
        "dccl_tune_wq_f32_sum": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_int, c_void_p, c_void_p]),
        "dccl_tune_unaligned_pair_f32_sum": (c_int, [c_void_p, c_void_p, c_size_t, c_size_t, c_int, c_void_p]),
        "dccl_tune_misaligned_f32_sum": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
        "dccl_tune_ceiling": (c_int, [c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
        "dccl_tune_write_num_variants": (c_int, []),
        "dccl_tune_shift_num_variants": (c_int, []),
        "dccl_tune_pipelined_f32_sum": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_size_t, c_void_p]),
        "dccl_tune_shift_f32_sum": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_void_p, c_void_p, c_void_p]),
        "dccl_tune_write_probe": (c_int, [c_int, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


def tune_variants() -> list:
    out = []
    for v in range(lib.dccl_tune_num_variants()):
        vals = [ctypes.c_int() for _ in range(4)]
        lib.dccl_tune_variant_info(v, *[ctypes.byref(x) for x in vals])
        out.append(dict(zip(("block", "unroll", "policy", "xcd"), (x.value for x in vals))))
    return out
