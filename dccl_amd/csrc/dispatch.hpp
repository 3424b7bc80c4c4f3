// dccl_amd/csrc/dispatch.hpp — enum -> (element type, op) dispatch of the combine.
//
// Mirrors the reference's ON_DCCL_DATATYPE (/root/reference/src/core/internal_common.hpp:350-413)
// and op switch (internal_common.hpp:564-585) with two deliberate fixes:
// ncclBfloat16 (9) and ncclFloat16 (6) are always supported, and an unknown dtype is an
// error (ncclInvalidArgument) instead of a silent no-op.
#pragma once

#include <cstddef>
#include <cstdint>

#include "combine.hpp"
#include "dccl/dccl_reduce.h"

namespace dccl_amd {

enum DType : int {
    kInt8 = 0, kUint8 = 1, kInt32 = 2, kUint32 = 3, kInt64 = 4, kUint64 = 5,
    kFloat16 = 6, kFloat32 = 7, kFloat64 = 8, kBfloat16 = 9,
};
constexpr int kAvg = 4;

inline size_t size_of_dtype(int dtype) {
    switch (dtype) {
    case kInt8: case kUint8: return 1;
    case kFloat16: case kBfloat16: return 2;
    case kInt32: case kUint32: case kFloat32: return 4;
    case kInt64: case kUint64: case kFloat64: return 8;
    default: return 0;
    }
}

// Order of checks follows the reference: the dtype switch is outermost, the op switch
// inside it, so an unknown dtype wins over a bad op.
inline int validate(int dtype, int op) {
    if (size_of_dtype(dtype) == 0) return DCCL_INVALID_ARGUMENT;
    if (op == kAvg) return DCCL_INVALID_USAGE;  // internal_common.hpp:577-580
    if (op < kSum || op > kMin) return DCCL_INVALID_ARGUMENT;
    return DCCL_SUCCESS;
}

// Operand ranges [a, a + bytes) and [b, b + bytes) that share bytes without being the same array.  The
// reference's loop (internal_common.hpp:550-560) walks such ranges in ascending order on one thread, so an
// element it writes can be read again later as a source; no parallel launch reproduces that order, and the
// boundary rejects the call with ncclInvalidArgument (SURVEY.md §8(b) "Ownership").  The same array
// (a == b) stays allowed: every combine is element-wise, each output depends only on its own index.
inline bool partial_overlap(const void* a, const void* b, size_t bytes) {
    const uintptr_t x = reinterpret_cast<uintptr_t>(a), y = reinterpret_cast<uintptr_t>(b);
    return x != y && (x < y ? y - x < bytes : x - y < bytes);
}

// The overlap rule of every combine entry point (include/dccl/dccl_reduce.h): each source against the
// destination, and `own` (chain forms; nullptr otherwise) against the destination.
inline bool sources_overlap_destination(const void* const* sends, int nsend, const void* own, const void* dst,
                                        size_t bytes) {
    for (int k = 0; k < nsend; ++k)
        if (partial_overlap(sends[k], dst, bytes)) return true;
    return own != nullptr && partial_overlap(own, dst, bytes);
}

template <typename Fn, typename T, typename... A>
inline int dispatch_op(int op, A&&... a) {
    switch (op) {
    case kSum: return Fn::template run<T, kSum>(a...);
    case kProd: return Fn::template run<T, kProd>(a...);
    case kMax: return Fn::template run<T, kMax>(a...);
    case kMin: return Fn::template run<T, kMin>(a...);
    case kAvg: return DCCL_INVALID_USAGE;
    default: return DCCL_INVALID_ARGUMENT;
    }
}

template <typename Fn, typename... A>
inline int dispatch(int dtype, int op, A&&... a) {
    switch (dtype) {
    case kInt8: return dispatch_op<Fn, int8_t>(op, a...);
    case kUint8: return dispatch_op<Fn, uint8_t>(op, a...);
    case kInt32: return dispatch_op<Fn, int32_t>(op, a...);
    case kUint32: return dispatch_op<Fn, uint32_t>(op, a...);
    case kInt64: return dispatch_op<Fn, int64_t>(op, a...);
    case kUint64: return dispatch_op<Fn, uint64_t>(op, a...);
    case kFloat16: return dispatch_op<Fn, f16_bits>(op, a...);
    case kFloat32: return dispatch_op<Fn, float>(op, a...);
    case kFloat64: return dispatch_op<Fn, double>(op, a...);
    case kBfloat16: return dispatch_op<Fn, bf16_bits>(op, a...);
    default: return DCCL_INVALID_ARGUMENT;
    }
}

}  // namespace dccl_amd
