// dccl_amd/csrc/synth.hip — device-side counter-based operand generator.
//
// Fills benchmark / parity operands in HBM without a host round trip.  Each element is a pure
// function of (seed, buffer_id, index), see include/dccl/dccl_synth.h for the value mapping; the
// host restatement oracle_synth_fill (oracle/host_reduce.c) regenerates any slice for checking.
// Write-bound: one 16-B store per lane per chunk, grid-stride over 16-B chunks.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dccl/dccl_reduce.h"
#include "dccl/dccl_synth.h"
#include "dispatch.hpp"

namespace dccl_amd {
namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// Element value from the 64 random bits x (exact constructions only).
template <typename T, bool PROD> __device__ __forceinline__ T value(uint64_t x) {
    if constexpr (std::is_same_v<T, float>) {
        if constexpr (PROD) return __builtin_bit_cast(float, static_cast<uint32_t>(((126u + (x >> 63)) << 23) | (x & 0x7fffffu)));
        return static_cast<float>(static_cast<int32_t>(x >> 40) - (1 << 23)) * 0x1p-23f;
    } else if constexpr (std::is_same_v<T, double>) {
        if constexpr (PROD) return __builtin_bit_cast(double, ((1022ull + (x >> 63)) << 52) | (x & 0xfffffffffffffull));
        return static_cast<double>(static_cast<int64_t>(x >> 11) - (1ll << 52)) * 0x1p-52;
    } else if constexpr (std::is_same_v<T, f16_bits>) {
        if constexpr (PROD) return f16_bits{static_cast<uint16_t>(((14u + (x >> 63)) << 10) | (x & 0x3ffu))};
        return f16_bits{f32_to_f16(static_cast<float>(static_cast<int32_t>(x >> 53) - (1 << 10)) * 0x1p-10f)};
    } else if constexpr (std::is_same_v<T, bf16_bits>) {
        if constexpr (PROD) return bf16_bits{static_cast<uint16_t>(((126u + (x >> 63)) << 7) | (x & 0x7fu))};
        return bf16_bits{f32_to_bf16(static_cast<float>(static_cast<int32_t>(x >> 56) - (1 << 7)) * 0x1p-7f)};
    } else {
        return static_cast<T>(x);  // integers: low bytes
    }
}

template <typename T, bool PROD>
__global__ void __launch_bounds__(256) synth_kernel(T* dst, size_t count, uint64_t key, size_t first,
                                                    bool aligned16) {
    constexpr size_t E = 16 / sizeof(T);
    const size_t nchunk = (count + E - 1) / E;
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t c = size_t(blockIdx.x) * blockDim.x + threadIdx.x; c < nchunk; c += stride) {
        const size_t i0 = c * E;
        if (aligned16 && i0 + E <= count) {
            union { T e[E]; uint4 v; } u;
#pragma unroll
            for (size_t k = 0; k < E; ++k) u.e[k] = value<T, PROD>(splitmix64(key ^ (first + i0 + k)));
            __builtin_nontemporal_store(u.v.x, reinterpret_cast<unsigned*>(dst + i0) + 0);
            __builtin_nontemporal_store(u.v.y, reinterpret_cast<unsigned*>(dst + i0) + 1);
            __builtin_nontemporal_store(u.v.z, reinterpret_cast<unsigned*>(dst + i0) + 2);
            __builtin_nontemporal_store(u.v.w, reinterpret_cast<unsigned*>(dst + i0) + 3);
        } else {
            for (size_t i = i0; i < count && i < i0 + E; ++i) dst[i] = value<T, PROD>(splitmix64(key ^ (first + i)));
        }
    }
}

template <typename T>
int fill(void* dst, size_t count, bool prod, uint64_t key, size_t first, hipStream_t stream) {
    constexpr size_t E = 16 / sizeof(T);
    const size_t nchunk = (count + E - 1) / E;
    size_t grid = (nchunk + 255) / 256;
    if (grid > 65536) grid = 65536;
    T* d = static_cast<T*>(dst);
    bool aligned16 = (reinterpret_cast<uintptr_t>(dst) & 15) == 0;
    void* args[] = {&d, &count, &key, &first, &aligned16};
    const void* fn = prod ? reinterpret_cast<const void*>(&synth_kernel<T, true>)
                          : reinterpret_cast<const void*>(&synth_kernel<T, false>);
    return hipLaunchKernel(fn, dim3(static_cast<unsigned>(grid)), dim3(256), args, 0, stream) == hipSuccess
               ? DCCL_SUCCESS
               : DCCL_UNHANDLED_DEVICE_ERROR;
}

}  // namespace
}  // namespace dccl_amd

using namespace dccl_amd;

extern "C" int dccl_synth_fill_range(void* dst, int dtype, size_t count, int op, uint64_t seed, uint64_t buffer_id,
                                     size_t first, void* hip_stream) {
    if (size_of_dtype(dtype) == 0 || op < 0 || op > kAvg) return DCCL_INVALID_ARGUMENT;
    if (count == 0) return DCCL_SUCCESS;
    if (dst == nullptr) return DCCL_INVALID_ARGUMENT;
    const uint64_t key = seed ^ (buffer_id << 40);
    const bool prod = op == kProd;
    const auto s = static_cast<hipStream_t>(hip_stream);
    switch (dtype) {
    case kInt8: return fill<int8_t>(dst, count, prod, key, first, s);
    case kUint8: return fill<uint8_t>(dst, count, prod, key, first, s);
    case kInt32: return fill<int32_t>(dst, count, prod, key, first, s);
    case kUint32: return fill<uint32_t>(dst, count, prod, key, first, s);
    case kInt64: return fill<int64_t>(dst, count, prod, key, first, s);
    case kUint64: return fill<uint64_t>(dst, count, prod, key, first, s);
    case kFloat16: return fill<f16_bits>(dst, count, prod, key, first, s);
    case kFloat32: return fill<float>(dst, count, prod, key, first, s);
    case kFloat64: return fill<double>(dst, count, prod, key, first, s);
    case kBfloat16: return fill<bf16_bits>(dst, count, prod, key, first, s);
    default: return DCCL_INVALID_ARGUMENT;
    }
}

extern "C" int dccl_synth_fill(void* dst, int dtype, size_t count, int op, uint64_t seed, uint64_t buffer_id,
                               void* hip_stream) {
    return dccl_synth_fill_range(dst, dtype, count, op, seed, buffer_id, 0, hip_stream);
}
