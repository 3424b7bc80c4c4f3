// dccl_amd/csrc/combine.hpp — per-element combine operators for gfx950.
//
// The element semantics are the reference's host loop
// (/root/reference/src/core/internal_common.hpp:546-549):
//     Sum  r += s      Prod r *= s      Max if (r < s) r = s      Min if (r > s) r = s
// NOT the reference's CUDA kernel (/root/reference/src/core/reduce.cu:19-35), which
// squares recv for Prod, treats Avg as Sum and selects with >= / <=.
//
// Integers wrap (arithmetic in the unsigned type of the same width; 8-bit types
// truncate like `int8_t r += s`).  Floats: one IEEE op, round-to-nearest-even,
// denormals preserved (this library is never built with fast-math or FTZ flags).
// fp16 / bf16 widen to fp32, apply the op, round back to nearest-even; for +/* that
// equals the correctly rounded 16-bit result (24 >= 2p+2).  Max/Min are
// compare-and-select on the widened values and return the ORIGINAL operand bits.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace dccl_amd {

enum Op : int { kSum = 0, kProd = 1, kMax = 2, kMin = 3 };

// 16-bit float storage types: raw bits, so loads/stores never canonicalise.
struct f16_bits { uint16_t v; };
struct bf16_bits { uint16_t v; };

template <typename T> struct IntTraits;
template <> struct IntTraits<int8_t> { using U = uint32_t; };
template <> struct IntTraits<uint8_t> { using U = uint32_t; };
template <> struct IntTraits<int32_t> { using U = uint32_t; };
template <> struct IntTraits<uint32_t> { using U = uint32_t; };
template <> struct IntTraits<int64_t> { using U = uint64_t; };
template <> struct IntTraits<uint64_t> { using U = uint64_t; };

__device__ __forceinline__ float f16_to_f32(uint16_t h) {
    return static_cast<float>(__builtin_bit_cast(_Float16, h));
}
__device__ __forceinline__ uint16_t f32_to_f16(float f) {
    return __builtin_bit_cast(uint16_t, static_cast<_Float16>(f));
}
__device__ __forceinline__ float bf16_to_f32(uint16_t b) {
    return __builtin_bit_cast(float, static_cast<uint32_t>(b) << 16);
}
// gfx950 lowers this cast to v_cvt_pk_bf16_f32: round-to-nearest-even, NaN stays NaN.
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
    return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}

template <typename T, int OP> struct Combine {
    // integer types
    __device__ __forceinline__ static T apply(T r, T s) {
        using U = typename IntTraits<T>::U;
        if constexpr (OP == kSum) return static_cast<T>(static_cast<U>(r) + static_cast<U>(s));
        if constexpr (OP == kProd) return static_cast<T>(static_cast<U>(r) * static_cast<U>(s));
        if constexpr (OP == kMax) return (r < s) ? s : r;
        if constexpr (OP == kMin) return (r > s) ? s : r;
        return r;
    }
};

template <int OP> struct Combine<float, OP> {
    __device__ __forceinline__ static float apply(float r, float s) {
        if constexpr (OP == kSum) return r + s;
        if constexpr (OP == kProd) return r * s;
        if constexpr (OP == kMax) return (r < s) ? s : r;
        if constexpr (OP == kMin) return (r > s) ? s : r;
        return r;
    }
};

template <int OP> struct Combine<double, OP> {
    __device__ __forceinline__ static double apply(double r, double s) {
        if constexpr (OP == kSum) return r + s;
        if constexpr (OP == kProd) return r * s;
        if constexpr (OP == kMax) return (r < s) ? s : r;
        if constexpr (OP == kMin) return (r > s) ? s : r;
        return r;
    }
};

template <int OP> struct Combine<f16_bits, OP> {
    __device__ __forceinline__ static f16_bits apply(f16_bits r, f16_bits s) {
        const float a = f16_to_f32(r.v), b = f16_to_f32(s.v);
        if constexpr (OP == kSum) return f16_bits{f32_to_f16(a + b)};
        if constexpr (OP == kProd) return f16_bits{f32_to_f16(a * b)};
        if constexpr (OP == kMax) return (a < b) ? s : r;
        if constexpr (OP == kMin) return (a > b) ? s : r;
        return r;
    }
};

template <int OP> struct Combine<bf16_bits, OP> {
    __device__ __forceinline__ static bf16_bits apply(bf16_bits r, bf16_bits s) {
        const float a = bf16_to_f32(r.v), b = bf16_to_f32(s.v);
        if constexpr (OP == kSum) return bf16_bits{f32_to_bf16(a + b)};
        if constexpr (OP == kProd) return bf16_bits{f32_to_bf16(a * b)};
        if constexpr (OP == kMax) return (a < b) ? s : r;
        if constexpr (OP == kMin) return (a > b) ? s : r;
        return r;
    }
};

// One 16-byte vector = 16/sizeof(T) elements, combined lane-locally.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <typename T> struct Pack {
    static constexpr int N = 16 / sizeof(T);
    T e[N];
};

template <typename T, int OP>
__device__ __forceinline__ u32x4 combine16(u32x4 r, u32x4 s) {
    Pack<T> pr = __builtin_bit_cast(Pack<T>, r);
    const Pack<T> ps = __builtin_bit_cast(Pack<T>, s);
#pragma unroll
    for (int i = 0; i < Pack<T>::N; ++i) pr.e[i] = Combine<T, OP>::apply(pr.e[i], ps.e[i]);
    return __builtin_bit_cast(u32x4, pr);
}

}  // namespace dccl_amd
