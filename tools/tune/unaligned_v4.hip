// tools/tune/unaligned_v4.hip — tuning variants of the k-way / chain combines into a destination that is not
// element-aligned (VERDICT r3 "What's weak" #3; reduce_multi_unaligned_kernel / reduce_chain_unaligned_kernel
// in dccl_amd/csrc/reduce_kernels.hpp), fp32 Sum only.  Tools only: never linked into the product.
//
// The production kernels pay per wave (one 64-lane tile per one-wave block) for: per-operand address and
// phase arithmetic (body - p), a runtime tile-order switch, a per-operand branch between the phase-0 and
// shifted loads, per-operand bounds checks, the lane-63 extra load under its own exec-mask branch per
// operand, and a uniform 4-way switch per operand for the funnel shift.  The variants remove these:
//   * the host passes each operand's 16-B aligned base and phase (UArgs), the order is a template parameter;
//   * tiles whose every vector (and lane 63's extra vector) is inside the body take a path without bounds
//     checks, with every operand's lane-63 extra load under ONE branch;
//   * SEL: the funnel shift picks its words with selects instead of a uniform switch (phase 0 goes through
//     the same code: alignbyte by 0 returns the low word);
//   * TPW tiles per wave (consecutive), amortising the wave's set-up.
//
//   extern "C" int uv4_combine(int variant, const void* const* sends, int k, const void* own, void* dst,
//                              size_t count, void* stream)       own == nullptr: k-way into dst; else chain
#include <hip/hip_runtime.h>

#include "reduce_kernels.hpp"

namespace dccl_amd {
namespace uv4 {

struct UArgs {
    const u32x4* a[9];  // 16-B aligned base of each operand's window stream: sources, then own / dst
    unsigned p[9];      // its byte phase (0..15)
    unsigned char* dst;
    const unsigned char* own;  // chain: own's bytes (tail); multi: nullptr
    const unsigned char* src[8];  // sources' bytes (tail)
    size_t nvec, count;
};

template <int ORDER>
__device__ __forceinline__ size_t first_tile(size_t b, size_t g) {
    if constexpr (ORDER == kOrderXcd) return (b % 8) * (g / 8) + b / 8;
    else if constexpr (ORDER == kOrderBlock) return b;
    else return xcd_group_tile(b, g);
}

// 16 bytes at byte offset p of the 32 bytes (lo, hi), without a branch on p
__device__ __forceinline__ u32x4 funnel_sel(u32x4 lo, u32x4 hi, unsigned p) {
    const unsigned d[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const bool q1 = (p & 4) != 0, q2 = (p & 8) != 0;
    unsigned y[7], z[5];
#pragma unroll
    for (int j = 0; j < 7; ++j) y[j] = q1 ? d[j + 1] : d[j];
#pragma unroll
    for (int j = 0; j < 5; ++j) z[j] = q2 ? y[j + 2] : y[j];
    const unsigned b = p & 3;
    u32x4 o;
    o.x = __builtin_amdgcn_alignbyte(z[1], z[0], b);
    o.y = __builtin_amdgcn_alignbyte(z[2], z[1], b);
    o.z = __builtin_amdgcn_alignbyte(z[3], z[2], b);
    o.w = __builtin_amdgcn_alignbyte(z[4], z[3], b);
    return o;
}

__device__ __forceinline__ u32x4 funnel_sw(u32x4 lo, u32x4 hi, unsigned p) {
    const unsigned b = p & 3;
    switch (p >> 2) {
    case 0: return funnel16<0>(lo, hi, b);
    case 1: return funnel16<1>(lo, hi, b);
    case 2: return funnel16<2>(lo, hi, b);
    default: return funnel16<3>(lo, hi, b);
    }
}

template <bool SEL>
__device__ __forceinline__ u32x4 shifted(u32x4 lo, u32x4 ex, unsigned p) {
    const u32x4 hi = from_next_lane_or(lo, ex);
    return SEL ? funnel_sel(lo, hi, p) : funnel_sw(lo, hi, p);
}

// one tile: N = K + 1 operands (sources, then own / the destination's window)
template <int K, bool CHAIN, bool SEL, bool FULL>
__device__ __forceinline__ void tile(const UArgs& A, size_t t) {
    constexpr int N = K + 1;
    const size_t v = t * 64 + threadIdx.x;
    u32x4 lo[N], ex[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        lo[k] = u32x4{0u, 0u, 0u, 0u};
        ex[k] = u32x4{0u, 0u, 0u, 0u};
    }
    if constexpr (FULL) {
#pragma unroll
        for (int k = 0; k < N; ++k) lo[k] = __builtin_nontemporal_load(A.a[k] + v);
        if (threadIdx.x == 63) {
#pragma unroll
            for (int k = 0; k < N; ++k) ex[k] = A.a[k][v + 1];
        }
    } else {
#pragma unroll
        for (int k = 0; k < N; ++k) {
            if (A.p[k] != 0 ? v <= A.nvec : v < A.nvec) lo[k] = __builtin_nontemporal_load(A.a[k] + v);
            if (A.p[k] != 0 && threadIdx.x == 63 && v < A.nvec) ex[k] = A.a[k][v + 1];
        }
    }
    u32x4 acc;
    if constexpr (CHAIN) {
        acc = shifted<SEL>(lo[0], ex[0], A.p[0]);
#pragma unroll
        for (int k = 1; k < K; ++k) acc = combine16<float, kSum>(shifted<SEL>(lo[k], ex[k], A.p[k]), acc);
        acc = combine16<float, kSum>(shifted<SEL>(lo[K], ex[K], A.p[K]), acc);
    } else {
        acc = shifted<SEL>(lo[K], ex[K], A.p[K]);
#pragma unroll
        for (int k = 0; k < K; ++k) acc = combine16<float, kSum>(acc, shifted<SEL>(lo[k], ex[k], A.p[k]));
    }
    if (FULL || v < A.nvec) __builtin_nontemporal_store(acc, reinterpret_cast<u32x4_u*>(A.dst + 16 * v));
}

template <int K, bool CHAIN, int ORDER, int TPW, bool SEL>
__global__ __launch_bounds__(64) void uv4_kernel(UArgs A) {
    const size_t g = gridDim.x;
    const size_t ntiles = (A.nvec + 63) / 64;
    // a full tile: lane 63's extra vector v + 1 is inside the body too
    const size_t nfull = A.nvec >= 65 ? (A.nvec - 1) / 64 : 0;
    for (size_t t0 = first_tile<ORDER>(blockIdx.x, g) * TPW; t0 < ntiles; t0 += g * TPW) {
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
            const size_t t = t0 + j;
            if (t < nfull) tile<K, CHAIN, SEL, true>(A, t);
            else if (t < ntiles) tile<K, CHAIN, SEL, false>(A, t);
        }
    }
    if (blockIdx.x == 0)
        for (size_t j = A.nvec * 4 + threadIdx.x; j < A.count; j += 64) {
            float acc;
            if constexpr (CHAIN) {
                acc = ld_elem<float, false>(A.src[0], j);
#pragma unroll
                for (int k = 1; k < K; ++k) acc = ld_elem<float, false>(A.src[k], j) + acc;
                acc = ld_elem<float, false>(A.own, j) + acc;
            } else {
                acc = ld_elem<float, false>(A.dst, j);
#pragma unroll
                for (int k = 0; k < K; ++k) acc = acc + ld_elem<float, false>(A.src[k], j);
            }
            st_elem<float, false>(A.dst, j, acc);
        }
}

template <int K, bool CHAIN, int ORDER, int TPW, bool SEL>
int launch_v(const UArgs& A, hipStream_t st) {
    const size_t ntiles = (A.nvec + 63) / 64;
    size_t g = ceil_div(ceil_div(ntiles, size_t(TPW)), size_t(8)) * 8;
    if (g == 0) g = 8;
    UArgs a = A;
    void* args[] = {&a};
    return launch(reinterpret_cast<const void*>(&uv4_kernel<K, CHAIN, ORDER, TPW, SEL>), g, args, st, 64);
}

// variant = 100 * order + 10 * tpw + sel   (order 0 xcd, 1 block, 2 group; tpw 1, 2, 4; sel 0 switch, 1 select)
template <int K, bool CHAIN>
int dispatch(int variant, const UArgs& A, hipStream_t st) {
    const int order = variant / 100, tpw = (variant / 10) % 10;
    const bool sel = variant % 10 != 0;
    auto by_tpw = [&](auto O) -> int {
        constexpr int ORD = decltype(O)::value;
        if (tpw == 1) return sel ? launch_v<K, CHAIN, ORD, 1, true>(A, st) : launch_v<K, CHAIN, ORD, 1, false>(A, st);
        if (tpw == 2) return sel ? launch_v<K, CHAIN, ORD, 2, true>(A, st) : launch_v<K, CHAIN, ORD, 2, false>(A, st);
        if (tpw == 4) return sel ? launch_v<K, CHAIN, ORD, 4, true>(A, st) : launch_v<K, CHAIN, ORD, 4, false>(A, st);
        return DCCL_INVALID_ARGUMENT;
    };
    if (order == 0) return by_tpw(std::integral_constant<int, kOrderXcd>{});
    if (order == 1) return by_tpw(std::integral_constant<int, kOrderBlock>{});
    if (order == 2) return by_tpw(std::integral_constant<int, kOrderGroup>{});
    return DCCL_INVALID_ARGUMENT;
}

}  // namespace uv4
}  // namespace dccl_amd

using namespace dccl_amd;

extern "C" int uv4_combine(int variant, const void* const* sends, int k, const void* own, void* dst, size_t count,
                           void* stream) {
    if (k != 4 && k != 8) return DCCL_INVALID_ARGUMENT;
    uv4::UArgs A{};
    const unsigned char* d = static_cast<unsigned char*>(dst);
    for (int j = 0; j < k; ++j) {
        const uintptr_t s = reinterpret_cast<uintptr_t>(sends[j]);
        A.p[j] = unsigned(s & 15);
        A.a[j] = reinterpret_cast<const u32x4*>(s - A.p[j]);
        A.src[j] = static_cast<const unsigned char*>(sends[j]);
    }
    const uintptr_t w = reinterpret_cast<uintptr_t>(own ? own : dst);
    A.p[k] = unsigned(w & 15);
    A.a[k] = reinterpret_cast<const u32x4*>(w - A.p[k]);
    A.dst = static_cast<unsigned char*>(dst);
    A.own = static_cast<const unsigned char*>(own);
    A.nvec = count / 4;
    A.count = count;
    (void)d;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (own)
        return k == 4 ? uv4::dispatch<4, true>(variant, A, st) : uv4::dispatch<8, true>(variant, A, st);
    return k == 4 ? uv4::dispatch<4, false>(variant, A, st) : uv4::dispatch<8, false>(variant, A, st);
}
