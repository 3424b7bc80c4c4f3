// dccl_amd/csrc/local_reduce.hip — the MI355X (gfx950) local bucket-reduction combine.
//
//   recv[i] = op(recv[i], send[i]),  i in [0, count)
//
// Replaces the reference's single CUDA kernel reduce_kernel<DT> and its launcher
// do_device_reduce (/root/reference/src/core/reduce.cu:9-100).  That kernel moves one
// scalar element per thread per iteration through a runtime op switch on a grid of
// num_SMs x 256 threads; this one is an HBM stream:
//   * 16-byte (global_load_dwordx4 / global_store_dwordx4) accesses of both operands;
//   * the shipped shape (DefaultCfg, chosen by tools/tune_reduce.py on MI355X): one-wave
//     (64-thread) blocks, one 16-B vector per lane and operand, i.e. one 1 KiB tile of each
//     operand per block and ~1M blocks for 1 GiB; every load and the store non-temporal;
//   * dtype and op are template parameters (no per-element switch);
//   * unaligned head / tail elements are folded into block 0 of the same launch;
//   * operands with different 16-B phases / element misalignment take scalar kernels.
// No LDS and no MFMA: each element is touched once (BASELINE.json north_star).
//
// Roofline: HBM, 3 * count * sizeof(T) algorithmic bytes (read send, read recv, write recv).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "combine.hpp"
#include "dccl/dccl_reduce.h"
#include "dccl/dccl_reduce_tuning.h"
#include "dispatch.hpp"

namespace dccl_amd {

constexpr int kBlock = 256;  // block size of the scalar fallback kernels

// Cache policy bits of the vector kernel.
enum : int {
    kNtSend = 1,   // non-temporal load of send (read once)
    kNtRecv = 2,   // non-temporal load of recv
    kNtStore = 4,  // non-temporal store of recv
};

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    return *p;
}

// Scalar element access that is correct for any alignment of the operand bases.
template <typename T, bool ALIGNED>
__device__ __forceinline__ T ld_elem(const unsigned char* base, size_t i) {
    if constexpr (ALIGNED) return reinterpret_cast<const T*>(base)[i];
    T v;
    __builtin_memcpy(&v, base + i * sizeof(T), sizeof(T));
    return v;
}
template <typename T, bool ALIGNED>
__device__ __forceinline__ void st_elem(unsigned char* base, size_t i, T v) {
    if constexpr (ALIGNED) { reinterpret_cast<T*>(base)[i] = v; return; }
    __builtin_memcpy(base + i * sizeof(T), &v, sizeof(T));
}

// ---------------------------------------------------------------------------------
// Vector kernel.  Operands are split as [head scalars | nvec 16-B vectors | tail
// scalars]; head aligns recv (and, by construction, send) to 16 B.
// ---------------------------------------------------------------------------------
// Kernel shape: BLOCK threads, UNROLL 16-B vectors per thread per operand, cache POLICY
// bits, XCD: remap block ids so that each XCD's blocks walk one contiguous range.
template <int BLOCK_, int UNROLL_, int POLICY_, bool XCD_>
struct VecCfg {
    static constexpr int BLOCK = BLOCK_, UNROLL = UNROLL_, POLICY = POLICY_;
    static constexpr bool XCD = XCD_;
    static constexpr size_t TILE = size_t(BLOCK_) * UNROLL_;
};

template <typename T, int OP, typename C>
__device__ __forceinline__ void full_tile(const u32x4* __restrict__ vs, u32x4* __restrict__ vr, size_t base) {
    u32x4 s[C::UNROLL], r[C::UNROLL];
#pragma unroll
    for (int u = 0; u < C::UNROLL; ++u) s[u] = ld16<(C::POLICY & kNtSend) != 0>(vs + base + u * C::BLOCK);
#pragma unroll
    for (int u = 0; u < C::UNROLL; ++u) r[u] = ld16<(C::POLICY & kNtRecv) != 0>(vr + base + u * C::BLOCK);
#pragma unroll
    for (int u = 0; u < C::UNROLL; ++u) {
        const u32x4 o = combine16<T, OP>(r[u], s[u]);
        if constexpr ((C::POLICY & kNtStore) != 0) __builtin_nontemporal_store(o, vr + base + u * C::BLOCK);
        else vr[base + u * C::BLOCK] = o;
    }
}

template <typename T, int OP, typename C>
__device__ __noinline__ void partial_tile(const u32x4* __restrict__ vs, u32x4* __restrict__ vr, size_t base,
                                          size_t nvec) {
#pragma unroll
    for (int u = 0; u < C::UNROLL; ++u) {
        const size_t i = base + u * C::BLOCK;
        if (i < nvec) vr[i] = combine16<T, OP>(vr[i], vs[i]);
    }
}

// Bijective XCD-aware remap (cdna_hip_programming.md, "XCD swizzle must be bijective"):
// blocks b and b+8 share an XCD, so give each group {b : b % 8 == x} one contiguous range.
__device__ __forceinline__ size_t xcd_remap(size_t b, size_t nb) {
    const size_t q = nb / 8, r = nb % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

template <typename T, int OP, typename C>
__global__ __launch_bounds__(C::BLOCK) void reduce_vec_kernel(const unsigned char* __restrict__ send,
                                                              unsigned char* __restrict__ recv,
                                                              size_t head, size_t nvec, size_t tail) {
    const u32x4* __restrict__ vs = reinterpret_cast<const u32x4*>(send + head * sizeof(T));
    u32x4* __restrict__ vr = reinterpret_cast<u32x4*>(recv + head * sizeof(T));
    const size_t nfull = nvec / C::TILE;
    const size_t bid = C::XCD ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;

    // Full tiles: no bounds checks, all 2*UNROLL loads in flight before the first use.
    for (size_t t = bid; t < nfull; t += gridDim.x)
        full_tile<T, OP, C>(vs, vr, t * C::TILE + threadIdx.x);

    // The partial last tile goes to the block after the last full one (mod grid).
    if (nfull * C::TILE < nvec && bid == nfull % gridDim.x)
        partial_tile<T, OP, C>(vs, vr, nfull * C::TILE + threadIdx.x, nvec);

    // Scalar head [0, head) and tail [head + nvec*V, count): < 16 elements each.
    if (blockIdx.x == 0 && threadIdx.x < head + tail) {
        const size_t i = threadIdx.x < head ? threadIdx.x
                                            : head + nvec * Pack<T>::N + (threadIdx.x - head);
        const T a = ld_elem<T, true>(recv, i), b = ld_elem<T, true>(send, i);
        st_elem<T, true>(recv, i, Combine<T, OP>::apply(a, b));
    }
}

// ---------------------------------------------------------------------------------
// Scalar fallback for operands whose 16-B phases differ (ALIGNED) or that are not
// even element-aligned (!ALIGNED).  Grid-stride, 4 independent elements per thread.
// ---------------------------------------------------------------------------------
template <typename T, int OP, bool ALIGNED>
__global__ __launch_bounds__(kBlock) void reduce_scalar_kernel(const unsigned char* __restrict__ send,
                                                               unsigned char* __restrict__ recv,
                                                               size_t count) {
    const size_t stride = size_t(gridDim.x) * kBlock;
    for (size_t i0 = size_t(blockIdx.x) * kBlock * 4 + threadIdx.x; i0 < count; i0 += stride * 4) {
        T a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t i = i0 + u * kBlock;
            if (i < count) { a[u] = ld_elem<T, ALIGNED>(recv, i); b[u] = ld_elem<T, ALIGNED>(send, i); }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t i = i0 + u * kBlock;
            if (i < count) st_elem<T, ALIGNED>(recv, i, Combine<T, OP>::apply(a[u], b[u]));
        }
    }
}

// ---------------------------------------------------------------------------------
// k-way vector kernel: recv = op(...op(op(recv, s0), s1)..., s{K-1}), one pass.
// ---------------------------------------------------------------------------------
struct SendList { const unsigned char* p[8]; };

template <typename T, int OP, int K, typename C>
__global__ __launch_bounds__(C::BLOCK) void reduce_multi_vec_kernel(SendList sends, unsigned char* __restrict__ recv,
                                                                    size_t head, size_t nvec, size_t tail) {
    u32x4* __restrict__ vr = reinterpret_cast<u32x4*>(recv + head * sizeof(T));
    const size_t ntiles = (nvec + C::TILE - 1) / C::TILE;
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const size_t base = t * C::TILE + threadIdx.x;
        u32x4 r[C::UNROLL], s[K][C::UNROLL];
#pragma unroll
        for (int u = 0; u < C::UNROLL; ++u) {
            const size_t i = base + u * C::BLOCK;
            if (i < nvec) {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    s[k][u] = ld16<(C::POLICY & kNtSend) != 0>(
                        reinterpret_cast<const u32x4*>(sends.p[k] + head * sizeof(T)) + i);
                r[u] = ld16<(C::POLICY & kNtRecv) != 0>(vr + i);
            }
        }
#pragma unroll
        for (int u = 0; u < C::UNROLL; ++u) {
            const size_t i = base + u * C::BLOCK;
            if (i < nvec) {
                u32x4 acc = r[u];
#pragma unroll
                for (int k = 0; k < K; ++k) acc = combine16<T, OP>(acc, s[k][u]);
                if constexpr ((C::POLICY & kNtStore) != 0) __builtin_nontemporal_store(acc, vr + i);
                else vr[i] = acc;
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < head + tail) {
        const size_t i = threadIdx.x < head ? threadIdx.x
                                            : head + nvec * Pack<T>::N + (threadIdx.x - head);
        T acc = ld_elem<T, true>(recv, i);
#pragma unroll
        for (int k = 0; k < K; ++k) acc = Combine<T, OP>::apply(acc, ld_elem<T, true>(sends.p[k], i));
        st_elem<T, true>(recv, i, acc);
    }
}

template <typename T, int OP, bool ALIGNED>
__global__ __launch_bounds__(kBlock) void reduce_multi_scalar_kernel(SendList sends, int nsend,
                                                                     unsigned char* __restrict__ recv,
                                                                     size_t count) {
    const size_t stride = size_t(gridDim.x) * kBlock;
    for (size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x; i < count; i += stride) {
        T acc = ld_elem<T, ALIGNED>(recv, i);
        for (int k = 0; k < nsend; ++k) acc = Combine<T, OP>::apply(acc, ld_elem<T, ALIGNED>(sends.p[k], i));
        st_elem<T, ALIGNED>(recv, i, acc);
    }
}

// ---------------------------------------------------------------------------------
// Host-side launch helpers
// ---------------------------------------------------------------------------------
namespace {

// Default configuration of the shipped kernel (chosen by tools/tune on MI355X).
// One-wave blocks, one 16-B vector per lane and operand, every access non-temporal: the
// fastest shape measured on MI355X at 1 GiB (tools/tune_reduce.py, profiles/r1_tune.json).
using DefaultCfg = VecCfg<64, 1, kNtSend | kNtRecv | kNtStore, false>;
// Optional occupancy cap: DCCL_REDUCE_LDS_CAP bytes of (unused) dynamic LDS per one-wave block
// (e.g. 7168 admits 22 blocks per CU instead of 32).  Off by default: with operands in a friendly
// physical placement the uncapped launch is 0.8 % faster (profiles/r1_occupancy_pooled_*.json);
// with separately allocated operands in the slow placement mode a 22-wave cap gained 1.0-1.4 %
// (profiles/r1_tune_occupancy*.json).  Read once per process.
size_t occupancy_lds() {
    static const size_t v = [] {
        const char* e = std::getenv("DCCL_REDUCE_LDS_CAP");
        const unsigned long long x = e ? std::strtoull(e, nullptr, 10) : 0ull;
        return static_cast<size_t>(x > (64ull << 10) ? (64ull << 10) : x);
    }();
    return v;
}
constexpr size_t kMaxGrid = size_t(1) << 24;  // grid-stride beyond this (2^24 x 64 threads)

inline int launch(const void* fn, size_t grid, void** args, hipStream_t stream, int block = kBlock,
                  size_t lds_bytes = 0) {
    if (grid == 0) return DCCL_SUCCESS;
    if (grid > kMaxGrid) grid = kMaxGrid;
    const hipError_t e =
        hipLaunchKernel(fn, dim3(static_cast<unsigned>(grid)), dim3(block), args, lds_bytes, stream);
    return e == hipSuccess ? DCCL_SUCCESS : DCCL_UNHANDLED_DEVICE_ERROR;
}

inline size_t ceil_div(size_t a, size_t b) { return (a + b - 1) / b; }

struct Split {
    size_t head, nvec, tail;
};

template <typename T>
inline Split split_for_vectors(uintptr_t recv, size_t count) {
    constexpr size_t V = Pack<T>::N;
    size_t head = ((16 - (recv & 15)) & 15) / sizeof(T);
    if (head > count) head = count;
    const size_t rest = count - head;
    const size_t nvec = rest / V;
    return Split{head, nvec, rest - nvec * V};
}

template <typename T, int OP, typename C>
int launch_vec(const unsigned char* s, unsigned char* r, Split sp, hipStream_t stream, size_t grid_cap,
               size_t lds_bytes = 0) {
    size_t grid = ceil_div(sp.nvec, C::TILE);
    if (grid == 0 && (sp.head + sp.tail) > 0) grid = 1;
    if (grid_cap && grid > grid_cap) grid = grid_cap;
    void* args[] = {&s, &r, &sp.head, &sp.nvec, &sp.tail};
    return launch(reinterpret_cast<const void*>(&reduce_vec_kernel<T, OP, C>), grid, args, stream, C::BLOCK,
                  lds_bytes);
}

template <typename T, int OP>
int launch_scalar(const unsigned char* s, unsigned char* r, size_t count, bool elem_aligned, hipStream_t stream) {
    const size_t grid = ceil_div(count, size_t(kBlock) * 4);
    void* args[] = {&s, &r, &count};
    const void* fn = elem_aligned ? reinterpret_cast<const void*>(&reduce_scalar_kernel<T, OP, true>)
                                  : reinterpret_cast<const void*>(&reduce_scalar_kernel<T, OP, false>);
    return launch(fn, grid, args, stream);
}

template <typename T, int OP>
int reduce_typed(const void* send, void* recv, size_t count, hipStream_t stream) {
    const auto s = static_cast<const unsigned char*>(send);
    const auto r = static_cast<unsigned char*>(recv);
    const uintptr_t as = reinterpret_cast<uintptr_t>(send), ar = reinterpret_cast<uintptr_t>(recv);
    if ((as | ar) % sizeof(T)) return launch_scalar<T, OP>(s, r, count, false, stream);
    if ((as ^ ar) & 15) return launch_scalar<T, OP>(s, r, count, true, stream);
    return launch_vec<T, OP, DefaultCfg>(s, r, split_for_vectors<T>(ar, count), stream, 0, occupancy_lds());
}

template <typename T, int OP, int K>
int launch_multi_vec(SendList sl, unsigned char* r, Split sp, hipStream_t stream) {
    using C = DefaultCfg;
    size_t grid = ceil_div(sp.nvec, C::TILE);
    if (grid == 0 && (sp.head + sp.tail) > 0) grid = 1;
    void* args[] = {&sl, &r, &sp.head, &sp.nvec, &sp.tail};
    return launch(reinterpret_cast<const void*>(&reduce_multi_vec_kernel<T, OP, K, C>), grid, args, stream, C::BLOCK);
}

template <typename T, int OP>
int reduce_multi_typed(const void* const* sends, int nsend, void* recv, size_t count, hipStream_t stream) {
    SendList sl{};
    const uintptr_t ar = reinterpret_cast<uintptr_t>(recv);
    bool vec_ok = (ar % sizeof(T)) == 0, elem_ok = vec_ok;
    for (int k = 0; k < nsend; ++k) {
        sl.p[k] = static_cast<const unsigned char*>(sends[k]);
        const uintptr_t a = reinterpret_cast<uintptr_t>(sends[k]);
        if (a % sizeof(T)) elem_ok = vec_ok = false;
        if ((a ^ ar) & 15) vec_ok = false;
    }
    auto r = static_cast<unsigned char*>(recv);
    if (!vec_ok) {
        const size_t grid = ceil_div(count, size_t(kBlock));
        void* args[] = {&sl, &nsend, &r, &count};
        const void* fn = elem_ok ? reinterpret_cast<const void*>(&reduce_multi_scalar_kernel<T, OP, true>)
                                 : reinterpret_cast<const void*>(&reduce_multi_scalar_kernel<T, OP, false>);
        return launch(fn, grid, args, stream);
    }
    const Split sp = split_for_vectors<T>(ar, count);
    switch (nsend) {
    case 1: return launch_multi_vec<T, OP, 1>(sl, r, sp, stream);
    case 2: return launch_multi_vec<T, OP, 2>(sl, r, sp, stream);
    case 3: return launch_multi_vec<T, OP, 3>(sl, r, sp, stream);
    case 4: return launch_multi_vec<T, OP, 4>(sl, r, sp, stream);
    case 5: return launch_multi_vec<T, OP, 5>(sl, r, sp, stream);
    case 6: return launch_multi_vec<T, OP, 6>(sl, r, sp, stream);
    case 7: return launch_multi_vec<T, OP, 7>(sl, r, sp, stream);
    case 8: return launch_multi_vec<T, OP, 8>(sl, r, sp, stream);
    default: return DCCL_INVALID_ARGUMENT;
    }
}

struct ReduceFn {
    template <typename T, int OP>
    static int run(const void* send, void* recv, size_t count, hipStream_t stream) {
        return reduce_typed<T, OP>(send, recv, count, stream);
    }
};

struct ReduceMultiFn {
    template <typename T, int OP>
    static int run(const void* const* sends, int nsend, void* recv, size_t count, hipStream_t stream) {
        return reduce_multi_typed<T, OP>(sends, nsend, recv, count, stream);
    }
};

}  // namespace
}  // namespace dccl_amd

using namespace dccl_amd;

extern "C" int dccl_local_reduce(const void* send, void* recv, int dtype, size_t count, int op, void* stream) {
    const int v = validate(dtype, op);
    if (v != DCCL_SUCCESS) return v;
    if (count == 0) return DCCL_SUCCESS;
    if (send == nullptr || recv == nullptr) return DCCL_INVALID_ARGUMENT;
    return dispatch<ReduceFn>(dtype, op, send, recv, count, static_cast<hipStream_t>(stream));
}

extern "C" int dccl_local_reduce_multi(const void* const* sends, int nsend, void* recv, int dtype, size_t count,
                                       int op, void* stream) {
    const int v = validate(dtype, op);
    if (v != DCCL_SUCCESS) return v;
    if (nsend < 1 || nsend > 8 || sends == nullptr) return DCCL_INVALID_ARGUMENT;
    if (count == 0) return DCCL_SUCCESS;
    if (recv == nullptr) return DCCL_INVALID_ARGUMENT;
    for (int k = 0; k < nsend; ++k)
        if (sends[k] == nullptr) return DCCL_INVALID_ARGUMENT;
    return dispatch<ReduceMultiFn>(dtype, op, sends, nsend, recv, count, static_cast<hipStream_t>(stream));
}

// ---------------------------------------------------------------------------------
// Tuning entry: fp32 Sum with an explicit kernel variant (include/dccl/dccl_reduce_tuning.h).
// ---------------------------------------------------------------------------------
namespace {
using TuneFn = int (*)(const unsigned char*, unsigned char*, Split, hipStream_t, size_t, size_t);
template <int B, int U, int P, bool X>
int tune_one(const unsigned char* s, unsigned char* r, Split sp, hipStream_t st, size_t cap, size_t lds) {
    return launch_vec<float, kSum, VecCfg<B, U, P, X>>(s, r, sp, st, cap, lds);
}
struct TuneEntry { int block, unroll, policy, xcd; TuneFn fn; };
#define DCCL_TV(B, U, P, X) TuneEntry{B, U, P, X, &tune_one<B, U, P, X>}
const TuneEntry kTune[] = {
    DCCL_TV(64, 1, 7, 0),  DCCL_TV(64, 1, 5, 0),  DCCL_TV(64, 1, 6, 0),  DCCL_TV(64, 1, 3, 0),
    DCCL_TV(64, 1, 1, 0),  DCCL_TV(64, 1, 7, 1),  DCCL_TV(64, 2, 7, 0),  DCCL_TV(64, 4, 7, 0),
    DCCL_TV(128, 1, 7, 0), DCCL_TV(128, 1, 5, 0), DCCL_TV(128, 1, 6, 0), DCCL_TV(128, 1, 7, 1),
    DCCL_TV(256, 1, 7, 0), DCCL_TV(256, 1, 7, 1), DCCL_TV(256, 4, 7, 0), DCCL_TV(1024, 1, 7, 0),
    DCCL_TV(256, 4, 1, 0),
};
#undef DCCL_TV
}  // namespace

extern "C" int dccl_tune_num_variants(void) { return int(sizeof(kTune) / sizeof(kTune[0])); }

extern "C" int dccl_tune_variant_info(int v, int* block, int* unroll, int* policy, int* xcd) {
    if (v < 0 || v >= dccl_tune_num_variants()) return DCCL_INVALID_ARGUMENT;
    *block = kTune[v].block; *unroll = kTune[v].unroll; *policy = kTune[v].policy; *xcd = kTune[v].xcd;
    return DCCL_SUCCESS;
}

extern "C" int dccl_tune_reduce_f32_sum_lds(const void* send, void* recv, size_t count, int variant,
                                            size_t grid_cap, size_t lds_bytes, void* stream) {
    if (variant < 0 || variant >= dccl_tune_num_variants()) return DCCL_INVALID_ARGUMENT;
    if (count == 0) return DCCL_SUCCESS;
    const uintptr_t as = reinterpret_cast<uintptr_t>(send), ar = reinterpret_cast<uintptr_t>(recv);
    if (((as | ar) & 3) || ((as ^ ar) & 15)) return DCCL_INVALID_ARGUMENT;
    return kTune[variant].fn(static_cast<const unsigned char*>(send), static_cast<unsigned char*>(recv),
                             split_for_vectors<float>(ar, count), static_cast<hipStream_t>(stream), grid_cap,
                             lds_bytes);
}

extern "C" int dccl_tune_reduce_f32_sum(const void* send, void* recv, size_t count, int variant, size_t grid_cap,
                                        void* stream) {
    return dccl_tune_reduce_f32_sum_lds(send, recv, count, variant, grid_cap, 0, stream);
}

// ---------------------------------------------------------------------------------
// Tuning only: one-wave blocks, one 16-B vector per lane and operand, cache-policy bits
// chosen in inline asm (the builtins only expose `nt`).  Requires count % 256 == 0 and
// 16-B aligned operands; fp32 Sum.
// ---------------------------------------------------------------------------------
namespace {
#define DCCL_ASM_LS(BITS_S, BITS_R)                                                              \
    asm volatile("global_load_dwordx4 %0, %2, off " BITS_S "\n\t"                                \
                 "global_load_dwordx4 %1, %3, off " BITS_R "\n\t"                                \
                 "s_waitcnt vmcnt(0)"                                                            \
                 : "=&v"(a), "=&v"(b)                                                            \
                 : "v"(ps), "v"(pr)                                                              \
                 : "memory")
#define DCCL_ASM_ST(BITS) asm volatile("global_store_dwordx4 %0, %1, off " BITS :: "v"(pr), "v"(o) : "memory")

template <int FLAVOR>
__global__ __launch_bounds__(64) void tune_asm_kernel(const u32x4* __restrict__ s, u32x4* __restrict__ r,
                                                      size_t nvec) {
    const size_t i = size_t(blockIdx.x) * 64 + threadIdx.x;
    if (i >= nvec) return;
    const u32x4* ps = s + i;
    u32x4* pr = r + i;
    u32x4 a, b;
    if constexpr (FLAVOR == 0) DCCL_ASM_LS("nt", "nt");
    if constexpr (FLAVOR == 1) DCCL_ASM_LS("sc1 nt", "sc1 nt");
    if constexpr (FLAVOR == 2) DCCL_ASM_LS("sc0 sc1 nt", "sc0 sc1 nt");
    if constexpr (FLAVOR == 3) DCCL_ASM_LS("nt", "nt");
    if constexpr (FLAVOR == 4) DCCL_ASM_LS("sc1", "sc1");
    if constexpr (FLAVOR == 5) DCCL_ASM_LS("nt", "nt");
    if constexpr (FLAVOR == 6) DCCL_ASM_LS("sc0 sc1", "nt");
    const u32x4 o = combine16<float, kSum>(b, a);
    if constexpr (FLAVOR == 0) DCCL_ASM_ST("nt");
    if constexpr (FLAVOR == 1) DCCL_ASM_ST("sc1 nt");
    if constexpr (FLAVOR == 2) DCCL_ASM_ST("sc0 sc1 nt");
    if constexpr (FLAVOR == 3) DCCL_ASM_ST("sc0 sc1 nt");
    if constexpr (FLAVOR == 4) DCCL_ASM_ST("nt");
    if constexpr (FLAVOR == 5) DCCL_ASM_ST("sc1");
    if constexpr (FLAVOR == 6) DCCL_ASM_ST("nt");
}
#undef DCCL_ASM_LS
#undef DCCL_ASM_ST
}  // namespace

extern "C" int dccl_tune_asm_f32_sum(const void* send, void* recv, size_t count, int flavor, void* stream) {
    if (count % 256 || ((reinterpret_cast<uintptr_t>(send) | reinterpret_cast<uintptr_t>(recv)) & 15))
        return DCCL_INVALID_ARGUMENT;
    const size_t nvec = count / 4;
    const void* fns[] = {reinterpret_cast<const void*>(&tune_asm_kernel<0>), reinterpret_cast<const void*>(&tune_asm_kernel<1>),
                         reinterpret_cast<const void*>(&tune_asm_kernel<2>), reinterpret_cast<const void*>(&tune_asm_kernel<3>),
                         reinterpret_cast<const void*>(&tune_asm_kernel<4>), reinterpret_cast<const void*>(&tune_asm_kernel<5>),
                         reinterpret_cast<const void*>(&tune_asm_kernel<6>)};
    if (flavor < 0 || flavor >= int(sizeof(fns) / sizeof(fns[0]))) return DCCL_INVALID_ARGUMENT;
    void* args[] = {&send, &recv, const_cast<size_t*>(&nvec)};
    return launch(fns[flavor], nvec / 64, args, static_cast<hipStream_t>(stream), 64);
}

// ---------------------------------------------------------------------------------
// Tuning only: decorrelate the send/recv addresses each wave issues together.  A block of
// WAVES one-wave tiles loads recv tile w and send tile (w + SKEW) % WAVES, so the two loads a
// wave has in flight are SKEW KiB apart; send vectors are exchanged through LDS behind one
// barrier.  SKEW = 0 is the control (same pairing as the shipped kernel, plus the LDS hop).
// fp32 Sum; count must be a multiple of WAVES * 256 elements.
// ---------------------------------------------------------------------------------
namespace {
template <int WAVES, int SKEW>
__global__ __launch_bounds__(WAVES * 64) void tune_skew_kernel(const u32x4* __restrict__ s, u32x4* __restrict__ r) {
    __shared__ u32x4 lds[WAVES * 64];
    const size_t base = size_t(blockIdx.x) * WAVES * 64;
    const int w = threadIdx.x / 64, l = threadIdx.x % 64;
    const int ws = (w + SKEW) % WAVES;
    const u32x4 sv = __builtin_nontemporal_load(s + base + ws * 64 + l);
    const u32x4 rv = __builtin_nontemporal_load(r + base + w * 64 + l);
    lds[ws * 64 + l] = sv;
    __syncthreads();
    __builtin_nontemporal_store(combine16<float, kSum>(rv, lds[w * 64 + l]), r + base + w * 64 + l);
}
}  // namespace

extern "C" int dccl_tune_skew_f32_sum(const void* send, void* recv, size_t count, int waves, int skew,
                                      void* stream) {
    if (((reinterpret_cast<uintptr_t>(send) | reinterpret_cast<uintptr_t>(recv)) & 15)) return DCCL_INVALID_ARGUMENT;
    const void* fn = nullptr;
    if (waves == 8 && skew == 0) fn = reinterpret_cast<const void*>(&tune_skew_kernel<8, 0>);
    if (waves == 8 && skew == 1) fn = reinterpret_cast<const void*>(&tune_skew_kernel<8, 1>);
    if (waves == 8 && skew == 2) fn = reinterpret_cast<const void*>(&tune_skew_kernel<8, 2>);
    if (waves == 8 && skew == 4) fn = reinterpret_cast<const void*>(&tune_skew_kernel<8, 4>);
    if (waves == 4 && skew == 0) fn = reinterpret_cast<const void*>(&tune_skew_kernel<4, 0>);
    if (waves == 4 && skew == 2) fn = reinterpret_cast<const void*>(&tune_skew_kernel<4, 2>);
    if (waves == 16 && skew == 8) fn = reinterpret_cast<const void*>(&tune_skew_kernel<16, 8>);
    if (waves == 16 && skew == 4) fn = reinterpret_cast<const void*>(&tune_skew_kernel<16, 4>);
    if (fn == nullptr || count % (size_t(waves) * 256)) return DCCL_INVALID_ARGUMENT;
    void* args[] = {&send, &recv};
    return launch(fn, count / (size_t(waves) * 256), args, static_cast<hipStream_t>(stream), waves * 64);
}
