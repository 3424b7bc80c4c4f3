// dccl_amd/csrc/reduce_kernels.hpp — device code of the combine and its launch helpers, shared by
// the production entry points (local_reduce.hip) and the tuning variants (tune_kernels.hip).
// See local_reduce.hip for the design; SURVEY.md §7 / DESIGN.md §3 for the rooflines.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include <cstddef>
#include <cstdint>

#include "caps.hpp"
#include "combine.hpp"
#include "dccl/dccl_reduce.h"

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

// Vector kernel: [head scalars | nvec 16-B vectors | tail scalars], the head aligning recv to its 128-B lines.
// Shape: BLOCK threads, UNROLL 16-B vectors per thread per operand, cache POLICY bits, XCD (each XCD's blocks walk
// one contiguous range) or the tile-run order RUN; TAG keeps the production (0) and tuning (1) translation units'
// instantiations distinct.
template <int BLOCK_, int UNROLL_, int POLICY_, bool XCD_, int TAG = 0, int RUN_ = 1>
struct VecCfg {
    static constexpr int BLOCK = BLOCK_, UNROLL = UNROLL_, POLICY = POLICY_, RUN = RUN_;  // RUN: run_tile below
    static constexpr bool XCD = XCD_;
    static constexpr size_t TILE = size_t(BLOCK_) * UNROLL_;
};

// Block 0's scalar elements outside the vector body: head [0, head) (< the recv alignment) and tail
// (< one vector).  SEND_ALIGNED false: send is not element-aligned (byte loads of its elements).
template <typename T, int OP, bool SEND_ALIGNED = true>
__device__ __forceinline__ void edge_scalars(const unsigned char* send, unsigned char* recv, size_t head,
                                             size_t nvec, size_t tail) {
    for (size_t j = threadIdx.x; j < head + tail; j += blockDim.x) {
        const size_t i = j < head ? j : head + nvec * Pack<T>::N + (j - head);
        const T a = ld_elem<T, true>(recv, i), b = ld_elem<T, SEND_ALIGNED>(send, i);
        st_elem<T, true>(recv, i, Combine<T, OP>::apply(a, b));
    }
}

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

// Tile-run order: in every full group of 8 RUN blocks, block 8 RUN q + r (XCD r % 8 under the round-robin
// dispatch) takes tile 8 RUN q + RUN (r % 8) + r / 8, so each XCD walks RUN consecutive tiles of the group
// while the groups sweep the range in order: a line two neighbouring tiles share is fetched by one L2 in
// RUN - 1 of RUN cases.  RUN 1 is block order, RUN 8 the group-interleaved order (xcd_group_tile).  A partial
// last group keeps the identity.  Bijective on [0, nb).
template <int RUN>
__device__ __forceinline__ size_t run_tile(size_t b, size_t nb) {
    if constexpr (RUN == 1) return b;
    constexpr size_t span = size_t(8) * RUN;
    const size_t q = b / span, r = b % span;
    return (q + 1) * span > nb ? b : q * span + (r % 8) * RUN + r / 8;
}
__device__ __forceinline__ size_t xcd_group_tile(size_t b, size_t nb) { return run_tile<8>(b, nb); }

// First tile of block b of a g-block grid (g a multiple of 8) for the misaligned-destination kernels, by a
// uniform runtime `order`: kOrderXcd gives each XCD one contiguous range (consecutive tiles on one XCD: the
// line two tiles share meets in one L2), kOrderBlock is block order, kOrderGroup the group-interleaved order
// above (one front for the chip, 7 of 8 tile boundaries inside one XCD).  Computed once per block.
enum : int { kOrderXcd = 0, kOrderBlock = 1, kOrderGroup = 2, kOrderRun4 = 3, kOrderRun2 = 4 };
__device__ __forceinline__ size_t tile_order(int order, size_t b, size_t g) {
    return order == kOrderXcd     ? (b % 8) * (g / 8) + b / 8
           : order == kOrderBlock ? b
           : order == kOrderRun4  ? run_tile<4>(b, g)
           : order == kOrderRun2  ? run_tile<2>(b, g)
                                  : xcd_group_tile(b, g);
}

template <typename T, int OP, typename C>
__global__ __launch_bounds__(C::BLOCK) void reduce_vec_kernel(const unsigned char* __restrict__ send,
                                                              unsigned char* __restrict__ recv,
                                                              size_t head, size_t nvec, size_t tail) {
    const u32x4* __restrict__ vs = reinterpret_cast<const u32x4*>(send + head * sizeof(T));
    u32x4* __restrict__ vr = reinterpret_cast<u32x4*>(recv + head * sizeof(T));
    const size_t nfull = nvec / C::TILE;
    const size_t bid = C::XCD ? xcd_remap(blockIdx.x, gridDim.x) : run_tile<C::RUN>(blockIdx.x, gridDim.x);

    // Full tiles: no bounds checks, all 2*UNROLL loads in flight before the first use.
    for (size_t t = bid; t < nfull; t += gridDim.x)
        full_tile<T, OP, C>(vs, vr, t * C::TILE + threadIdx.x);

    // The partial last tile goes to the block after the last full one (mod grid).
    if (nfull * C::TILE < nvec && bid == nfull % gridDim.x)
        partial_tile<T, OP, C>(vs, vr, nfull * C::TILE + threadIdx.x, nvec);

    // Scalar head [0, head) and tail [head + nvec*V, count)
    if (blockIdx.x == 0) edge_scalars<T, OP>(send, recv, head, nvec, tail);
}

// Shifted vector kernel: element-aligned operands whose 16-B phases differ (any DCCL chunk size that is not
// a multiple of 16 B).  recv is walked in aligned 16-B vectors; send's bytes start p bytes (0 < p < 16) past a
// 16-B boundary A.  Every lane loads the ALIGNED vector A[v], takes A[v+1] from its right-hand neighbour (DPP
// wave shift; lane 63 loads it itself) and funnel-shifts the 32 bytes by p (v_alignbyte_b32), so every access
// stays a 16-B vector.  A[nvec] is read although only its first p bytes are send's: an aligned 16-B load never
// leaves the page of its first byte.  p may be any byte count: a send that is not element-aligned takes this
// kernel too (SEND_ALIGNED false: its head / tail elements are read bytewise).
constexpr int kNtExtra = 8;  // policy bit: non-temporal load of lane 63's extra vector

template <int Q>
__device__ __forceinline__ u32x4 funnel16(u32x4 lo, u32x4 hi, unsigned b) {
    const unsigned d[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    u32x4 o;
    o.x = __builtin_amdgcn_alignbyte(d[Q + 1], d[Q + 0], b);
    o.y = __builtin_amdgcn_alignbyte(d[Q + 2], d[Q + 1], b);
    o.z = __builtin_amdgcn_alignbyte(d[Q + 3], d[Q + 2], b);
    o.w = __builtin_amdgcn_alignbyte(d[Q + 4], d[Q + 3], b);
    return o;
}

// Cross-lane moves by one lane with DPP wave shifts (a VALU modifier, no LDS round trip), lane mapping
// verified on gfx950 by dpp_probe.hip@4f20423: wave_rol:1 (0x134) gives lane l lane (l+1) % 64's value,
// wave_shl:1 (0x130) the same except that lane 63 keeps `old`; wave_ror:1 (0x13C) gives lane l lane
// (l+63) % 64's value, wave_shr:1 (0x138) the same except that lane 0 keeps `old`.
template <int CTRL>
__device__ __forceinline__ u32x4 dpp16(u32x4 x, u32x4 old) {
    u32x4 o;
    o.x = unsigned(__builtin_amdgcn_update_dpp(int(old.x), int(x.x), CTRL, 0xF, 0xF, false));
    o.y = unsigned(__builtin_amdgcn_update_dpp(int(old.y), int(x.y), CTRL, 0xF, 0xF, false));
    o.z = unsigned(__builtin_amdgcn_update_dpp(int(old.z), int(x.z), CTRL, 0xF, 0xF, false));
    o.w = unsigned(__builtin_amdgcn_update_dpp(int(old.w), int(x.w), CTRL, 0xF, 0xF, false));
    return o;
}
// lane l < 63 receives lane l+1's x, lane 63 keeps its own `last` (the tuning code's other shifts:
// misaligned_2pass.hpp@4f20423)
__device__ __forceinline__ u32x4 from_next_lane_or(u32x4 x, u32x4 last) { return dpp16<0x130>(x, last); }

template <typename T, int OP, int POLICY, bool XCD, int TAG = 0, bool SEND_ALIGNED = true, int RUN = 1>
__global__ __launch_bounds__(64) void reduce_shift_kernel(const unsigned char* __restrict__ send,
                                                          unsigned char* __restrict__ recv, size_t head,
                                                          size_t nvec, size_t tail, unsigned p) {
    const unsigned char* sa = send + head * sizeof(T);
    const u32x4* va = reinterpret_cast<const u32x4*>(sa - p);  // A: 16-B aligned
    u32x4* vr = reinterpret_cast<u32x4*>(recv + head * sizeof(T));
    const size_t ntiles = (nvec + 63) / 64;
    const size_t bid = XCD ? xcd_remap(blockIdx.x, gridDim.x) : run_tile<RUN>(blockIdx.x, gridDim.x);
    const unsigned q = p >> 2, b = p & 3;
    const bool last_lane = threadIdx.x == 63;
    for (size_t t = bid; t < ntiles; t += gridDim.x) {  // uniform per wave: every lane reaches the lane exchange
        const size_t v = t * 64 + threadIdx.x;
        u32x4 lo = {0u, 0u, 0u, 0u}, ex = {0u, 0u, 0u, 0u}, r = {0u, 0u, 0u, 0u};
        if (v <= nvec) lo = ld16<(POLICY & kNtSend) != 0>(va + v);
        if (v < nvec) r = ld16<(POLICY & kNtRecv) != 0>(vr + v);
        if (last_lane && v < nvec) ex = ld16<(POLICY & kNtExtra) != 0>(va + v + 1);
        const u32x4 hi = from_next_lane_or(lo, ex);
        if (v < nvec) {
            u32x4 s;
            switch (q) {  // uniform
            case 0: s = funnel16<0>(lo, hi, b); break;
            case 1: s = funnel16<1>(lo, hi, b); break;
            case 2: s = funnel16<2>(lo, hi, b); break;
            default: s = funnel16<3>(lo, hi, b); break;
            }
            const u32x4 o = combine16<T, OP>(r, s);
            if constexpr ((POLICY & kNtStore) != 0) __builtin_nontemporal_store(o, vr + v);
            else vr[v] = o;
        }
    }
    if (blockIdx.x == 0) edge_scalars<T, OP, SEND_ALIGNED>(send, recv, head, nvec, tail);
}

// ---------------------------------------------------------------------------------
// A recv that is not element-aligned (e.g. fp32 at an odd byte address; the reference's host loop takes
// it with a warning, internal_common.hpp:504-512, its CUDA kernel not at all).  gfx950 executes
// global_store_dwordx4 at any byte address (unaligned_probe.hip@4f20423 checks every element), so lane i owns
// the 16 bytes of elements [V i, V i + V) at their displaced address (V = 16 / sizeof(T)): adjacent lanes'
// windows are disjoint and hold whole elements, so no byte is written twice.  Both operands' windows are
// read the shifted kernel's way (aligned loads, lane exchange, funnel shift by the operand's own phase);
// unaligned 16-B loads of recv ran 2-5 points slower, of send 7-10.  A 1 KiB tile spans 9 lines of recv,
// one shared with the next tile: the launch takes the group-interleaved tile order (tile_order), so 7 of 8 such
// lines meet in one L2 while the chip sweeps one front, uncapped: 85.1-85.2 % of peak, the aligned kernel's
// rate, against 80.7-82.1 % for round 2's XCD ranges under a 24-wave cap (profiles/r3_s4_*).  The tail
// (< V elements) is block 0's, element by element.  Kernel: after ld_phased below.
// ---------------------------------------------------------------------------------
typedef u32x4 u32x4_u __attribute__((aligned(1)));

// ---------------------------------------------------------------------------------
// k-way vector kernel: recv = op(...op(op(recv, s0), s1)..., s{K-1}), one pass.
// ---------------------------------------------------------------------------------
struct SendList { const unsigned char* p[8]; };

template <typename T, int OP, int K, typename C>
__global__ __launch_bounds__(C::BLOCK) void reduce_multi_vec_kernel(SendList sends, unsigned char* __restrict__ recv,
                                                                    size_t head, size_t nvec, size_t tail) {
    u32x4* __restrict__ vr = reinterpret_cast<u32x4*>(recv + head * sizeof(T));
    const size_t ntiles = (nvec + C::TILE - 1) / C::TILE;
    for (size_t t = C::XCD ? xcd_remap(blockIdx.x, gridDim.x) : run_tile<C::RUN>(blockIdx.x, gridDim.x); t < ntiles;
         t += gridDim.x) {
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
    if (blockIdx.x == 0) {
        for (size_t j = threadIdx.x; j < head + tail; j += blockDim.x) {
            const size_t i = j < head ? j : head + nvec * Pack<T>::N + (j - head);
            T acc = ld_elem<T, true>(recv, i);
#pragma unroll
            for (int k = 0; k < K; ++k) acc = Combine<T, OP>::apply(acc, ld_elem<T, true>(sends.p[k], i));
            st_elem<T, true>(recv, i, acc);
        }
    }
}

// ---------------------------------------------------------------------------------
// Chain kernel: the association order of the reference's ring reduce-scatter for one chunk,
// in one pass over all contributions:
//     dst = op(own, op(s{K-1}, ... op(s2, op(s1, s0))))
// Every application is op(recv = the next rank's own data, send = the partial that arrived),
// exactly as reduce_scatter_ring.cpp:84-94 applies it, so results are bit-identical to the ring
// for every dtype and op (Max/Min NaN and signed-zero selection included).  `own` may alias `dst`.
// ---------------------------------------------------------------------------------
template <typename T, int OP, int K, typename C>
__global__ __launch_bounds__(C::BLOCK) void reduce_chain_vec_kernel(SendList sends, const unsigned char* own,
                                                                    unsigned char* dst, size_t head, size_t nvec,
                                                                    size_t tail) {
    static_assert(C::UNROLL == 1, "one vector per lane");
    const size_t off = head * sizeof(T);
    const u32x4* vo = reinterpret_cast<const u32x4*>(own + off);
    u32x4* vd = reinterpret_cast<u32x4*>(dst + off);
    const size_t ntiles = (nvec + C::TILE - 1) / C::TILE;
    for (size_t t = C::XCD ? xcd_remap(blockIdx.x, gridDim.x) : run_tile<C::RUN>(blockIdx.x, gridDim.x); t < ntiles;
         t += gridDim.x) {
        const size_t i = t * C::TILE + threadIdx.x;
        if (i < nvec) {
            u32x4 s[K];
#pragma unroll
            for (int k = 0; k < K; ++k)
                s[k] = ld16<(C::POLICY & kNtSend) != 0>(reinterpret_cast<const u32x4*>(sends.p[k] + off) + i);
            const u32x4 o = ld16<true>(vo + i);
            u32x4 acc = s[0];
#pragma unroll
            for (int k = 1; k < K; ++k) acc = combine16<T, OP>(s[k], acc);
            __builtin_nontemporal_store(combine16<T, OP>(o, acc), vd + i);
        }
    }
    if (blockIdx.x == 0) {
        for (size_t j = threadIdx.x; j < head + tail; j += blockDim.x) {
            const size_t i = j < head ? j : head + nvec * Pack<T>::N + (j - head);
            T acc = ld_elem<T, true>(sends.p[0], i);
#pragma unroll
            for (int k = 1; k < K; ++k) acc = Combine<T, OP>::apply(ld_elem<T, true>(sends.p[k], i), acc);
            st_elem<T, true>(dst, i, Combine<T, OP>::apply(ld_elem<T, true>(own, i), acc));
        }
    }
}

// ---------------------------------------------------------------------------------
// Phased k-way and chain kernels: an element-aligned destination and operands whose 16-B phases differ
// from it (DCCL chunks of sizes that are not a multiple of 16 B, read from peers or scratchpads at
// other phases; operands need not even be element-aligned).  Operand j's body starts p_j bytes
// (ph.p[j], 0 <= p_j < 16) past a 16-B boundary A_j.  An operand with p_j != 0 is read the shifted
// kernel's way: every lane loads the ALIGNED vector A_j[v] (non-temporal), lane 63 also loads A_j[v+1]
// (through the caches), the other lanes take it from their right-hand neighbour (DPP wave shift), and
// the 32 bytes are funnel-shifted by p_j (v_alignbyte_b32, any byte count).  An operand with p_j == 0 is
// a plain vector load.  The head / tail scalars read operands bytewise (any alignment).  One operand at a
// time, uncapped (74-79 % of peak, profiles/r1_s5_phased_probe.json), or, from k = 5 (k-way) / k = 4 (chain),
// every operand's loads first under caps of their own (below; DESIGN.md §3, caps.hpp).
// One-wave blocks and a per-tile loop uniform per wave: every lane reaches the lane exchange.
// ---------------------------------------------------------------------------------
struct PhaseList { unsigned p[9]; };

// ld_phased in two halves, so a kernel can issue every operand's loads before it uses any of them (one wait
// for all of them instead of one round trip per operand): ld_phased_issue starts the loads,
// ld_phased_finish does the lane exchange and the shift.  All 64 lanes call both (p is uniform).
struct PhasedLoad {
    u32x4 lo, ex;
};
__device__ __forceinline__ PhasedLoad ld_phased_issue(const unsigned char* body, unsigned p, size_t v, size_t nvec) {
    // one load path for every phase (no uniform branch between two operands' loads): with p == 0, va is
    // the body itself and vector nvec is not read
    PhasedLoad x{{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
    const u32x4* va = reinterpret_cast<const u32x4*>(body - p);
    if (p != 0 ? v <= nvec : v < nvec) x.lo = __builtin_nontemporal_load(va + v);  // A[nvec]: the last p bytes
    if (p != 0 && (threadIdx.x & 63) == 63 && v < nvec) x.ex = va[v + 1];
    return x;
}
__device__ __forceinline__ u32x4 ld_phased_finish(const PhasedLoad& x, unsigned p) {
    if (p == 0) return x.lo;
    const u32x4 hi = from_next_lane_or(x.lo, x.ex);
    const unsigned b = p & 3;
    switch (p >> 2) {  // uniform
    case 0: return funnel16<0>(x.lo, hi, b);
    case 1: return funnel16<1>(x.lo, hi, b);
    case 2: return funnel16<2>(x.lo, hi, b);
    default: return funnel16<3>(x.lo, hi, b);
    }
}

// XCD: consecutive tiles on one XCD (xcd_remap), so the vector lane 63 reads past its tile and the
// next tile's first line meet in one L2.  It pays while few operands share the L2.  1 GiB fp32 Sum,
// sources 4 B off phase, on two boxes (phased_probe.py@4f20423, profiles/r2_phased_xcd_*.json), points of
// HBM peak gained: k-way k = 2 +2.1..+4.0, k = 3 +2.1..+2.5, k = 4 +0.6..+1.7, k = 5 -0.2..+0.8,
// k = 7 -2.2..-5.1; the chain kernel (in place) within 0.5 points of the same at every k.
inline constexpr int kPhasedXcdMaxK = 4;
// Where caps::kMultiPhasedFirst / kChainPhasedFirst (caps.hpp) have an entry, the phased kernels take the
// loads-first form (ld_phased_issue / ld_phased_finish) under that cap and in the tile-run order caps::kRun
// (caps.hpp); uncapped it loses (too many streams in flight).

// The 16 body bytes of vector v (zero for v >= nvec) of an operand whose body starts at `body`,
// phase p.  All 64 lanes must call it (p is uniform).
__device__ __forceinline__ u32x4 ld_phased(const unsigned char* body, unsigned p, size_t v, size_t nvec) {
    u32x4 lo = {0u, 0u, 0u, 0u};
    if (p == 0) {
        if (v < nvec) lo = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(body) + v);
        return lo;
    }
    const u32x4* va = reinterpret_cast<const u32x4*>(body - p);
    const bool last_lane = (threadIdx.x & 63) == 63;
    u32x4 ex = {0u, 0u, 0u, 0u};
    if (v <= nvec) lo = __builtin_nontemporal_load(va + v);  // A[nvec] holds the last p body bytes
    if (last_lane && v < nvec) ex = va[v + 1];
    const u32x4 hi = from_next_lane_or(lo, ex);
    const unsigned b = p & 3;
    switch (p >> 2) {  // uniform
    case 0: return funnel16<0>(lo, hi, b);
    case 1: return funnel16<1>(lo, hi, b);
    case 2: return funnel16<2>(lo, hi, b);
    default: return funnel16<3>(lo, hi, b);
    }
}

// grid: a multiple of 8.  Block b takes tile (b % 8) * (grid / 8) + b / 8, then strides by grid.  Lane i's
// window is recv's elements [V i, V i + V): its 16 bytes at the displaced address are read the shifted
// kernel's way (aligned loads, lane exchange, funnel shift by recv & 15), like send's (phase p), all loads
// issued before the first wait, and the result goes back with one 16-B store at the displaced address.
// Reading recv through aligned loads instead of one unaligned 16-B load per lane: +2.4 points (recv + 1 B)
// and +4.8 (recv + 2 B, send + 3 B) on one box, bit-exact (profiles/r3_s2_ab_recv_phased.json).  The bytes a
// lane takes from A[v + 1] are its own window's, so the neighbouring tile's stores never touch them.
template <typename T, int OP>
__global__ __launch_bounds__(64) void reduce_unaligned_kernel(const unsigned char* __restrict__ send, unsigned p,
                                                              unsigned char* __restrict__ recv, size_t nvec,
                                                              size_t count, int order) {
    const size_t g = gridDim.x;
    const unsigned pr = unsigned(reinterpret_cast<uintptr_t>(recv) & 15);
    for (size_t t = tile_order(order, blockIdx.x, g); t * 64 < nvec; t += g) {
        const size_t i = t * 64 + threadIdx.x;
        const PhasedLoad xr = ld_phased_issue(recv, pr, i, nvec), xs = ld_phased_issue(send, p, i, nvec);
        const u32x4 o = combine16<T, OP>(ld_phased_finish(xr, pr), ld_phased_finish(xs, p));
        if (i < nvec) __builtin_nontemporal_store(o, reinterpret_cast<u32x4_u*>(recv + 16 * i));
    }
    if (blockIdx.x == 0)
        for (size_t j = nvec * Pack<T>::N + threadIdx.x; j < count; j += 64)
            st_elem<T, false>(recv, j, Combine<T, OP>::apply(ld_elem<T, false>(recv, j), ld_elem<T, false>(send, j)));
}

template <typename T, int OP, int K, bool XCD, bool FIRST = false, int RUN = 1>
__global__ __launch_bounds__(64) void reduce_multi_phased_kernel(SendList sends, PhaseList ph,
                                                                 unsigned char* __restrict__ recv, size_t head,
                                                                 size_t nvec, size_t tail) {
    const size_t off = head * sizeof(T);
    u32x4* vr = reinterpret_cast<u32x4*>(recv + off);
    const size_t ntiles = (nvec + 63) / 64;
    for (size_t t = XCD ? xcd_remap(blockIdx.x, gridDim.x) : run_tile<RUN>(blockIdx.x, gridDim.x); t < ntiles;
         t += gridDim.x) {
        const size_t v = t * 64 + threadIdx.x;
        if constexpr (FIRST) {  // recv, then every source's loads, then the shifts and combines
            u32x4 acc = {0u, 0u, 0u, 0u};
            if (v < nvec) acc = ld16<true>(vr + v);
            PhasedLoad x[K];
#pragma unroll
            for (int k = 0; k < K; ++k) x[k] = ld_phased_issue(sends.p[k] + off, ph.p[k], v, nvec);
#pragma unroll
            for (int k = 0; k < K; ++k) acc = combine16<T, OP>(acc, ld_phased_finish(x[k], ph.p[k]));
            if (v < nvec) __builtin_nontemporal_store(acc, vr + v);
            continue;
        }
        u32x4 s[K];
#pragma unroll
        for (int k = 0; k < K; ++k) s[k] = ld_phased(sends.p[k] + off, ph.p[k], v, nvec);
        if (v < nvec) {
            u32x4 acc = ld16<true>(vr + v);
#pragma unroll
            for (int k = 0; k < K; ++k) acc = combine16<T, OP>(acc, s[k]);
            __builtin_nontemporal_store(acc, vr + v);
        }
    }
    if (blockIdx.x == 0) {
        for (size_t j = threadIdx.x; j < head + tail; j += blockDim.x) {
            const size_t i = j < head ? j : head + nvec * Pack<T>::N + (j - head);
            T acc = ld_elem<T, true>(recv, i);
#pragma unroll
            for (int k = 0; k < K; ++k) acc = Combine<T, OP>::apply(acc, ld_elem<T, false>(sends.p[k], i));
            st_elem<T, true>(recv, i, acc);
        }
    }
}

// Chain order as reduce_chain_vec_kernel; ph.p[K] is own's phase.
template <typename T, int OP, int K, bool XCD, bool FIRST = false, int RUN = 1>
__global__ __launch_bounds__(64) void reduce_chain_phased_kernel(SendList sends, PhaseList ph,
                                                                 const unsigned char* own, unsigned char* dst,
                                                                 size_t head, size_t nvec, size_t tail) {
    const size_t off = head * sizeof(T);
    u32x4* vd = reinterpret_cast<u32x4*>(dst + off);
    const size_t ntiles = (nvec + 63) / 64;
    for (size_t t = XCD ? xcd_remap(blockIdx.x, gridDim.x) : run_tile<RUN>(blockIdx.x, gridDim.x); t < ntiles;
         t += gridDim.x) {
        const size_t v = t * 64 + threadIdx.x;
        if constexpr (FIRST) {  // every operand's loads, then the shifts and combines in chain order
            PhasedLoad x[K + 1];
#pragma unroll
            for (int k = 0; k < K; ++k) x[k] = ld_phased_issue(sends.p[k] + off, ph.p[k], v, nvec);
            x[K] = ld_phased_issue(own + off, ph.p[K], v, nvec);
            u32x4 acc = ld_phased_finish(x[0], ph.p[0]);
#pragma unroll
            for (int k = 1; k < K; ++k) acc = combine16<T, OP>(ld_phased_finish(x[k], ph.p[k]), acc);
            const u32x4 o = ld_phased_finish(x[K], ph.p[K]);
            if (v < nvec) __builtin_nontemporal_store(combine16<T, OP>(o, acc), vd + v);
            continue;
        }
        u32x4 s[K];
#pragma unroll
        for (int k = 0; k < K; ++k) s[k] = ld_phased(sends.p[k] + off, ph.p[k], v, nvec);
        const u32x4 o = ld_phased(own + off, ph.p[K], v, nvec);
        if (v < nvec) {
            u32x4 acc = s[0];
#pragma unroll
            for (int k = 1; k < K; ++k) acc = combine16<T, OP>(s[k], acc);
            __builtin_nontemporal_store(combine16<T, OP>(o, acc), vd + v);
        }
    }
    if (blockIdx.x == 0) {
        for (size_t j = threadIdx.x; j < head + tail; j += blockDim.x) {
            const size_t i = j < head ? j : head + nvec * Pack<T>::N + (j - head);
            T acc = ld_elem<T, false>(sends.p[0], i);
#pragma unroll
            for (int k = 1; k < K; ++k) acc = Combine<T, OP>::apply(ld_elem<T, false>(sends.p[k], i), acc);
            st_elem<T, true>(dst, i, Combine<T, OP>::apply(ld_elem<T, false>(own, i), acc));
        }
    }
}

// ---------------------------------------------------------------------------------
// k-way and chain combines into a destination that is not element-aligned (reduce_unaligned_kernel's
// scheme for K operands): lane i's window is the 16 bytes of elements [V i, V i + V) at the destination's
// own address (one unaligned 16-B store, gfx950); every operand -- the sources, then `own` (chain) or the
// destination's own window (k-way) -- is read at its own byte phase through aligned loads, the lane
// exchange and the funnel shift, one operand at a time.  A window and the bytes lane i reads for it belong
// to lane i alone, so own may alias dst.  Round 4: the host passes every operand's 16-B
// aligned base and phase (WindowArgs), the tile order is a template parameter, and tiles whose every vector
// (and lane 63's extra one) lies inside the body take a path without bounds checks; the tail (< V
// elements) is block 0's, element by element.  Grid: a multiple of 8 (the XCD / group orders).
// ---------------------------------------------------------------------------------
struct WindowArgs {
    const u32x4* a[9];  // 16-B aligned base of each operand's window stream: sources, then own / the destination
    unsigned p[9];      // its byte phase, 0..15
    const unsigned char* src[8];  // the sources' bytes (tail elements)
    const unsigned char* own;     // chain: own's bytes; k-way: the destination's
    unsigned char* dst;
    size_t nvec, count;
};

template <int ORDER>
__device__ __forceinline__ size_t first_tile(size_t b, size_t g) {
    if constexpr (ORDER == kOrderXcd) return (b % 8) * (g / 8) + b / 8;
    else if constexpr (ORDER == kOrderBlock) return b;
    else if constexpr (ORDER == kOrderRun4) return run_tile<4>(b, g);
    else if constexpr (ORDER == kOrderRun2) return run_tile<2>(b, g);
    else return xcd_group_tile(b, g);
}

// One operand's window for vector v (the 16 bytes at byte phase p past aligned vector a[v]); all 64 lanes
// call it (p is uniform).  FULL: v and lane 63's extra vector v + 1 lie inside the body (no bounds checks).
template <bool FULL>
__device__ __forceinline__ u32x4 ld_window(const u32x4* a, unsigned p, size_t v, size_t nvec) {
    u32x4 lo = {0u, 0u, 0u, 0u}, ex = {0u, 0u, 0u, 0u};
    if (FULL || (p != 0 ? v <= nvec : v < nvec)) lo = __builtin_nontemporal_load(a + v);
    if (p == 0) return lo;
    if ((threadIdx.x & 63) == 63 && (FULL || v < nvec)) ex = a[v + 1];
    const u32x4 hi = from_next_lane_or(lo, ex);
    const unsigned b = p & 3;
    switch (p >> 2) {  // uniform
    case 0: return funnel16<0>(lo, hi, b);
    case 1: return funnel16<1>(lo, hi, b);
    case 2: return funnel16<2>(lo, hi, b);
    default: return funnel16<3>(lo, hi, b);
    }
}

template <typename T, int OP, int K, bool CHAIN, bool FULL>
__device__ __forceinline__ void window_tile(const WindowArgs& A, size_t t) {
    const size_t v = t * 64 + threadIdx.x;
    u32x4 acc;
    if constexpr (CHAIN) {  // dst = op(own, op(s{K-1}, ... op(s1, s0)))
        acc = ld_window<FULL>(A.a[0], A.p[0], v, A.nvec);
#pragma unroll
        for (int k = 1; k < K; ++k) acc = combine16<T, OP>(ld_window<FULL>(A.a[k], A.p[k], v, A.nvec), acc);
        acc = combine16<T, OP>(ld_window<FULL>(A.a[K], A.p[K], v, A.nvec), acc);
    } else {  // recv = op(...op(op(recv, s0), s1)..., s{K-1})
        acc = ld_window<FULL>(A.a[K], A.p[K], v, A.nvec);
#pragma unroll
        for (int k = 0; k < K; ++k) acc = combine16<T, OP>(acc, ld_window<FULL>(A.a[k], A.p[k], v, A.nvec));
    }
    if (FULL || v < A.nvec) __builtin_nontemporal_store(acc, reinterpret_cast<u32x4_u*>(A.dst + 16 * v));
}

// The loads-first tile: every operand's aligned load and lane 63's extra vectors are issued before any lane
// exchange, so a wave waits once per tile.  (In window_tile the uniform phase branches keep the compiler
// from hoisting the next operand's load above the previous one's exchange: K + 1 round trips per tile.)
// Twice the VGPRs in flight, so it runs under a resident-wave cap (caps.hpp kWindowsFirst).
template <typename T, int OP, int K, bool CHAIN, bool FULL>
__device__ __forceinline__ void window_tile_first(const WindowArgs& A, size_t t) {
    const size_t v = t * 64 + threadIdx.x;
    u32x4 lo[K + 1], ex[K + 1];
#pragma unroll
    for (int k = 0; k <= K; ++k) {
        lo[k] = u32x4{0u, 0u, 0u, 0u};
        ex[k] = u32x4{0u, 0u, 0u, 0u};
        if (FULL || (A.p[k] != 0 ? v <= A.nvec : v < A.nvec)) lo[k] = __builtin_nontemporal_load(A.a[k] + v);
    }
    if ((threadIdx.x & 63) == 63) {
#pragma unroll
        for (int k = 0; k <= K; ++k)
            if (A.p[k] != 0 && (FULL || v < A.nvec)) ex[k] = A.a[k][v + 1];
    }
    u32x4 w[K + 1];
#pragma unroll
    for (int k = 0; k <= K; ++k) {
        const unsigned p = A.p[k];
        if (p == 0) {
            w[k] = lo[k];
            continue;
        }
        const u32x4 hi = from_next_lane_or(lo[k], ex[k]);
        const unsigned b = p & 3;
        switch (p >> 2) {  // uniform
        case 0: w[k] = funnel16<0>(lo[k], hi, b); break;
        case 1: w[k] = funnel16<1>(lo[k], hi, b); break;
        case 2: w[k] = funnel16<2>(lo[k], hi, b); break;
        default: w[k] = funnel16<3>(lo[k], hi, b); break;
        }
    }
    u32x4 acc;
    if constexpr (CHAIN) {
        acc = w[0];
#pragma unroll
        for (int k = 1; k < K; ++k) acc = combine16<T, OP>(w[k], acc);
        acc = combine16<T, OP>(w[K], acc);
    } else {
        acc = w[K];
#pragma unroll
        for (int k = 0; k < K; ++k) acc = combine16<T, OP>(acc, w[k]);
    }
    if (FULL || v < A.nvec) __builtin_nontemporal_store(acc, reinterpret_cast<u32x4_u*>(A.dst + 16 * v));
}

template <typename T, int OP, int K, bool CHAIN, int ORDER, bool FIRST = false>
__global__ __launch_bounds__(64) void reduce_windows_kernel(WindowArgs A) {
    const size_t g = gridDim.x;
    const size_t ntiles = (A.nvec + 63) / 64;
    for (size_t t = first_tile<ORDER>(blockIdx.x, g); t < ntiles; t += g) {
        const bool full = (t + 1) * 64 < A.nvec;  // lane 63's extra vector inside too
        if constexpr (FIRST) {
            if (full) window_tile_first<T, OP, K, CHAIN, true>(A, t);
            else window_tile_first<T, OP, K, CHAIN, false>(A, t);
        } else if (full) {
            window_tile<T, OP, K, CHAIN, true>(A, t);
        } else {
            window_tile<T, OP, K, CHAIN, false>(A, t);
        }
    }
    if (blockIdx.x == 0)
        for (size_t j = A.nvec * Pack<T>::N + threadIdx.x; j < A.count; j += 64) {
            T acc;
            if constexpr (CHAIN) {
                acc = ld_elem<T, false>(A.src[0], j);
#pragma unroll
                for (int k = 1; k < K; ++k) acc = Combine<T, OP>::apply(ld_elem<T, false>(A.src[k], j), acc);
                acc = Combine<T, OP>::apply(ld_elem<T, false>(A.own, j), acc);
            } else {
                acc = ld_elem<T, false>(A.own, j);
#pragma unroll
                for (int k = 0; k < K; ++k) acc = Combine<T, OP>::apply(acc, ld_elem<T, false>(A.src[k], j));
            }
            st_elem<T, false>(A.dst, j, acc);
        }
}

// The round-3 forms, kept for k <= 2: every operand through ld_phased with bounds checks and a
// runtime tile order.  At k = 2 they run 2.5-4.3 points faster than reduce_windows_kernel (83.8 / 82.1 % against
// 79.5 / 79.6 %, destination + 2 B, sources in phase; profiles/r4_s7_ab_windows.json), which wins from k = 3.
template <typename T, int OP, int K>
__global__ __launch_bounds__(64) void reduce_multi_unaligned_kernel(SendList sends, PhaseList ph,
                                                                    unsigned char* __restrict__ recv, size_t nvec,
                                                                    size_t count, int order) {
    const size_t g = gridDim.x;
    const unsigned pr = unsigned(reinterpret_cast<uintptr_t>(recv) & 15);
    for (size_t t = tile_order(order, blockIdx.x, g); t * 64 < nvec; t += g) {
        const size_t i = t * 64 + threadIdx.x;
        const PhasedLoad xr = ld_phased_issue(recv, pr, i, nvec);  // recv's window, as reduce_unaligned_kernel
        u32x4 s[K];
#pragma unroll
        for (int k = 0; k < K; ++k) s[k] = ld_phased(sends.p[k], ph.p[k], i, nvec);
        u32x4 acc = ld_phased_finish(xr, pr);
#pragma unroll
        for (int k = 0; k < K; ++k) acc = combine16<T, OP>(acc, s[k]);
        if (i < nvec) __builtin_nontemporal_store(acc, reinterpret_cast<u32x4_u*>(recv + 16 * i));
    }
    if (blockIdx.x == 0)
        for (size_t j = nvec * Pack<T>::N + threadIdx.x; j < count; j += 64) {
            T acc = ld_elem<T, false>(recv, j);
#pragma unroll
            for (int k = 0; k < K; ++k) acc = Combine<T, OP>::apply(acc, ld_elem<T, false>(sends.p[k], j));
            st_elem<T, false>(recv, j, acc);
        }
}

// Chain order as reduce_chain_vec_kernel; ph.p[K] is own's phase.
template <typename T, int OP, int K>
__global__ __launch_bounds__(64) void reduce_chain_unaligned_kernel(SendList sends, PhaseList ph,
                                                                    const unsigned char* own, unsigned char* dst,
                                                                    size_t nvec, size_t count, int order) {
    const size_t g = gridDim.x;
    for (size_t t = tile_order(order, blockIdx.x, g); t * 64 < nvec; t += g) {
        const size_t i = t * 64 + threadIdx.x;
        u32x4 s[K];
#pragma unroll
        for (int k = 0; k < K; ++k) s[k] = ld_phased(sends.p[k], ph.p[k], i, nvec);
        const u32x4 o = ld_phased(own, ph.p[K], i, nvec);
        u32x4 acc = s[0];
#pragma unroll
        for (int k = 1; k < K; ++k) acc = combine16<T, OP>(s[k], acc);
        if (i < nvec) __builtin_nontemporal_store(combine16<T, OP>(o, acc), reinterpret_cast<u32x4_u*>(dst + 16 * i));
    }
    if (blockIdx.x == 0)
        for (size_t j = nvec * Pack<T>::N + threadIdx.x; j < count; j += 64) {
            T acc = ld_elem<T, false>(sends.p[0], j);
#pragma unroll
            for (int k = 1; k < K; ++k) acc = Combine<T, OP>::apply(ld_elem<T, false>(sends.p[k], j), acc);
            st_elem<T, false>(dst, j, Combine<T, OP>::apply(ld_elem<T, false>(own, j), acc));
        }
}

// ---------------------------------------------------------------------------------
// Host-side launch helpers
// ---------------------------------------------------------------------------------
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

// Runtime source count -> compile-time K: f(std::integral_constant<int, K>{}) for k in [LO, HI],
// DCCL_INVALID_ARGUMENT outside it.
template <int LO, int HI, typename F>
int with_k(int k, F&& f) {
    if constexpr (LO > HI) {
        (void)k;
        (void)f;
        return DCCL_INVALID_ARGUMENT;
    } else {
        if (k == LO) return f(std::integral_constant<int, LO>{});
        return with_k<LO + 1, HI>(k, static_cast<F&&>(f));
    }
}

struct Split {
    size_t head, nvec, tail;
};

// head scalars bring recv to an `align`-byte boundary (16 or more, a power of two).  Aligning recv to
// its 128-B lines keeps every tile's recv loads and stores whole-line: a recv that straddles lines
// costs 10-15 % (phase_probe.py@4f20423, profiles/r1_s3_phase_probe.json).  head < align / sizeof(T).
template <typename T>
inline Split split_for_vectors(uintptr_t recv, size_t count, size_t align = 16) {
    constexpr size_t V = Pack<T>::N;
    size_t head = ((align - (recv & (align - 1))) & (align - 1)) / sizeof(T);
    if (head > count) head = count;
    const size_t rest = count - head;
    const size_t nvec = rest / V;
    return Split{head, nvec, rest - nvec * V};
}

template <typename T, int OP, typename C>
int launch_vec(const unsigned char* s, unsigned char* r, Split sp, hipStream_t stream, size_t grid_cap = 0,
               size_t lds_bytes = 0) {
    size_t grid = ceil_div(sp.nvec, C::TILE);
    if (grid == 0 && (sp.head + sp.tail) > 0) grid = 1;
    if (grid_cap && grid > grid_cap) grid = grid_cap;
    void* args[] = {&s, &r, &sp.head, &sp.nvec, &sp.tail};
    return launch(reinterpret_cast<const void*>(&reduce_vec_kernel<T, OP, C>), grid, args, stream, C::BLOCK,
                  lds_bytes);
}

// Element-aligned operands with different 16-B phases (or an element-aligned recv and a send at any byte
// address, SEND_ALIGNED false): the shifted vector kernel.
template <typename T, int OP, int POLICY, bool XCD, int TAG = 0, bool SEND_ALIGNED = true, int RUN = 1>
int launch_shift(const unsigned char* s, unsigned char* r, size_t count, hipStream_t stream, size_t align = 16,
                 size_t lds_bytes = 0, size_t grid_cap = 0) {
    Split sp = split_for_vectors<T>(reinterpret_cast<uintptr_t>(r), count, align);
    unsigned p = unsigned((reinterpret_cast<uintptr_t>(s) + sp.head * sizeof(T)) & 15);
    size_t grid = ceil_div(sp.nvec, size_t(64));
    if (grid == 0 && (sp.head + sp.tail) > 0) grid = 1;
    if (grid_cap && grid > grid_cap) grid = grid_cap;
    void* args[] = {&s, &r, &sp.head, &sp.nvec, &sp.tail, &p};
    return launch(reinterpret_cast<const void*>(&reduce_shift_kernel<T, OP, POLICY, XCD, TAG, SEND_ALIGNED, RUN>), grid,
                  args, stream, 64, lds_bytes);
}

// 16-B phase of an operand whose body starts `off` bytes in (see PhaseList).
inline unsigned phase_word(const unsigned char* base, size_t off) {
    return unsigned((reinterpret_cast<uintptr_t>(base) + off) & 15);
}

// The phased k-way and chain launches, instantiated for every (T, OP) in phased_multi.hip and
// phased_chain.hip (their own translation units, so they compile beside local_reduce.hip).
template <typename T, int OP>
int multi_phased_typed(SendList sl, PhaseList ph, int nsend, unsigned char* r, Split sp, hipStream_t stream);
// In-phase k-way and chain launches whose sources straddle recv's 128-B lines: sources loaded
// through the caches (the pairwise StraddleCfg rule), instantiated in the same translation units.
template <typename T, int OP>
int multi_straddle_typed(SendList sl, int nsend, unsigned char* r, Split sp, hipStream_t stream);
template <typename T, int OP>
int chain_straddle_typed(SendList sl, int nsend, const unsigned char* own, unsigned char* d, Split sp,
                         hipStream_t stream);
template <typename T, int OP>
int chain_phased_typed(SendList sl, PhaseList ph, int nsend, const unsigned char* own, unsigned char* d, Split sp,
                       hipStream_t stream);
// k-way (2 <= nsend <= 8) and chain (1 <= nsend <= 8) combines into a destination that is not
// element-aligned, instantiated for every (T, OP) in unaligned_multi.hip.  ph.p[k] = sends[k] & 15
// (and ph.p[nsend] = own & 15 for the chain).
template <typename T, int OP>
int multi_unaligned_typed(SendList sl, PhaseList ph, int nsend, unsigned char* r, size_t count, hipStream_t stream);
template <typename T, int OP>
int chain_unaligned_typed(SendList sl, PhaseList ph, int nsend, const unsigned char* own, unsigned char* d,
                          size_t count, hipStream_t stream);

}  // namespace dccl_amd
