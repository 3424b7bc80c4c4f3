// tools/tune/misaligned_2pass.hpp — TUNING ONLY (not shipped): a two-pass combine for a recv that is not
// element-aligned, kept for the record of round 2's measurements.  On MI355X it ran at
// 74.6-75.6 % of HBM peak (4 vectors per lane, send cached), 1-2 points above the one-access-per-lane kernel
// that ships (reduce_unaligned_kernel: 73.6-74.8 %), which needs no scratch, no second launch and no
// allocation on the device path (tools/ab_combine.py --tune, profiles/r2_misaligned_ab.json).
//
// The reference's host loop accepts such a recv with a warning (/root/reference/src/core/
// internal_common.hpp:504-512); its CUDA kernel cannot take one at all.  Round 1 ran it as a byte kernel
// (65-73 % of HBM peak).  The difficulty is the write side: with recv's elements straddling every 16-B
// vector boundary, an element that straddles the boundary between two waves' tiles is half written by
// each, and whichever wave writes first destroys the original bytes the other still has to read.  Byte
// stores of the shared vector by both waves were measured in round 1 and lose (partial line writes,
// DESIGN.md §9 item 4).  Here every 16-B vector of recv is written whole, by exactly one wave:
//
//   1. boundary pass: for every tile t (64 x U vectors), copy the ORIGINAL vector just before the tile and
//      the one just after it into a small stream-ordered scratch (32 B per tile);
//   2. vector pass: lane l holds recv vectors R_v, v = 64U t + 64u + l (u < U); its right-hand neighbour
//      R_{v+1} comes from lane l+1 (a DPP wave rotate; lane 63 takes lane 0's next vector, the last one the
//      saved vector after the tile); (R_v, R_{v+1}) funnel-shifted by recv's element offset m give
//      A_v = 16 bytes of WHOLE elements; the matching send bytes come the same way at send's own byte phase;
//      C_v = op(A_v, S_v); C_{v-1} comes from lane l-1 (lane 0 of the first vector recomputes it from the
//      saved vector before the tile); the output vector O_v is bytes [16 - m, 32 - m) of (C_{v-1}, C_v).
//      No wave reads a byte another wave writes; the at most two vectors that contain recv's first or last
//      byte are stored bytewise.
//
// Vectors are on recv's 128-B line grid (tile boundaries on lines), so full-vector stores fill whole lines.
// U > 1 amortises the boundary pass (two line reads per tile) and the tile-edge work over more bytes.
#pragma once

#include <hip/hip_runtime.h>

#include "reduce_kernels.hpp"

namespace dccl_amd {
// Tuning-only cross-lane moves (the product needs only from_next_lane_or, reduce_kernels.hpp).
// lane l receives lane (l+1) % 64's vector
__device__ __forceinline__ u32x4 from_next_lane(u32x4 x) { return dpp16<0x134>(x, x); }
// lane l receives lane (l+63) % 64's vector
__device__ __forceinline__ u32x4 from_prev_lane(u32x4 x) { return dpp16<0x13C>(x, x); }
// lane l > 0 receives lane l-1's x, lane 0 keeps its own `first`
__device__ __forceinline__ u32x4 from_prev_lane_or(u32x4 x, u32x4 first) { return dpp16<0x138>(x, first); }
}  // namespace dccl_amd

namespace dccl_amd {
namespace mis {

struct Geometry {
    uintptr_t g;      // recv's 128-B line grid origin (<= recv)
    uintptr_t r, e;   // recv bytes [r, e)
    uintptr_t sg;     // send's 16-B grid origin for A_0
    uintptr_t s, se;  // send bytes [s, se)
    size_t nvec;      // vectors of the grid that start before e
    unsigned m;       // recv element offset within each vector, 0 < m < sizeof(T)
    unsigned ps;      // send byte phase of A_v, 0..15
};

__device__ __forceinline__ bool hits(uintptr_t a, uintptr_t lo, uintptr_t hi) { return a + 16 > lo && a < hi; }

template <bool NT>
__device__ __forceinline__ u32x4 ld_if(uintptr_t a, bool ok) {
    u32x4 v = {0u, 0u, 0u, 0u};
    if (ok) v = ld16<NT>(reinterpret_cast<const u32x4*>(a));
    return v;
}

// bytes [b, b + 16) of the 32 bytes (lo, hi), 0 <= b < 16; b is uniform
__device__ __forceinline__ u32x4 funnel(u32x4 lo, u32x4 hi, unsigned b) {
    switch (b >> 2) {
    case 0: return funnel16<0>(lo, hi, b & 3);
    case 1: return funnel16<1>(lo, hi, b & 3);
    case 2: return funnel16<2>(lo, hi, b & 3);
    default: return funnel16<3>(lo, hi, b & 3);
    }
}

__device__ __forceinline__ u32x4 sel(bool c, u32x4 a, u32x4 b) {
    return u32x4{c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w};
}

// Pass 1: the original vectors around every tile of 64 x U vectors (before it: 2t, after it: 2t + 1).
template <int U>
__global__ __launch_bounds__(256) void save_boundaries_kernel(Geometry g, u32x4* __restrict__ saved, size_t ntiles) {
    constexpr size_t span = size_t(64) * U;
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t t = size_t(blockIdx.x) * blockDim.x + threadIdx.x; t < ntiles; t += stride) {
        const size_t before = span * t - 1, after = span * (t + 1);
        const uintptr_t ab = g.g + 16 * before, aa = g.g + 16 * after;
        saved[2 * t] = ld_if<true>(ab, t > 0 && hits(ab, g.r, g.e));
        saved[2 * t + 1] = ld_if<true>(aa, after < g.nvec && hits(aa, g.r, g.e));
    }
}

// Pass 2.  One-wave blocks; the tile loop is uniform per wave, so every lane reaches the lane moves.
// SEND_NT: non-temporal send loads (else through the caches: send's lines straddle the tiles in general,
// and a line two neighbouring tiles share is then fetched from HBM once).
template <typename T, int OP, int U, bool SEND_NT>
__global__ __launch_bounds__(64) void reduce_misaligned_kernel(Geometry g, const u32x4* __restrict__ saved,
                                                               size_t ntiles) {
    const unsigned lane = threadIdx.x;
    const bool first = lane == 0, last = lane == 63;
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const size_t v0 = size_t(64 * U) * t + lane;
        u32x4 R[U], S[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t v = v0 + 64 * u;
            const uintptr_t ar = g.g + 16 * v, as = g.sg + 16 * v;
            R[u] = ld_if<true>(ar, v < g.nvec && hits(ar, g.r, g.e));
            S[u] = ld_if<SEND_NT>(as, hits(as, g.s, g.se));
        }
        // tile edges: lane 63 the vectors after the tile, lane 0 the ones before it
        const uintptr_t as_after = g.sg + 16 * (v0 + 64 * (U - 1) + 1), as_before = g.sg + 16 * (v0 - 1);
        const u32x4 r_after = last ? saved[2 * t + 1] : u32x4{0u, 0u, 0u, 0u};
        const u32x4 s_after = ld_if<SEND_NT>(as_after, last && hits(as_after, g.s, g.se));
        const u32x4 r_before = first ? saved[2 * t] : u32x4{0u, 0u, 0u, 0u};
        const u32x4 s_before = ld_if<SEND_NT>(as_before, first && hits(as_before, g.s, g.se));
        u32x4 C[U];
        u32x4 rx = from_next_lane(R[0]), sx = from_next_lane(S[0]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            u32x4 rn, sn;
            if (u + 1 < U) {  // lane 63's right-hand neighbour is lane 0's next vector
                const u32x4 rx1 = from_next_lane(R[u + 1]), sx1 = from_next_lane(S[u + 1]);
                rn = sel(last, rx1, rx);
                sn = sel(last, sx1, sx);
                rx = rx1;
                sx = sx1;
            } else {
                rn = sel(last, r_after, rx);
                sn = sel(last, s_after, sx);
            }
            C[u] = combine16<T, OP>(funnel(R[u], rn, g.m), funnel(S[u], sn, g.ps));
        }
        // C_{v-1}: lane 0 of the first vector recomputes it from the saved vector before the tile
        const u32x4 c_before = combine16<T, OP>(funnel(r_before, R[0], g.m), funnel(s_before, S[0], g.ps));
        u32x4 cy = from_prev_lane(C[0]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            u32x4 cp;
            if (u == 0) {
                cp = sel(first, c_before, cy);
            } else {  // lane 0's left-hand neighbour is lane 63's previous vector
                const u32x4 cy1 = from_prev_lane(C[u]);
                cp = sel(first, cy, cy1);
                cy = cy1;
            }
            const size_t v = v0 + 64 * u;
            if (v < g.nvec) {
                const uintptr_t ar = g.g + 16 * v;
                const u32x4 o = funnel(cp, C[u], 16 - g.m);
                if (ar >= g.r && ar + 16 <= g.e) {
                    __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(ar));
                } else if (hits(ar, g.r, g.e)) {  // recv's first or last vector: only recv's own bytes
                    const unsigned w[4] = {o.x, o.y, o.z, o.w};
                    for (unsigned b = 0; b < 16; ++b)
                        if (ar + b >= g.r && ar + b < g.e)
                            reinterpret_cast<unsigned char*>(ar)[b] =
                                static_cast<unsigned char>(w[b >> 2] >> (8 * (b & 3)));
                }
            }
        }
    }
}

// The two passes on `stream`, with a stream-ordered scratch of 32 B per tile.  -1 if it cannot be
// allocated (the caller then takes the byte kernel).
template <typename T, int OP, int U, bool SEND_NT>
int launch_misaligned(const unsigned char* s, unsigned char* r, size_t count, hipStream_t stream) {
    constexpr size_t E = sizeof(T);
    Geometry g{};
    g.r = reinterpret_cast<uintptr_t>(r);
    g.e = g.r + count * E;
    g.g = g.r & ~uintptr_t(127);
    g.m = unsigned((g.r - g.g) % E);
    g.s = reinterpret_cast<uintptr_t>(s);
    g.se = g.s + count * E;
    // A_0 starts at grid byte m: element index (g + m - r) / E, whose send bytes start at s + (g + m - r)
    const uintptr_t sigma = g.s + (g.g + g.m - g.r);  // below s for the first vectors; only ever compared
    g.sg = sigma & ~uintptr_t(15);
    g.ps = unsigned(sigma - g.sg);
    g.nvec = (g.e - g.g + 15) / 16;
    constexpr size_t span = size_t(64) * U;
    size_t ntiles = (g.nvec + span - 1) / span;
    u32x4* saved = nullptr;
    if (hipMallocAsync(reinterpret_cast<void**>(&saved), 2 * ntiles * sizeof(u32x4), stream) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    void* a1[] = {&g, &saved, &ntiles};
    int rc = launch(reinterpret_cast<const void*>(&save_boundaries_kernel<U>), ceil_div(ntiles, size_t(256)), a1,
                    stream, 256);
    const u32x4* csaved = saved;
    void* a2[] = {&g, &csaved, &ntiles};
    if (rc == DCCL_SUCCESS)
        rc = launch(reinterpret_cast<const void*>(&reduce_misaligned_kernel<T, OP, U, SEND_NT>), ntiles, a2, stream, 64);
    if (hipFreeAsync(saved, stream) != hipSuccess) {
        (void)hipGetLastError();
        if (rc == DCCL_SUCCESS) rc = DCCL_UNHANDLED_DEVICE_ERROR;
    }
    return rc;
}

}  // namespace mis
}  // namespace dccl_amd
