// dccl_amd/csrc/misaligned.hip — the combine for a recv that is not element-aligned (e.g. an fp32 chunk at
// an odd byte address), at vector speed.
//
// The reference's host loop accepts such a recv with a warning (/root/reference/src/core/
// internal_common.hpp:504-512); its CUDA kernel cannot take one at all.  Round 1 ran it as a byte kernel
// (69-71 % of HBM peak).  The difficulty is the write side: with recv's elements straddling every 16-B
// vector boundary, an element that straddles the boundary between two waves' tiles is half written by
// each, and whichever wave writes first destroys the original bytes the other still has to read.  Byte
// stores of the shared vector by both waves were measured in round 1 and lose (partial line writes,
// DESIGN.md §9 item 4).  Here every 16-B vector of recv is written whole, by exactly one wave:
//
//   1. boundary pass: for every 1 KiB tile t (64 vectors), copy the ORIGINAL vector just before the tile
//      and the one just after it into a small stream-ordered scratch (32 B per tile, 3 % of the traffic);
//   2. main pass: lane l of tile t loads recv vector R_v (v = 64t + l), takes R_{v+1} from lane l+1 (lane
//      63: the saved vector after the tile), funnel-shifts (R_v, R_{v+1}) by recv's element offset m into
//      A_v = 16 bytes of WHOLE elements, loads the matching send bytes the same way at send's own byte
//      phase, combines C_v = op(A_v, S_v), takes C_{v-1} from lane l-1 (lane 0 recomputes it from the
//      saved vector before the tile) and stores the output vector O_v = bytes [16 - m, 32 - m) of
//      (C_{v-1}, C_v).  No wave reads a byte another wave writes; the at most two vectors that contain
//      recv's first or last byte are stored bytewise.
//
// Vectors are on recv's 128-B line grid (tile boundaries on lines), so every full-vector store fills
// whole lines with its neighbours in the wave.
#include <hip/hip_runtime.h>

#include "dispatch.hpp"
#include "reduce_kernels.hpp"

namespace dccl_amd {
namespace {

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

__device__ __forceinline__ u32x4 ld_if(uintptr_t a, bool ok) {
    u32x4 v = {0u, 0u, 0u, 0u};
    if (ok) v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a));
    return v;
}

// bytes [b, b + 16) of the 32 bytes (lo, hi), 0 <= b < 16
__device__ __forceinline__ u32x4 funnel(u32x4 lo, u32x4 hi, unsigned b) {
    switch (b >> 2) {  // uniform
    case 0: return funnel16<0>(lo, hi, b & 3);
    case 1: return funnel16<1>(lo, hi, b & 3);
    case 2: return funnel16<2>(lo, hi, b & 3);
    default: return funnel16<3>(lo, hi, b & 3);
    }
}

__device__ __forceinline__ u32x4 from_prev_lane(u32x4 x) {
    const int a = int((threadIdx.x + 63) & 63) << 2;
    u32x4 o;
    o.x = unsigned(__builtin_amdgcn_ds_bpermute(a, int(x.x)));
    o.y = unsigned(__builtin_amdgcn_ds_bpermute(a, int(x.y)));
    o.z = unsigned(__builtin_amdgcn_ds_bpermute(a, int(x.z)));
    o.w = unsigned(__builtin_amdgcn_ds_bpermute(a, int(x.w)));
    return o;
}

// Pass 1: the original vectors around every tile (before it: index 2t, after it: 2t + 1).
__global__ __launch_bounds__(256) void save_boundaries_kernel(Geometry g, u32x4* __restrict__ saved, size_t ntiles) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t t = size_t(blockIdx.x) * blockDim.x + threadIdx.x; t < ntiles; t += stride) {
        const size_t before = 64 * t - 1, after = 64 * (t + 1);
        const uintptr_t ab = g.g + 16 * before, aa = g.g + 16 * after;
        saved[2 * t] = ld_if(ab, t > 0 && hits(ab, g.r, g.e));
        saved[2 * t + 1] = ld_if(aa, after < g.nvec && hits(aa, g.r, g.e));
    }
}

// Pass 2.  One-wave blocks; the tile loop is uniform per wave, so every lane reaches the bpermutes.
template <typename T, int OP>
__global__ __launch_bounds__(64) void reduce_misaligned_kernel(Geometry g, const u32x4* __restrict__ saved,
                                                               size_t ntiles) {
    const unsigned lane = threadIdx.x;
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const size_t v = 64 * t + lane;
        const uintptr_t ar = g.g + 16 * v, as = g.sg + 16 * v;
        const u32x4 rv = ld_if(ar, v < g.nvec && hits(ar, g.r, g.e));
        const u32x4 sv = ld_if(as, hits(as, g.s, g.se));
        u32x4 rn = from_next_lane(rv), sn = from_next_lane(sv);
        u32x4 rp = {0u, 0u, 0u, 0u}, sp = {0u, 0u, 0u, 0u};
        if (lane == 63) {
            rn = saved[2 * t + 1];
            sn = ld_if(as + 16, hits(as + 16, g.s, g.se));
        }
        if (lane == 0) {
            rp = saved[2 * t];
            sp = ld_if(as - 16, hits(as - 16, g.s, g.se));
        }
        const u32x4 c = combine16<T, OP>(funnel(rv, rn, g.m), funnel(sv, sn, g.ps));
        u32x4 cp = from_prev_lane(c);
        if (lane == 0) cp = combine16<T, OP>(funnel(rp, rv, g.m), funnel(sp, sv, g.ps));
        if (v < g.nvec) {
            const u32x4 o = funnel(cp, c, 16 - g.m);
            if (ar >= g.r && ar + 16 <= g.e) {
                __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(ar));
            } else if (hits(ar, g.r, g.e)) {  // recv's first or last vector: only recv's own bytes
                const unsigned w[4] = {o.x, o.y, o.z, o.w};
                for (unsigned b = 0; b < 16; ++b)
                    if (ar + b >= g.r && ar + b < g.e)
                        reinterpret_cast<unsigned char*>(ar)[b] = static_cast<unsigned char>(w[b >> 2] >> (8 * (b & 3)));
            }
        }
    }
}

}  // namespace

template <typename T, int OP>
int reduce_misaligned_typed(const unsigned char* s, unsigned char* r, size_t count, hipStream_t stream) {
    constexpr size_t E = sizeof(T);
    Geometry g{};
    g.r = reinterpret_cast<uintptr_t>(r);
    g.e = g.r + count * E;
    g.g = g.r & ~uintptr_t(127);
    g.m = unsigned((g.r - g.g) % E);
    g.s = reinterpret_cast<uintptr_t>(s);
    g.se = g.s + count * E;
    // A_0 starts at grid byte m: element index (g + m - r) / E, whose send bytes start at s + (g + m - r)
    const uintptr_t sigma = g.s + (g.g + g.m - g.r);  // wraps below s for the first tile; only compared
    g.sg = sigma & ~uintptr_t(15);
    g.ps = unsigned(sigma - g.sg);
    g.nvec = (g.e - g.g + 15) / 16;
    const size_t ntiles = (g.nvec + 63) / 64;
    u32x4* saved = nullptr;
    if (hipMallocAsync(reinterpret_cast<void**>(&saved), 2 * ntiles * sizeof(u32x4), stream) != hipSuccess) {
        (void)hipGetLastError();
        return kNoScratch;  // the caller takes the byte kernel instead
    }
    size_t ntiles_arg = ntiles;
    void* a1[] = {&g, &saved, &ntiles_arg};
    int rc = launch(reinterpret_cast<const void*>(&save_boundaries_kernel), ceil_div(ntiles, size_t(256)), a1, stream,
                    256);
    const u32x4* csaved = saved;
    void* a2[] = {&g, &csaved, &ntiles_arg};
    if (rc == DCCL_SUCCESS)
        rc = launch(reinterpret_cast<const void*>(&reduce_misaligned_kernel<T, OP>), ntiles, a2, stream, 64);
    if (hipFreeAsync(saved, stream) != hipSuccess) {
        (void)hipGetLastError();
        if (rc == DCCL_SUCCESS) rc = DCCL_UNHANDLED_DEVICE_ERROR;
    }
    return rc;
}

#define DCCL_MISALIGNED_INST(T)                                                                          \
    template int reduce_misaligned_typed<T, kSum>(const unsigned char*, unsigned char*, size_t, hipStream_t);  \
    template int reduce_misaligned_typed<T, kProd>(const unsigned char*, unsigned char*, size_t, hipStream_t); \
    template int reduce_misaligned_typed<T, kMax>(const unsigned char*, unsigned char*, size_t, hipStream_t);  \
    template int reduce_misaligned_typed<T, kMin>(const unsigned char*, unsigned char*, size_t, hipStream_t);
DCCL_MISALIGNED_INST(int32_t)
DCCL_MISALIGNED_INST(uint32_t)
DCCL_MISALIGNED_INST(int64_t)
DCCL_MISALIGNED_INST(uint64_t)
DCCL_MISALIGNED_INST(f16_bits)
DCCL_MISALIGNED_INST(float)
DCCL_MISALIGNED_INST(double)
DCCL_MISALIGNED_INST(bf16_bits)
#undef DCCL_MISALIGNED_INST

}  // namespace dccl_amd
