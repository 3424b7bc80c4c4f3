// tools/tune/tune_kernels.hip — tuning-only variants of the fp32 Sum combine (not part of the drop-in
// boundary; tools/tune/dccl_reduce_tuning.h).  Built into its own library, tools/lib/libdccl_amd_tune.so
// (dccl_amd/build.py), so the product library carries none of it, and kept in its own translation unit
// so its instantiations cannot perturb the production kernel's code generation.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dccl/dccl_reduce.h"
#include "dccl_reduce_tuning.h"
#include "misaligned_2pass.hpp"
#include "reduce_kernels.hpp"

using namespace dccl_amd;

// ---------------------------------------------------------------------------------
// Tuning entry: fp32 Sum with an explicit kernel variant (include/dccl/dccl_reduce_tuning.h).
// ---------------------------------------------------------------------------------
namespace {
using TuneFn = int (*)(const unsigned char*, unsigned char*, Split, hipStream_t, size_t, size_t);
template <int B, int U, int P, bool X>
int tune_one(const unsigned char* s, unsigned char* r, Split sp, hipStream_t st, size_t cap, size_t lds) {
    return launch_vec<float, kSum, VecCfg<B, U, P, X, 1>>(s, r, sp, st, cap, lds);
}
struct TuneEntry { int block, unroll, policy, xcd; TuneFn fn; };
#define DCCL_TV(B, U, P, X) TuneEntry{B, U, P, X, &tune_one<B, U, P, X>}
const TuneEntry kTune[] = {
    DCCL_TV(64, 1, 7, 0),  DCCL_TV(64, 1, 5, 0),  DCCL_TV(64, 1, 6, 0),  DCCL_TV(64, 1, 3, 0),
    DCCL_TV(64, 1, 1, 0),  DCCL_TV(64, 1, 7, 1),  DCCL_TV(64, 2, 7, 0),  DCCL_TV(64, 4, 7, 0),
    DCCL_TV(128, 1, 7, 0), DCCL_TV(128, 1, 5, 0), DCCL_TV(128, 1, 6, 0), DCCL_TV(128, 1, 7, 1),
    DCCL_TV(256, 1, 7, 0), DCCL_TV(256, 1, 7, 1), DCCL_TV(256, 4, 7, 0), DCCL_TV(1024, 1, 7, 0),
    DCCL_TV(256, 4, 1, 0), DCCL_TV(64, 1, 6, 1),  DCCL_TV(64, 1, 2, 0),  DCCL_TV(64, 1, 2, 1),
};
#undef DCCL_TV
}  // namespace

// recv alignment of the tuning launches: DCCL_TUNE_ALIGN (default 16, the alignment every earlier
// tuning table was measured with)
static size_t tune_align() {
    const char* e = std::getenv("DCCL_TUNE_ALIGN");
    const unsigned long long x = e ? std::strtoull(e, nullptr, 10) : 16ull;
    return (x >= 16 && x <= 4096 && (x & (x - 1)) == 0) ? static_cast<size_t>(x) : size_t(16);
}

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
                             split_for_vectors<float>(ar, count, tune_align()), static_cast<hipStream_t>(stream), grid_cap,
                             lds_bytes);
}

// The shipped aligned shape (one-wave blocks, one 16-B vector per lane, every access non-temporal) in the
// group-interleaved XCD tile order (xcd_group_tile: each XCD walks 8 consecutive tiles of every group of 64
// blocks, one front for the chip).  recv and send must be 16-B aligned with count % 4 == 0 (no head / tail).
namespace {
__global__ __launch_bounds__(64) void tune_vec_group_kernel(const u32x4* __restrict__ vs, u32x4* __restrict__ vr,
                                                            size_t nvec) {
    const size_t ntiles = (nvec + 63) / 64;
    for (size_t t = xcd_group_tile(blockIdx.x, gridDim.x); t < ntiles; t += gridDim.x) {
        const size_t i = t * 64 + threadIdx.x;
        if (i < nvec)
            __builtin_nontemporal_store(combine16<float, kSum>(__builtin_nontemporal_load(vr + i),
                                                               __builtin_nontemporal_load(vs + i)), vr + i);
    }
}
}  // namespace
extern "C" int dccl_tune_group_f32_sum(const void* send, void* recv, size_t count, size_t lds_bytes, void* stream) {
    if (((reinterpret_cast<uintptr_t>(send) | reinterpret_cast<uintptr_t>(recv)) & 15) || (count & 3) ||
        lds_bytes > (64u << 10))
        return DCCL_INVALID_ARGUMENT;
    size_t nvec = count / 4;
    void* args[] = {&send, &recv, &nvec};
    return launch(reinterpret_cast<const void*>(&tune_vec_group_kernel), ceil_div(nvec, size_t(64)), args,
                  static_cast<hipStream_t>(stream), 64, lds_bytes);
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


// ---------------------------------------------------------------------------------
// Tuning only: k-way fp32 Sum (dccl_local_reduce_multi's kernel) with an explicit shape.
// Variant v: 0 = shipped (64 threads, 1 vector, all nt), 1 = 64 threads x 2 vectors,
// 2 = 256 threads x 1 vector, 3 = only send loads nt, 4 = 64 threads x 4 vectors,
// 5/6/7 = staged: recv + s0 first, then the other sends 1/2/3 at a time (aligned operands only); 8 = sources
// through the caches (the shipped line-straddle shape), 9 / 10 = 0 / 8 with each XCD's tiles one contiguous
// range (xcd_remap); 11 / 12 / 13 = 0 / 8 / 3 with the head scalars aligning sends[0] to its 128-B line
// instead of recv (recv straddles its lines, the sources sharing sends[0]'s line phase do not); 14 = sources
// cached only in the tile's two partial lines (tune_multi_edge_cached_kernel); 15 / 16 = 8 / 0 in the
// group-interleaved XCD tile order (tune_multi_group_kernel); `lds_bytes` of
// unused dynamic LDS per block caps the resident blocks per CU (160 KiB / lds_bytes).
// ---------------------------------------------------------------------------------
namespace {
// Staged k-way: first recv and s0 together, then the remaining sends G at a time; each stage
// waits for its loads before the next stage issues (the empty asm consumes the accumulator and
// fences memory), so a wave never has more than max(2, G) 16-B loads per lane in flight and
// the chip sees the two-stream read pattern it streams fastest (tools/ceiling_probe.py).
template <int K, int G>
__global__ __launch_bounds__(64) void tune_multi_staged_kernel(SendList sends, unsigned char* __restrict__ recv,
                                                               size_t nvec) {
    const size_t i = size_t(blockIdx.x) * 64 + threadIdx.x;
    if (i < nvec) {
        u32x4* vr = reinterpret_cast<u32x4*>(recv);
        u32x4 acc = combine16<float, kSum>(__builtin_nontemporal_load(vr + i),
                                           __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sends.p[0]) + i));
#pragma unroll
        for (int k0 = 1; k0 < K; k0 += G) {
            asm volatile("" : "+v"(acc)::"memory");
            u32x4 sv[G];
#pragma unroll
            for (int g = 0; g < G; ++g)
                if (k0 + g < K) sv[g] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sends.p[k0 + g]) + i);
#pragma unroll
            for (int g = 0; g < G; ++g)
                if (k0 + g < K) acc = combine16<float, kSum>(acc, sv[g]);
        }
        __builtin_nontemporal_store(acc, vr + i);
    }
}
template <int K, int G>
int tune_multi_staged(SendList sl, unsigned char* r, Split sp, hipStream_t stream, size_t lds) {
    if (sp.head || sp.tail) return DCCL_INVALID_ARGUMENT;
    void* args[] = {&sl, &r, &sp.nvec};
    return launch(reinterpret_cast<const void*>(&tune_multi_staged_kernel<K, G>), ceil_div(sp.nvec, 64), args, stream,
                  64, lds);
}

template <int K, typename C>
int tune_multi_launch(SendList sl, unsigned char* r, Split sp, hipStream_t stream, size_t lds = 0) {
    size_t grid = ceil_div(sp.nvec, C::TILE);
    if (grid == 0 && (sp.head + sp.tail) > 0) grid = 1;
    void* args[] = {&sl, &r, &sp.head, &sp.nvec, &sp.tail};
    return launch(reinterpret_cast<const void*>(&reduce_multi_vec_kernel<float, kSum, K, C>), grid, args, stream,
                  C::BLOCK, lds);
}
// Line-straddling in-phase sources: only the lanes whose vectors lie in a source's first or last (partial)
// 128-B line of the tile, the lines the neighbouring tiles share, load through the caches; the rest
// non-temporal.  One-wave blocks, one vector per lane, recv and store non-temporal.
template <int K>
__global__ __launch_bounds__(64) void tune_multi_edge_cached_kernel(SendList sends, unsigned char* __restrict__ recv,
                                                                    size_t head, size_t nvec, size_t tail) {
    u32x4* __restrict__ vr = reinterpret_cast<u32x4*>(recv + head * sizeof(float));
    const size_t ntiles = (nvec + 63) / 64;
    const unsigned lane = threadIdx.x & 63;
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const size_t i = t * 64 + lane;
        u32x4 s[K];
        u32x4 r = {0u, 0u, 0u, 0u};
        if (i < nvec) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const u32x4* p = reinterpret_cast<const u32x4*>(sends.p[k] + head * sizeof(float)) + i;
                const unsigned lo = unsigned(reinterpret_cast<uintptr_t>(p - lane) & 127) / 16;  // tile's line phase
                const bool edge = lane < (8 - lo) % 8 || lane >= 64 - lo;
                if (lo != 0 && edge) s[k] = *p;
                else s[k] = __builtin_nontemporal_load(p);
            }
            r = __builtin_nontemporal_load(vr + i);
        }
        if (i < nvec) {
            u32x4 acc = r;
#pragma unroll
            for (int k = 0; k < K; ++k) acc = combine16<float, kSum>(acc, s[k]);
            __builtin_nontemporal_store(acc, vr + i);
        }
    }
    if (blockIdx.x == 0)
        for (size_t j = threadIdx.x; j < head + tail; j += 64) {
            const size_t e = j < head ? j : head + nvec * 4 + (j - head);
            float acc = ld_elem<float, true>(recv, e);
#pragma unroll
            for (int k = 0; k < K; ++k) acc = Combine<float, kSum>::apply(acc, ld_elem<float, true>(sends.p[k], e));
            st_elem<float, true>(recv, e, acc);
        }
}
template <int K>
int tune_multi_edge_cached(SendList sl, unsigned char* r, Split sp, hipStream_t st, size_t lds) {
    size_t grid = ceil_div(sp.nvec, size_t(64));
    if (grid == 0) grid = 1;
    void* args[] = {&sl, &r, &sp.head, &sp.nvec, &sp.tail};
    return launch(reinterpret_cast<const void*>(&tune_multi_edge_cached_kernel<K>), grid, args, st, 64, lds);
}

// The shipped k-way kernel with the group-interleaved XCD tile order (xcd_group_tile: within every group of 64
// blocks, each XCD walks 8 consecutive tiles; the groups sweep the range in order, so the chip keeps one
// front).  Tiles t and t+1 then share an L2 in 7 of 8 cases, so a line-straddling source's line that two
// neighbouring tiles share is fetched from HBM once instead of twice (PMC: each straddling source reads
// 1.125 x in block order).  P: cache policy bits (6: sources cached, 7: all non-temporal).
// Round 3: `run` generalises the order: in every group of 8 * run blocks each XCD walks `run` consecutive tiles
// (run 8 = xcd_group_tile, run 1 = block order); a partial last group keeps the identity.
__device__ __forceinline__ size_t run_tile_rt(size_t b, size_t g, unsigned run) {
    const size_t span = size_t(8) * run, q = b / span, r = b % span;
    return (q + 1) * span > g ? b : q * span + (r % 8) * run + r / 8;
}
template <int K, int P>
__global__ __launch_bounds__(64) void tune_multi_group_kernel(SendList sends, unsigned char* __restrict__ recv,
                                                              size_t head, size_t nvec, size_t tail, unsigned run) {
    u32x4* __restrict__ vr = reinterpret_cast<u32x4*>(recv + head * sizeof(float));
    const size_t ntiles = (nvec + 63) / 64;
    for (size_t t = run_tile_rt(blockIdx.x, gridDim.x, run); t < ntiles; t += gridDim.x) {
        const size_t i = t * 64 + threadIdx.x;
        if (i < nvec) {
            u32x4 s[K];
#pragma unroll
            for (int k = 0; k < K; ++k)
                s[k] = ld16<(P & kNtSend) != 0>(reinterpret_cast<const u32x4*>(sends.p[k] + head * sizeof(float)) + i);
            u32x4 acc = ld16<(P & kNtRecv) != 0>(vr + i);
#pragma unroll
            for (int k = 0; k < K; ++k) acc = combine16<float, kSum>(acc, s[k]);
            __builtin_nontemporal_store(acc, vr + i);
        }
    }
    if (blockIdx.x == 0)
        for (size_t j = threadIdx.x; j < head + tail; j += 64) {
            const size_t e = j < head ? j : head + nvec * 4 + (j - head);
            float acc = ld_elem<float, true>(recv, e);
#pragma unroll
            for (int k = 0; k < K; ++k) acc = Combine<float, kSum>::apply(acc, ld_elem<float, true>(sends.p[k], e));
            st_elem<float, true>(recv, e, acc);
        }
}
template <int K, int P>
int tune_multi_group(SendList sl, unsigned char* r, Split sp, hipStream_t st, size_t lds, unsigned run = 8) {
    size_t grid = ceil_div(sp.nvec, size_t(64));
    if (grid == 0) grid = 1;
    void* args[] = {&sl, &r, &sp.head, &sp.nvec, &sp.tail, &run};
    return launch(reinterpret_cast<const void*>(&tune_multi_group_kernel<K, P>), grid, args, st, 64, lds);
}

template <int K>
int tune_multi_k(int variant, SendList sl, unsigned char* r, Split sp, hipStream_t st, size_t lds) {
    switch (variant) {
    case 0: return tune_multi_launch<K, VecCfg<64, 1, 7, false, 1>>(sl, r, sp, st, lds);
    case 1: return tune_multi_launch<K, VecCfg<64, 2, 7, false, 1>>(sl, r, sp, st, lds);
    case 2: return tune_multi_launch<K, VecCfg<256, 1, 7, false, 1>>(sl, r, sp, st, lds);
    case 3: return tune_multi_launch<K, VecCfg<64, 1, 1, false, 1>>(sl, r, sp, st, lds);
    case 4: return tune_multi_launch<K, VecCfg<64, 4, 7, false, 1>>(sl, r, sp, st, lds);
    case 5: return tune_multi_staged<K, 1>(sl, r, sp, st, lds);
    case 6: return tune_multi_staged<K, 2>(sl, r, sp, st, lds);
    case 7: return tune_multi_staged<K, 3>(sl, r, sp, st, lds);
    case 8: return tune_multi_launch<K, VecCfg<64, 1, 6, false, 1>>(sl, r, sp, st, lds);
    case 9: return tune_multi_launch<K, VecCfg<64, 1, 7, true, 1>>(sl, r, sp, st, lds);
    case 10: return tune_multi_launch<K, VecCfg<64, 1, 6, true, 1>>(sl, r, sp, st, lds);
    case 14: return tune_multi_edge_cached<K>(sl, r, sp, st, lds);
    case 15: return tune_multi_group<K, kNtRecv | kNtStore>(sl, r, sp, st, lds);
    case 16: return tune_multi_group<K, kNtSend | kNtRecv | kNtStore>(sl, r, sp, st, lds);
    // round 3: the line-straddling rule (sources through the caches) with 2 / 4 consecutive vectors per lane,
    // so a wave's tile is 2 / 4 KiB and only one line per tile is shared with the neighbouring wave
    case 19: return tune_multi_group<K, kNtRecv | kNtStore>(sl, r, sp, st, lds, 2);
    case 20: return tune_multi_group<K, kNtRecv | kNtStore>(sl, r, sp, st, lds, 4);
    case 21: return tune_multi_group<K, kNtRecv | kNtStore>(sl, r, sp, st, lds, 16);
    case 17: return tune_multi_launch<K, VecCfg<64, 2, 6, false, 1>>(sl, r, sp, st, lds);
    case 18: return tune_multi_launch<K, VecCfg<64, 4, 6, false, 1>>(sl, r, sp, st, lds);
    default: return DCCL_INVALID_ARGUMENT;
    }
}
}  // namespace

extern "C" int dccl_tune_multi_f32_sum(const void* const* sends, int nsend, void* recv, size_t count, int variant,
                                       size_t lds_bytes, void* stream) {
    if (lds_bytes > (64u << 10)) return DCCL_INVALID_ARGUMENT;
    if (nsend < 1 || nsend > 8 || sends == nullptr || recv == nullptr) return DCCL_INVALID_ARGUMENT;
    SendList sl{};
    const uintptr_t ar = reinterpret_cast<uintptr_t>(recv);
    for (int k = 0; k < nsend; ++k) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(sends[k]);
        if ((a & 3) || ((a ^ ar) & 15)) return DCCL_INVALID_ARGUMENT;
        sl.p[k] = static_cast<const unsigned char*>(sends[k]);
    }
    if (ar & 3) return DCCL_INVALID_ARGUMENT;
    if (count == 0) return DCCL_SUCCESS;
    // recv line-aligned, as the shipped launch; variants 11-13: sends[0] line-aligned instead (recv straddles)
    const bool src_anchor = variant >= 11 && variant <= 13;
    const uintptr_t anchor = src_anchor ? reinterpret_cast<uintptr_t>(sends[0]) : ar;
    const Split sp = split_for_vectors<float>(anchor, count, 128);
    if (src_anchor) variant = variant == 11 ? 0 : variant == 12 ? 8 : 3;
    auto r = static_cast<unsigned char*>(recv);
    const auto st = static_cast<hipStream_t>(stream);
    switch (nsend) {
    case 1: return tune_multi_k<1>(variant, sl, r, sp, st, lds_bytes);
    case 2: return tune_multi_k<2>(variant, sl, r, sp, st, lds_bytes);
    case 3: return tune_multi_k<3>(variant, sl, r, sp, st, lds_bytes);
    case 4: return tune_multi_k<4>(variant, sl, r, sp, st, lds_bytes);
    case 5: return tune_multi_k<5>(variant, sl, r, sp, st, lds_bytes);
    case 6: return tune_multi_k<6>(variant, sl, r, sp, st, lds_bytes);
    case 7: return tune_multi_k<7>(variant, sl, r, sp, st, lds_bytes);
    default: return tune_multi_k<8>(variant, sl, r, sp, st, lds_bytes);
    }
}

// ---------------------------------------------------------------------------------
// Tuning only: the chain kernel (dccl_local_reduce_chain's in-phase kernel) with an explicit occupancy
// cap: `lds_bytes` of unused dynamic LDS per one-wave block (0 = 32 waves per CU).
// ---------------------------------------------------------------------------------
namespace {
template <int K, int POLICY = 7>
int tune_chain_k(SendList sl, const unsigned char* own, unsigned char* d, Split sp, hipStream_t st, size_t lds) {
    using C = VecCfg<64, 1, POLICY, false, 1>;
    size_t grid = ceil_div(sp.nvec, C::TILE);
    if (grid == 0 && (sp.head + sp.tail) > 0) grid = 1;
    void* args[] = {&sl, &own, &d, &sp.head, &sp.nvec, &sp.tail};
    return launch(reinterpret_cast<const void*>(&reduce_chain_vec_kernel<float, kSum, K, C>), grid, args, st, 64, lds);
}
}  // namespace

extern "C" int dccl_tune_chain_f32_sum(const void* const* sends, int nsend, const void* own, void* dst, size_t count,
                                       size_t lds_bytes, void* stream) {
    return dccl_tune_chain_policy_f32_sum(sends, nsend, own, dst, count, lds_bytes, 7, stream);
}

// policy 7: every access non-temporal (the in-phase launch); 6: sources through the caches (the
// line-straddle launch's shape).
extern "C" int dccl_tune_chain_policy_f32_sum(const void* const* sends, int nsend, const void* own, void* dst,
                                              size_t count, size_t lds_bytes, int policy, void* stream) {
    if (policy != 6 && policy != 7) return DCCL_INVALID_ARGUMENT;
    if (lds_bytes > (64u << 10)) return DCCL_INVALID_ARGUMENT;
    if (nsend < 1 || nsend > 8 || sends == nullptr || own == nullptr || dst == nullptr) return DCCL_INVALID_ARGUMENT;
    SendList sl{};
    const uintptr_t ad = reinterpret_cast<uintptr_t>(dst);
    if ((ad & 3) || ((reinterpret_cast<uintptr_t>(own) ^ ad) & 15)) return DCCL_INVALID_ARGUMENT;
    for (int k = 0; k < nsend; ++k) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(sends[k]);
        if ((a & 3) || ((a ^ ad) & 15)) return DCCL_INVALID_ARGUMENT;
        sl.p[k] = static_cast<const unsigned char*>(sends[k]);
    }
    if (count == 0) return DCCL_SUCCESS;
    const Split sp = split_for_vectors<float>(ad, count, 128);
    const auto o = static_cast<const unsigned char*>(own);
    auto d = static_cast<unsigned char*>(dst);
    const auto st = static_cast<hipStream_t>(stream);
    if (policy == 6) {
        switch (nsend) {
        case 1: return tune_chain_k<1, 6>(sl, o, d, sp, st, lds_bytes);
        case 2: return tune_chain_k<2, 6>(sl, o, d, sp, st, lds_bytes);
        case 3: return tune_chain_k<3, 6>(sl, o, d, sp, st, lds_bytes);
        case 4: return tune_chain_k<4, 6>(sl, o, d, sp, st, lds_bytes);
        case 5: return tune_chain_k<5, 6>(sl, o, d, sp, st, lds_bytes);
        case 6: return tune_chain_k<6, 6>(sl, o, d, sp, st, lds_bytes);
        case 7: return tune_chain_k<7, 6>(sl, o, d, sp, st, lds_bytes);
        default: return tune_chain_k<8, 6>(sl, o, d, sp, st, lds_bytes);
        }
    }
    switch (nsend) {
    case 1: return tune_chain_k<1>(sl, o, d, sp, st, lds_bytes);
    case 2: return tune_chain_k<2>(sl, o, d, sp, st, lds_bytes);
    case 3: return tune_chain_k<3>(sl, o, d, sp, st, lds_bytes);
    case 4: return tune_chain_k<4>(sl, o, d, sp, st, lds_bytes);
    case 5: return tune_chain_k<5>(sl, o, d, sp, st, lds_bytes);
    case 6: return tune_chain_k<6>(sl, o, d, sp, st, lds_bytes);
    case 7: return tune_chain_k<7>(sl, o, d, sp, st, lds_bytes);
    default: return tune_chain_k<8>(sl, o, d, sp, st, lds_bytes);
    }
}

// ---------------------------------------------------------------------------------
// Tuning only: HBM ceiling probes, to place the combine's 2-read/1-write mix between the chip's
// own streaming limits.  Shape A = the shipped one (one-wave blocks, one 16-B vector per lane);
// shape B = 256-thread blocks, 4 vectors per lane (a quarter of the workgroups, the same bytes).
// Every access is non-temporal.  Loaded values are consumed by an empty asm statement, so no
// load can be elided and no byte is written.
//   0 read send (A)          1 read send + recv (A)    2 write recv (A)    3 copy send -> recv (A)
//   4 the fp32 Sum combine (A, control)                5 read send + recv (B)
//   6 write recv (B)         7 empty workgroups (A's grid: dispatch cost alone)
//   8 the combine (A) with the recv load issued before the send load
// ---------------------------------------------------------------------------------
namespace {
__device__ __forceinline__ void consume(u32x4 v) { asm volatile("" ::"v"(v)); }

template <int KIND, int BLOCK, int U>
__global__ __launch_bounds__(BLOCK) void tune_ceiling_kernel(const u32x4* __restrict__ s, u32x4* __restrict__ r,
                                                             size_t nvec) {
    const size_t base = size_t(blockIdx.x) * BLOCK * U + threadIdx.x;
    if constexpr (KIND == 7) return;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + size_t(u) * BLOCK;
        if (i >= nvec) continue;
        if constexpr (KIND == 0) {
            consume(__builtin_nontemporal_load(s + i));
        } else if constexpr (KIND == 1 || KIND == 5) {
            consume(__builtin_nontemporal_load(s + i));
            consume(__builtin_nontemporal_load(r + i));
        } else if constexpr (KIND == 2 || KIND == 6) {
            const uint32_t v = uint32_t(i);
            __builtin_nontemporal_store(u32x4{v, v, v, v}, r + i);
        } else if constexpr (KIND == 3) {
            __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), r + i);
        } else if constexpr (KIND == 8) {
            const u32x4 b = __builtin_nontemporal_load(r + i);
            const u32x4 a = __builtin_nontemporal_load(s + i);
            __builtin_nontemporal_store(combine16<float, kSum>(b, a), r + i);
        } else {
            const u32x4 a = __builtin_nontemporal_load(s + i);
            const u32x4 b = __builtin_nontemporal_load(r + i);
            __builtin_nontemporal_store(combine16<float, kSum>(b, a), r + i);
        }
    }
}

struct CeilingEntry { const void* fn; int block, unroll; };
template <int KIND, int BLOCK, int U>
CeilingEntry ceiling_entry() {
    return {reinterpret_cast<const void*>(&tune_ceiling_kernel<KIND, BLOCK, U>), BLOCK, U};
}
}  // namespace

extern "C" int dccl_tune_ceiling(int kind, const void* send, void* recv, size_t count_f32, void* stream) {
    if (count_f32 % 4096 || ((reinterpret_cast<uintptr_t>(send) | reinterpret_cast<uintptr_t>(recv)) & 15))
        return DCCL_INVALID_ARGUMENT;
    const CeilingEntry tab[] = {ceiling_entry<0, 64, 1>(),  ceiling_entry<1, 64, 1>(),  ceiling_entry<2, 64, 1>(),
                                ceiling_entry<3, 64, 1>(),  ceiling_entry<4, 64, 1>(),  ceiling_entry<5, 256, 4>(),
                                ceiling_entry<6, 256, 4>(), ceiling_entry<7, 64, 1>(),  ceiling_entry<8, 64, 1>()};
    if (kind < 0 || kind >= int(sizeof(tab) / sizeof(tab[0]))) return DCCL_INVALID_ARGUMENT;
    size_t nvec = count_f32 / 4;
    void* args[] = {&send, &recv, &nvec};
    const CeilingEntry& e = tab[kind];
    return launch(e.fn, nvec / (size_t(e.block) * e.unroll), args, static_cast<hipStream_t>(stream), e.block);
}

// ---------------------------------------------------------------------------------
// Tuning only: write-only streaming probe over block shapes and store policies, to find the
// chip's write ceiling (the one-wave shape is dispatch-bound when it only writes).
// Variant v: (block, vectors per lane, store policy 0 = plain, 1 = nt, 2 = sc1 via asm).
// ---------------------------------------------------------------------------------
namespace {
template <int BLOCK, int U, int POL>
__global__ __launch_bounds__(BLOCK) void tune_write_kernel(u32x4* __restrict__ r, size_t nvec) {
    const size_t base = size_t(blockIdx.x) * BLOCK * U + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + size_t(u) * BLOCK;
        if (i >= nvec) continue;
        const uint32_t v = uint32_t(i);
        const u32x4 o{v, v, v, v};
        if constexpr (POL == 0) r[i] = o;
        if constexpr (POL == 1) __builtin_nontemporal_store(o, r + i);
        if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(r + i), "v"(o) : "memory");
    }
}
struct WriteEntry { const void* fn; int block, unroll, policy; };
template <int B, int U, int P>
WriteEntry write_entry() { return {reinterpret_cast<const void*>(&tune_write_kernel<B, U, P>), B, U, P}; }
const WriteEntry kWrite[] = {
    write_entry<64, 1, 1>(),  write_entry<64, 2, 1>(),  write_entry<64, 4, 1>(),  write_entry<64, 8, 1>(),
    write_entry<128, 4, 1>(), write_entry<256, 1, 1>(), write_entry<256, 2, 1>(), write_entry<256, 4, 1>(),
    write_entry<256, 8, 1>(), write_entry<512, 4, 1>(), write_entry<256, 4, 0>(), write_entry<64, 4, 0>(),
    write_entry<256, 4, 2>(), write_entry<1024, 4, 1>(),
};
}  // namespace

extern "C" int dccl_tune_write_num_variants(void) { return int(sizeof(kWrite) / sizeof(kWrite[0])); }

extern "C" int dccl_tune_write_probe(int variant, void* recv, size_t count_f32, int* block, int* unroll, int* policy,
                                     void* stream) {
    if (variant < 0 || variant >= dccl_tune_write_num_variants()) return DCCL_INVALID_ARGUMENT;
    if (count_f32 % 32768 || (reinterpret_cast<uintptr_t>(recv) & 15)) return DCCL_INVALID_ARGUMENT;
    const WriteEntry& e = kWrite[variant];
    *block = e.block; *unroll = e.unroll; *policy = e.policy;
    if (stream == reinterpret_cast<void*>(~uintptr_t(0))) return DCCL_SUCCESS;  // info only
    size_t nvec = count_f32 / 4;
    void* args[] = {&recv, &nvec};
    return launch(e.fn, nvec / (size_t(e.block) * e.unroll), args, static_cast<hipStream_t>(stream), e.block);
}

// ---------------------------------------------------------------------------------
// Tuning only: the shifted kernel (operands with different 16-B phases), fp32 Sum, by cache policy
// and block order.
// ---------------------------------------------------------------------------------
namespace {
using ShiftFn = int (*)(const unsigned char*, unsigned char*, size_t, hipStream_t, size_t, size_t);
struct ShiftEntry { int policy, xcd; ShiftFn fn; };
#define DCCL_SV(P, X) ShiftEntry{P, X, &launch_shift<float, kSum, P, X, 1>}
const ShiftEntry kShift[] = {DCCL_SV(7, false), DCCL_SV(15, false), DCCL_SV(6, false), DCCL_SV(7, true),
                             DCCL_SV(6, true),  DCCL_SV(3, false),  DCCL_SV(5, false)};
#undef DCCL_SV
}  // namespace

extern "C" int dccl_tune_shift_num_variants(void) { return int(sizeof(kShift) / sizeof(kShift[0])); }

extern "C" int dccl_tune_shift_f32_sum(const void* send, void* recv, size_t count, int variant, int* policy,
                                       int* xcd, void* stream) {
    if (variant < 0 || variant >= dccl_tune_shift_num_variants()) return DCCL_INVALID_ARGUMENT;
    const uintptr_t as = reinterpret_cast<uintptr_t>(send), ar = reinterpret_cast<uintptr_t>(recv);
    if (((as | ar) & 3) || ((as ^ ar) & 15) == 0) return DCCL_INVALID_ARGUMENT;
    if (policy) *policy = kShift[variant].policy;
    if (xcd) *xcd = kShift[variant].xcd;
    if (count == 0) return DCCL_SUCCESS;
    return kShift[variant].fn(static_cast<const unsigned char*>(send), static_cast<unsigned char*>(recv), count,
                              static_cast<hipStream_t>(stream), tune_align(), 0);
}

// ---------------------------------------------------------------------------------
// Tuning only: persistent one-wave blocks with a software pipeline, fp32 Sum, 16-B aligned operands.
// Each wave walks tiles t, t+G, t+2G, ... (G = grid) and issues the loads of its next tile before it
// combines and stores the current one, so two tiles' loads are in flight per wave without relaunching
// waves; DEPTH tiles ahead (1 or 2).
// ---------------------------------------------------------------------------------
namespace {
template <int DEPTH>
__global__ __launch_bounds__(64) void tune_pipelined_kernel(const u32x4* __restrict__ vs, u32x4* __restrict__ vr,
                                                            size_t nvec) {
    const size_t G = gridDim.x;
    const size_t ntiles = nvec / 64;  // full tiles only (the probe passes a multiple of 64 vectors)
    size_t t = blockIdx.x;
    u32x4 s[DEPTH + 1], r[DEPTH + 1];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
        const size_t td = t + size_t(d) * G;
        if (td < ntiles) {
            s[d] = __builtin_nontemporal_load(vs + td * 64 + threadIdx.x);
            r[d] = __builtin_nontemporal_load(vr + td * 64 + threadIdx.x);
        }
    }
    for (; t < ntiles; t += G) {
        const size_t tn = t + size_t(DEPTH) * G;
        if (tn < ntiles) {
            s[DEPTH] = __builtin_nontemporal_load(vs + tn * 64 + threadIdx.x);
            r[DEPTH] = __builtin_nontemporal_load(vr + tn * 64 + threadIdx.x);
        }
        __builtin_nontemporal_store(combine16<float, kSum>(r[0], s[0]), vr + t * 64 + threadIdx.x);
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            s[d] = s[d + 1];
            r[d] = r[d + 1];
        }
    }
}
}  // namespace

extern "C" int dccl_tune_pipelined_f32_sum(const void* send, void* recv, size_t count, int depth, size_t grid,
                                           void* stream) {
    const uintptr_t as = reinterpret_cast<uintptr_t>(send), ar = reinterpret_cast<uintptr_t>(recv);
    if (((as | ar) & 15) || count % 256 || grid == 0 || (depth != 1 && depth != 2)) return DCCL_INVALID_ARGUMENT;
    size_t nvec = count / 4;
    const void* fn = depth == 1 ? reinterpret_cast<const void*>(&tune_pipelined_kernel<1>)
                                : reinterpret_cast<const void*>(&tune_pipelined_kernel<2>);
    void* args[] = {&send, &recv, &nvec};
    return hipLaunchKernel(fn, dim3(unsigned(grid)), dim3(64), args, 0, static_cast<hipStream_t>(stream)) == hipSuccess
               ? DCCL_SUCCESS
               : DCCL_UNHANDLED_DEVICE_ERROR;
}

// ---------------------------------------------------------------------------------
// Tuning only: the misaligned-recv combine in shape `variant` (two-pass: misaligned_2pass.hpp):
// 0/1 = 1 vector per lane, send cached / non-temporal; 2/3 = 2 vectors; 4/5 = 4 vectors; 6 = the byte kernel;
// 7/8/9 = one 16-B access per lane at the displaced address itself (align-1 vector types: gfx950 takes
// global_load/store_dwordx4 at any byte address, tools/unaligned_probe.hip), 7 all non-temporal (the shipped
// reduce_unaligned_kernel's shape), 8 send cached, 9 nothing non-temporal; 10-17 the walking / XCD-grouped
// forms of 7 (tune_unaligned_walk_kernel).  Adjacent lanes' 16-B windows are disjoint and hold whole elements.
namespace {
// ---------------------------------------------------------------------------------
// Tuning only: the byte-gather kernel the misaligned-recv combine used before round 2 (!ALIGNED: byte
// gathers, 4 independent elements per thread, grid-stride), kept as the comparison point.
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

template <int P>  // policy bits as VecCfg: kNtSend | kNtRecv | kNtStore
__global__ __launch_bounds__(64) void tune_unaligned_kernel(const unsigned char* s, unsigned char* r, size_t nvec,
                                                            size_t count) {
    const size_t i = size_t(blockIdx.x) * 64 + threadIdx.x;
    if (i < nvec) {
        const u32x4_u* ps = reinterpret_cast<const u32x4_u*>(s + 16 * i);
        u32x4_u* pr = reinterpret_cast<u32x4_u*>(r + 16 * i);
        u32x4 a, b;
        if constexpr ((P & kNtRecv) != 0) a = __builtin_nontemporal_load(pr); else a = *pr;
        if constexpr ((P & kNtSend) != 0) b = __builtin_nontemporal_load(ps); else b = *ps;
        const u32x4 o = combine16<float, kSum>(a, b);
        if constexpr ((P & kNtStore) != 0) __builtin_nontemporal_store(o, pr); else *pr = o;
    }
    if (blockIdx.x == 0)
        for (size_t j = 4 * nvec + threadIdx.x; j < count; j += 64)
            st_elem<float, false>(r, j, Combine<float, kSum>::apply(ld_elem<float, false>(r, j), ld_elem<float, false>(s, j)));
}
template <int P>
int tune_unaligned(const unsigned char* s, unsigned char* r, size_t count, hipStream_t st) {
    size_t nvec = count / 4;
    void* args[] = {const_cast<unsigned char**>(&s), &r, &nvec, &count};
    return launch(reinterpret_cast<const void*>(&tune_unaligned_kernel<P>), ceil_div(nvec, size_t(64)) + 1, args, st, 64);
}
// Each wave walks CH consecutive 1 KiB chunks (so the lines two chunks share are touched by one wave, in
// one XCD's L2), four chunks' loads in flight at a time.  XCD: CH = 1 and consecutive tiles on one XCD
// (blocks are dealt round-robin over the 8 XCDs).
template <int P, int CH, bool XCD>
__global__ __launch_bounds__(64) void tune_unaligned_walk_kernel(const unsigned char* s, unsigned char* r, size_t nvec,
                                                                 size_t count) {
    size_t t0 = size_t(blockIdx.x) * CH;
    if constexpr (XCD) {
        const size_t per = gridDim.x / 8;  // grid is a multiple of 8
        t0 = size_t(blockIdx.x % 8) * per + blockIdx.x / 8;
    }
    constexpr int G = CH < 4 ? CH : 4;
    for (int c0 = 0; c0 < CH; c0 += G) {
        u32x4 a[G], b[G];
#pragma unroll
        for (int c = 0; c < G; ++c) {
            const size_t i = (t0 + c0 + c) * 64 + threadIdx.x;
            if (i < nvec) {
                const u32x4_u* ps = reinterpret_cast<const u32x4_u*>(s + 16 * i);
                const u32x4_u* pr = reinterpret_cast<const u32x4_u*>(r + 16 * i);
                if constexpr ((P & kNtRecv) != 0) a[c] = __builtin_nontemporal_load(pr); else a[c] = *pr;
                if constexpr ((P & kNtSend) != 0) b[c] = __builtin_nontemporal_load(ps); else b[c] = *ps;
            }
        }
#pragma unroll
        for (int c = 0; c < G; ++c) {
            const size_t i = (t0 + c0 + c) * 64 + threadIdx.x;
            if (i < nvec) {
                u32x4_u* pr = reinterpret_cast<u32x4_u*>(r + 16 * i);
                const u32x4 o = combine16<float, kSum>(a[c], b[c]);
                if constexpr ((P & kNtStore) != 0) __builtin_nontemporal_store(o, pr); else *pr = o;
            }
        }
    }
    if (blockIdx.x == 0)
        for (size_t j = 4 * nvec + threadIdx.x; j < count; j += 64)
            st_elem<float, false>(r, j, Combine<float, kSum>::apply(ld_elem<float, false>(r, j), ld_elem<float, false>(s, j)));
}
template <int P, int CH, bool XCD>
int tune_unaligned_walk(const unsigned char* s, unsigned char* r, size_t count, hipStream_t st) {
    size_t nvec = count / 4;
    size_t grid = ceil_div(ceil_div(nvec, size_t(64)), size_t(CH));
    if (XCD) grid = ceil_div(grid, size_t(8)) * 8;
    if (grid == 0) grid = 1;
    if (grid > kMaxGrid) return DCCL_INVALID_ARGUMENT;  // no grid stride here
    void* args[] = {const_cast<unsigned char**>(&s), &r, &nvec, &count};
    return launch(reinterpret_cast<const void*>(&tune_unaligned_walk_kernel<P, CH, XCD>), grid, args, st, 64);
}
// The shipped misaligned-recv kernel (reduce_unaligned_kernel) with the stores of the lanes that write into the
// tile's first or last E-byte sector (shared with the neighbouring tile, so each wave writes only part of it)
// going through the L2 as write-back stores instead of non-temporal ones: the two partial writes of a shared
// sector can then merge in the L2 (consecutive tiles run on one XCD) before the line goes to HBM, instead of
// reaching the memory as two masked partial writes (PMC: +4.75 % write bytes, ~1 extra write request per tile).
template <int E>
__global__ __launch_bounds__(64) void tune_unaligned_edge_kernel(const unsigned char* __restrict__ send, unsigned p,
                                                                 unsigned char* __restrict__ recv, size_t nvec,
                                                                 size_t count) {
    const size_t g = gridDim.x;
    for (size_t t = size_t(blockIdx.x % 8) * (g / 8) + blockIdx.x / 8; t * 64 < nvec; t += g) {
        const size_t i = t * 64 + threadIdx.x;
        const u32x4 b = ld_phased(send, p, i, nvec);
        if (i < nvec) {
            const uintptr_t a0 = reinterpret_cast<uintptr_t>(recv) + 16 * t * 64;
            const uintptr_t lo = (a0 & ~uintptr_t(E - 1)) + E, hi = (a0 + 1024) & ~uintptr_t(E - 1);
            const uintptr_t a = a0 + 16 * threadIdx.x;
            u32x4_u* pr = reinterpret_cast<u32x4_u*>(recv + 16 * i);
            const u32x4 o = combine16<float, kSum>(__builtin_nontemporal_load(pr), b);
            if (a < lo || a + 16 > hi) *pr = o;
            else __builtin_nontemporal_store(o, pr);
        }
    }
    if (blockIdx.x == 0)
        for (size_t j = nvec * 4 + threadIdx.x; j < count; j += 64)
            st_elem<float, false>(recv, j, Combine<float, kSum>::apply(ld_elem<float, false>(recv, j),
                                                                       ld_elem<float, false>(send, j)));
}
template <int E>
int tune_unaligned_edge(const unsigned char* s, unsigned char* r, size_t count, hipStream_t st, int waves) {
    const size_t nvec = count / 4;
    size_t grid = ceil_div(ceil_div(nvec, size_t(64)), size_t(8)) * 8;
    if (grid == 0) grid = 8;  // the tail elements still need block 0
    unsigned p = unsigned(reinterpret_cast<uintptr_t>(s) & 15);
    size_t cnt = count, nv = nvec;
    void* args[] = {const_cast<unsigned char**>(&s), &p, &r, &nv, &cnt};
    return launch(reinterpret_cast<const void*>(&tune_unaligned_edge_kernel<E>), grid, args, st, 64, caps::lds_for_waves(waves));
}
// Aligned-vector form of the misaligned-recv combine (walks of W tiles per wave).  recv's body is walked in
// ALIGNED 16-B vectors V_v (from the first 16-B boundary inside recv, Vstart); every element boundary then
// falls inside a vector, c bytes before its end (c = (Vstart - recv) mod e, 1 <= c < e).  Lane l builds the
// element-aligned 16 bytes X that start at the element straddling its vector's first byte (the last c bytes
// of V_{v-1}, from the lane to its left, and the first 16 - c of V_v), the matching send bytes SX (aligned
// send vectors, funnel shift by sigma), combines them, takes the next element-aligned result from the lane to
// its right, and stores the 16 output bytes of V_v whole.  A wave walks W consecutive tiles, carrying lane
// 63's original V into the next tile's lane 0, so a recv line is never written by two waves except at walk
// edges: the element straddling a walk edge belongs to the walk on its left, which writes its e - c bytes past
// the edge bytewise; the walk on the right writes its first vector without them.  Head elements (up to the
// one straddling Vstart) and tail elements (after the one straddling Vend) are block 0's, element by element.
__device__ __forceinline__ u32x4 funnel_at(u32x4 lo, u32x4 hi, unsigned k) {  // bytes [k, k + 16), k < 16
    const unsigned b = k & 3;
    switch (k >> 2) {  // uniform
    case 0: return funnel16<0>(lo, hi, b);
    case 1: return funnel16<1>(lo, hi, b);
    case 2: return funnel16<2>(lo, hi, b);
    default: return funnel16<3>(lo, hi, b);
    }
}
__device__ __forceinline__ unsigned char byte_of(u32x4 x, unsigned k) {
    const unsigned d[4] = {x.x, x.y, x.z, x.w};
    return static_cast<unsigned char>(d[k >> 2] >> (8 * (k & 3)));
}
template <typename T, int OP, int W>
__global__ __launch_bounds__(64) void tune_unaligned_walk_vec_kernel(
    const unsigned char* __restrict__ send, unsigned char* __restrict__ recv, unsigned char* vbase,
    const unsigned char* ubase, size_t nv, unsigned c, unsigned sigma, size_t js, size_t je, size_t count) {
    constexpr unsigned e = sizeof(T);
    const unsigned lane = threadIdx.x;
    u32x4* vr = reinterpret_cast<u32x4*>(vbase);
    const u32x4* vu = reinterpret_cast<const u32x4*>(ubase);
    const u32x4 zero = {0u, 0u, 0u, 0u};
    const size_t nwalks = (nv + 64 * W - 1) / (64 * W);
    for (size_t w = blockIdx.x; w < nwalks; w += gridDim.x) {
        const size_t w0 = w * 64 * W, w1 = w0 + 64 * W < nv ? w0 + 64 * W : nv;
        u32x4 carry = zero;
        for (int j = 0; j < W; ++j) {
            const size_t t0 = w0 + size_t(64) * j;
            if (t0 >= w1) break;  // uniform
            const size_t v = t0 + lane;
            const bool in = v < w1;
            const bool last = in && (lane == 63 || v + 1 == w1);
            u32x4 vc = zero, u0 = zero, vn = zero, x1 = zero, x2 = zero;
            if (in) {
                vc = __builtin_nontemporal_load(vr + v);
                u0 = __builtin_nontemporal_load(vu + v);
            }
            if (last) {
                vn = vr[v + 1];
                x1 = vu[v + 1];
                if (sigma + e > 16) x2 = vu[v + 2];
            }
            u32x4 u1 = from_next_lane_or(u0, x1);
            if (last) u1 = x1;
            const u32x4 vp = from_prev_lane_or(vc, carry);
            const u32x4 ox = combine16<T, OP>(funnel_at(vp, vc, 16 - c), funnel_at(u0, u1, sigma));
            u32x4 oys = zero;
            if (last) oys = combine16<T, OP>(funnel_at(vc, vn, 16 - c), funnel_at(x1, x2, sigma));
            u32x4 oy = from_next_lane_or(ox, oys);
            if (last) oy = oys;
            const u32x4 out = funnel_at(ox, oy, c);
            carry.x = unsigned(__builtin_amdgcn_readlane(int(vc.x), 63));
            carry.y = unsigned(__builtin_amdgcn_readlane(int(vc.y), 63));
            carry.z = unsigned(__builtin_amdgcn_readlane(int(vc.z), 63));
            carry.w = unsigned(__builtin_amdgcn_readlane(int(vc.w), 63));
            if (in) {
                unsigned char* pv = reinterpret_cast<unsigned char*>(vr + v);
                if (j == 0 && lane == 0) {  // walk edge: the straddling element's first e - c bytes are the left walk's
                    for (unsigned k = e - c; k < 16; ++k) pv[k] = byte_of(out, k);
                } else {
                    __builtin_nontemporal_store(out, vr + v);
                }
                if (v + 1 == w1)  // walk edge: this walk owns the element straddling it, e - c bytes past the edge
                    for (unsigned k = c; k < e; ++k) pv[16 + k - c] = byte_of(oy, k);
            }
        }
    }
    if (blockIdx.x == 0) {
        for (size_t i = lane; i <= js; i += 64)
            st_elem<T, false>(recv, i, Combine<T, OP>::apply(ld_elem<T, false>(recv, i), ld_elem<T, false>(send, i)));
        for (size_t i = je + 1 + lane; i < count; i += 64)
            st_elem<T, false>(recv, i, Combine<T, OP>::apply(ld_elem<T, false>(recv, i), ld_elem<T, false>(send, i)));
    }
}
template <typename T, int OP, int W>
int tune_unaligned_walk_vec(const unsigned char* s, unsigned char* r, size_t count, hipStream_t st, int waves) {
    constexpr size_t e = sizeof(T);
    const uintptr_t ar = reinterpret_cast<uintptr_t>(r), as = reinterpret_cast<uintptr_t>(s);
    const uintptr_t vs = (ar + 15) & ~uintptr_t(15), endb = ar + e * count, ve = endb & ~uintptr_t(15);
    size_t nv = 0, js = count - 1, je = count - 1;
    unsigned c = 0, sigma = 0;
    const unsigned char* ub = s;
    if (ve > vs) {
        nv = (ve - vs) / 16;
        js = (vs - ar) / e;
        je = (ve - ar) / e;
        c = unsigned(vs - (ar + e * js));
        const uintptr_t sw = as + e * js;
        sigma = unsigned(sw & 15);
        ub = reinterpret_cast<const unsigned char*>(sw - sigma);
    }
    unsigned char* vb = r + (vs - ar);
    size_t grid = ceil_div(nv, size_t(64) * W);
    if (grid == 0) grid = 1;
    void* args[] = {const_cast<unsigned char**>(&s), &r, &vb, &ub, &nv, &c, &sigma, &js, &je, &count};
    return launch(reinterpret_cast<const void*>(&tune_unaligned_walk_vec_kernel<T, OP, W>), grid, args, st, 64,
                  caps::lds_for_waves(waves));
}
}  // namespace
// recv must not be element-aligned (fp32: an address that is not a multiple of 4).
// ---------------------------------------------------------------------------------
extern "C" int dccl_tune_misaligned_f32_sum(const void* send, void* recv, size_t count, int variant, void* stream) {
    const auto s = static_cast<const unsigned char*>(send);
    const auto r = static_cast<unsigned char*>(recv);
    const auto st = static_cast<hipStream_t>(stream);
    if ((reinterpret_cast<uintptr_t>(recv) & 3) == 0 || count == 0) return DCCL_INVALID_ARGUMENT;
    switch (variant) {
    case 0: return mis::launch_misaligned<float, kSum, 1, false>(s, r, count, st);
    case 1: return mis::launch_misaligned<float, kSum, 1, true>(s, r, count, st);
    case 2: return mis::launch_misaligned<float, kSum, 2, false>(s, r, count, st);
    case 3: return mis::launch_misaligned<float, kSum, 2, true>(s, r, count, st);
    case 4: return mis::launch_misaligned<float, kSum, 4, false>(s, r, count, st);
    case 5: return mis::launch_misaligned<float, kSum, 4, true>(s, r, count, st);
    case 6: {
        void* args[] = {const_cast<unsigned char**>(&s), const_cast<unsigned char**>(&r), &count};
        return launch(reinterpret_cast<const void*>(&reduce_scalar_kernel<float, kSum, false>),
                      ceil_div(count, size_t(kBlock) * 4), args, st);
    }
    case 7: return tune_unaligned<kNtSend | kNtRecv | kNtStore>(s, r, count, st);
    case 8: return tune_unaligned<kNtRecv | kNtStore>(s, r, count, st);
    case 9: return tune_unaligned<0>(s, r, count, st);
    case 10: return tune_unaligned_walk<kNtSend | kNtRecv | kNtStore, 4, false>(s, r, count, st);
    case 11: return tune_unaligned_walk<kNtStore, 4, false>(s, r, count, st);
    case 12: return tune_unaligned_walk<kNtSend | kNtRecv | kNtStore, 16, false>(s, r, count, st);
    case 13: return tune_unaligned_walk<kNtStore, 16, false>(s, r, count, st);
    case 14: return tune_unaligned_walk<0, 16, false>(s, r, count, st);
    case 15: return tune_unaligned_walk<kNtStore, 1, true>(s, r, count, st);
    case 16: return tune_unaligned_walk<kNtSend | kNtRecv | kNtStore, 1, true>(s, r, count, st);
    case 17: return tune_unaligned_walk<kNtStore, 64, false>(s, r, count, st);
    case 20: case 21: case 22: case 23: case 24: case 25: {  // the shipped kernel, capped at 26/22/20/16/13/24 waves
        const int waves[] = {26, 22, 20, 16, 13, 24};
        const size_t lds = ((160u << 10) / waves[variant - 20] + 255) / 256 * 256;
        const size_t nvec = count / 4;
        size_t grid = ceil_div(ceil_div(nvec, size_t(64)), size_t(8)) * 8;
        if (grid == 0) grid = 8;  // the tail elements still need block 0
        unsigned p = unsigned(reinterpret_cast<uintptr_t>(send) & 15);
        size_t cnt = count;
        size_t nv = nvec;
        int order = kOrderXcd;  // the round-2 order these caps were measured in
        void* args[] = {const_cast<unsigned char**>(&s), &p, const_cast<unsigned char**>(&r), &nv, &cnt, &order};
        return launch(reinterpret_cast<const void*>(&reduce_unaligned_kernel<float, kSum>), grid, args, st, 64, lds);
    }
    // the shipped kernel with write-back stores in the tile's shared edge sectors (tune_unaligned_edge_kernel):
    // 30/31 64-B sectors at 24/32 waves, 32/33 128-B lines at 24/32 waves
    case 30: return tune_unaligned_edge<64>(s, r, count, st, 24);
    case 31: return tune_unaligned_edge<64>(s, r, count, st, 32);
    case 32: return tune_unaligned_edge<128>(s, r, count, st, 24);
    case 33: return tune_unaligned_edge<128>(s, r, count, st, 32);
    // aligned-vector walks (tune_unaligned_walk_vec_kernel): 40-43 W = 4 / 8 / 16 / 32 uncapped, 44-47 the same
    // at 24 waves, 48-49 W = 8 / 16 at 16 waves, 50 W = 1 (one tile per wave, walk edges at every tile)
    case 40: return tune_unaligned_walk_vec<float, kSum, 4>(s, r, count, st, 32);
    case 41: return tune_unaligned_walk_vec<float, kSum, 8>(s, r, count, st, 32);
    case 42: return tune_unaligned_walk_vec<float, kSum, 16>(s, r, count, st, 32);
    case 43: return tune_unaligned_walk_vec<float, kSum, 32>(s, r, count, st, 32);
    case 44: return tune_unaligned_walk_vec<float, kSum, 4>(s, r, count, st, 24);
    case 45: return tune_unaligned_walk_vec<float, kSum, 8>(s, r, count, st, 24);
    case 46: return tune_unaligned_walk_vec<float, kSum, 16>(s, r, count, st, 24);
    case 47: return tune_unaligned_walk_vec<float, kSum, 32>(s, r, count, st, 24);
    case 48: return tune_unaligned_walk_vec<float, kSum, 8>(s, r, count, st, 16);
    case 49: return tune_unaligned_walk_vec<float, kSum, 16>(s, r, count, st, 16);
    case 50: return tune_unaligned_walk_vec<float, kSum, 1>(s, r, count, st, 32);
    default: return DCCL_INVALID_ARGUMENT;
    }
}


// ---------------------------------------------------------------------------------
// Tuning only: the phased k-way combine (sources element-aligned at other 16-B phases than recv) in
// shape `variant`, recv 128-B aligned past the head scalars:
//   0 the shipped shape (reduce_multi_phased_kernel: aligned loads, DPP neighbour, funnel shift);
//   1 the same with consecutive tiles on one XCD (lane 63's extra vector and the next tile's first line
//     then meet in one L2);
//   2 every off-phase source read with one 16-B load at its own (unaligned) address, no lane exchange;
//   3 = 2 with consecutive tiles on one XCD;
//   8 every operand's loads issued before the first shift (ld_phased_issue / ld_phased_finish); 9 = 8 with
//     consecutive tiles on one XCD; 16 / 24 / 25 = 0 / 8 / 9 under the k-way kernel's wave caps (multi_lds);
//   32: 0 with each source's first line and lane 63's neighbour vector loaded through the caches; 64: 0 with
//     every source load cached;
//   lds_bytes != 0: that much unused dynamic LDS per one-wave block instead (an explicit wave cap).
//   4 the shipped shape in the group-interleaved XCD order (xcd_group_tile: 8 consecutive tiles per XCD
//     within each group of 64 blocks, the groups in order).
// ---------------------------------------------------------------------------------
namespace {
// ld_phased with cached loads: C = 1 only lanes 0-7 (the tile's first line, the one the previous tile's
// lane 63 also reads) and lane 63's neighbour vector; C = 2 every load.
template <int C>
__device__ __forceinline__ u32x4 ld_phased_cached(const unsigned char* body, unsigned p, size_t v, size_t nvec) {
    u32x4 lo = {0u, 0u, 0u, 0u};
    const u32x4* va = reinterpret_cast<const u32x4*>(body - p);
    const unsigned lane = threadIdx.x & 63;
    if (p != 0 ? v <= nvec : v < nvec) {
        if (C == 2 || lane < 8) lo = va[v];
        else lo = __builtin_nontemporal_load(va + v);
    }
    if (p == 0) return lo;
    u32x4 ex = {0u, 0u, 0u, 0u};
    if (lane == 63 && v < nvec) ex = va[v + 1];
    const u32x4 hi = from_next_lane_or(lo, ex);
    const unsigned b = p & 3;
    switch (p >> 2) {
    case 0: return funnel16<0>(lo, hi, b);
    case 1: return funnel16<1>(lo, hi, b);
    case 2: return funnel16<2>(lo, hi, b);
    default: return funnel16<3>(lo, hi, b);
    }
}

template <int K, int MODE>
__global__ __launch_bounds__(64) void tune_phased_kernel(SendList sends, PhaseList ph, unsigned char* __restrict__ recv,
                                                         size_t head, size_t nvec, size_t tail) {
    constexpr bool XCD = (MODE & 1) != 0, UNALIGNED = (MODE & 2) != 0, GROUP = (MODE & 4) != 0,
                   FIRST = (MODE & 8) != 0;  // MODE & 16: the k-way kernel's wave caps (launch side)
    constexpr int CACHE = (MODE >> 5) & 3;  // 1: each source's first line (lanes 0-7) cached; 2: every source load cached
    const size_t off = head * sizeof(float);
    u32x4* vr = reinterpret_cast<u32x4*>(recv + off);
    const size_t ntiles = (nvec + 63) / 64;
    const size_t t0 = XCD ? xcd_remap(blockIdx.x, gridDim.x) : GROUP ? xcd_group_tile(blockIdx.x, gridDim.x) : blockIdx.x;
    for (size_t t = t0; t < ntiles; t += gridDim.x) {
        const size_t v = t * 64 + threadIdx.x;
        if constexpr (FIRST) {  // recv, then every source's loads, then the shifts and combines
            u32x4 acc = {0u, 0u, 0u, 0u};
            if (v < nvec) acc = ld16<true>(vr + v);
            PhasedLoad x[K];
#pragma unroll
            for (int k = 0; k < K; ++k) x[k] = ld_phased_issue(sends.p[k] + off, ph.p[k], v, nvec);
#pragma unroll
            for (int k = 0; k < K; ++k) acc = combine16<float, kSum>(acc, ld_phased_finish(x[k], ph.p[k]));
            if (v < nvec) __builtin_nontemporal_store(acc, vr + v);
            continue;
        }
        u32x4 s[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if constexpr (UNALIGNED) {
                s[k] = u32x4{0u, 0u, 0u, 0u};
                if (v < nvec) s[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u*>(sends.p[k] + off) + v);
            } else {
                if constexpr (CACHE == 0) s[k] = ld_phased(sends.p[k] + off, ph.p[k], v, nvec);
                else s[k] = ld_phased_cached<CACHE>(sends.p[k] + off, ph.p[k], v, nvec);
            }
        }
        if (v < nvec) {
            u32x4 acc = ld16<true>(vr + v);
#pragma unroll
            for (int k = 0; k < K; ++k) acc = combine16<float, kSum>(acc, s[k]);
            __builtin_nontemporal_store(acc, vr + v);
        }
    }
    if (blockIdx.x == 0) {
        for (size_t j = threadIdx.x; j < head + tail; j += blockDim.x) {
            const size_t i = j < head ? j : head + nvec * 4 + (j - head);
            float acc = ld_elem<float, true>(recv, i);
#pragma unroll
            for (int k = 0; k < K; ++k) acc = Combine<float, kSum>::apply(acc, ld_elem<float, true>(sends.p[k], i));
            st_elem<float, true>(recv, i, acc);
        }
    }
}
template <int K, int MODE>
int tune_phased_k(SendList sl, PhaseList ph, unsigned char* r, Split sp, hipStream_t st, size_t lds) {
    size_t grid = ceil_div(sp.nvec, size_t(64));
    if (grid == 0) grid = 1;
    if (grid > kMaxGrid) return DCCL_INVALID_ARGUMENT;  // one tile per block (the XCD map is over the grid)
    void* args[] = {&sl, &ph, &r, &sp.head, &sp.nvec, &sp.tail};
    return launch(reinterpret_cast<const void*>(&tune_phased_kernel<K, MODE>), grid, args, st, 64,
                  lds != 0 ? lds : (MODE & 16) ? caps::lds(caps::kMulti, K, size_t(1) << 30) : 0);
}
template <int MODE>
int tune_phased_mode(SendList sl, PhaseList ph, int k, unsigned char* r, Split sp, hipStream_t st, size_t lds) {
    switch (k) {
    case 1: return tune_phased_k<1, MODE>(sl, ph, r, sp, st, lds);
    case 2: return tune_phased_k<2, MODE>(sl, ph, r, sp, st, lds);
    case 3: return tune_phased_k<3, MODE>(sl, ph, r, sp, st, lds);
    case 4: return tune_phased_k<4, MODE>(sl, ph, r, sp, st, lds);
    case 5: return tune_phased_k<5, MODE>(sl, ph, r, sp, st, lds);
    case 6: return tune_phased_k<6, MODE>(sl, ph, r, sp, st, lds);
    case 7: return tune_phased_k<7, MODE>(sl, ph, r, sp, st, lds);
    case 8: return tune_phased_k<8, MODE>(sl, ph, r, sp, st, lds);
    default: return DCCL_INVALID_ARGUMENT;
    }
}
}  // namespace

extern "C" int dccl_tune_phased_f32_sum(const void* const* sends, int nsend, void* recv, size_t count, int variant,
                                        size_t lds_bytes, void* stream) {
    if (lds_bytes > (64u << 10)) return DCCL_INVALID_ARGUMENT;
    if (sends == nullptr || recv == nullptr) return DCCL_INVALID_ARGUMENT;
    const uintptr_t ar = reinterpret_cast<uintptr_t>(recv);
    if (ar & 3) return DCCL_INVALID_ARGUMENT;
    SendList sl{};
    for (int k = 0; k < nsend && k < 8; ++k) {
        if (reinterpret_cast<uintptr_t>(sends[k]) & 3) return DCCL_INVALID_ARGUMENT;
        sl.p[k] = static_cast<const unsigned char*>(sends[k]);
    }
    const Split sp = split_for_vectors<float>(ar, count, 128);
    PhaseList ph{};
    for (int k = 0; k < nsend && k < 8; ++k) ph.p[k] = phase_word(sl.p[k], sp.head * sizeof(float));
    auto r = static_cast<unsigned char*>(recv);
    const auto st = static_cast<hipStream_t>(stream);
    switch (variant) {
    case 0: return tune_phased_mode<0>(sl, ph, nsend, r, sp, st, lds_bytes);
    case 1: return tune_phased_mode<1>(sl, ph, nsend, r, sp, st, lds_bytes);
    case 2: return tune_phased_mode<2>(sl, ph, nsend, r, sp, st, lds_bytes);
    case 3: return tune_phased_mode<3>(sl, ph, nsend, r, sp, st, lds_bytes);
    case 4: return tune_phased_mode<4>(sl, ph, nsend, r, sp, st, lds_bytes);
    case 8: return tune_phased_mode<8>(sl, ph, nsend, r, sp, st, lds_bytes);
    case 9: return tune_phased_mode<9>(sl, ph, nsend, r, sp, st, lds_bytes);
    case 24: return tune_phased_mode<24>(sl, ph, nsend, r, sp, st, lds_bytes);
    case 25: return tune_phased_mode<25>(sl, ph, nsend, r, sp, st, lds_bytes);
    case 16: return tune_phased_mode<16>(sl, ph, nsend, r, sp, st, lds_bytes);
    case 32: return tune_phased_mode<32>(sl, ph, nsend, r, sp, st, lds_bytes);
    case 64: return tune_phased_mode<64>(sl, ph, nsend, r, sp, st, lds_bytes);
    default: return DCCL_INVALID_ARGUMENT;
    }
}

// Tuning only: the shipped phased chain kernel with the XCD tile order forced on (xcd 1) or off (0).
namespace {
template <int K, bool X>
int tune_chain_phased_k(SendList sl, PhaseList ph, const unsigned char* own, unsigned char* d, Split sp, hipStream_t st) {
    size_t grid = ceil_div(sp.nvec, size_t(64));
    if (grid == 0) grid = 1;
    void* args[] = {&sl, &ph, &own, &d, &sp.head, &sp.nvec, &sp.tail};
    return launch(reinterpret_cast<const void*>(&reduce_chain_phased_kernel<float, kSum, K, X>), grid, args, st, 64);
}
template <bool X>
int tune_chain_phased_x(SendList sl, PhaseList ph, int k, const unsigned char* own, unsigned char* d, Split sp,
                        hipStream_t st) {
    switch (k) {
    case 1: return tune_chain_phased_k<1, X>(sl, ph, own, d, sp, st);
    case 2: return tune_chain_phased_k<2, X>(sl, ph, own, d, sp, st);
    case 3: return tune_chain_phased_k<3, X>(sl, ph, own, d, sp, st);
    case 4: return tune_chain_phased_k<4, X>(sl, ph, own, d, sp, st);
    case 5: return tune_chain_phased_k<5, X>(sl, ph, own, d, sp, st);
    case 7: return tune_chain_phased_k<7, X>(sl, ph, own, d, sp, st);
    default: return DCCL_INVALID_ARGUMENT;
    }
}
}  // namespace

extern "C" int dccl_tune_chain_phased_f32_sum(const void* const* sends, int nsend, const void* own, void* dst,
                                              size_t count, int xcd, void* stream) {
    if (sends == nullptr || own == nullptr || dst == nullptr || nsend < 1 || nsend > 8) return DCCL_INVALID_ARGUMENT;
    const uintptr_t ad = reinterpret_cast<uintptr_t>(dst);
    if ((ad & 3) || (reinterpret_cast<uintptr_t>(own) & 3)) return DCCL_INVALID_ARGUMENT;
    SendList sl{};
    for (int k = 0; k < nsend; ++k) {
        if (reinterpret_cast<uintptr_t>(sends[k]) & 3) return DCCL_INVALID_ARGUMENT;
        sl.p[k] = static_cast<const unsigned char*>(sends[k]);
    }
    const Split sp = split_for_vectors<float>(ad, count, 128);
    PhaseList ph{};
    for (int k = 0; k < nsend; ++k) ph.p[k] = phase_word(sl.p[k], sp.head * sizeof(float));
    const auto o = static_cast<const unsigned char*>(own);
    ph.p[nsend] = phase_word(o, sp.head * sizeof(float));
    auto d = static_cast<unsigned char*>(dst);
    const auto st = static_cast<hipStream_t>(stream);
    return xcd ? tune_chain_phased_x<true>(sl, ph, nsend, o, d, sp, st) : tune_chain_phased_x<false>(sl, ph, nsend, o, d, sp, st);
}

// ---------------------------------------------------------------------------------
// Tuning only: the phased k-way combine with U consecutive tiles per wave (dccl_tune_phased_walk_f32_sum):
// lane 63's neighbour vector for tile c is lane 0's vector of tile c + 1 (a wave rotate), so only the
// last tile's loads one vector past the wave's range; the line two waves share is fetched twice once per
// U KiB instead of once per KiB.  ORDER 0: blocks in order; 1: range split per XCD (xcd_remap);
// 2: group-interleaved (xcd_group_tile).
// ---------------------------------------------------------------------------------
namespace {
template <int Q>
__device__ __forceinline__ u32x4 shift_q(u32x4 lo, u32x4 hi, unsigned b) { return funnel16<Q>(lo, hi, b); }

template <int K, int U, int ORDER>
__global__ __launch_bounds__(64) void tune_phased_walk_kernel(SendList sends, PhaseList ph,
                                                              unsigned char* __restrict__ recv, size_t head,
                                                              size_t nvec, size_t tail) {
    const size_t off = head * sizeof(float);
    u32x4* vr = reinterpret_cast<u32x4*>(recv + off);
    const size_t nw = (nvec + 64 * U - 1) / (64 * U);
    const size_t b0 = ORDER == 1 ? xcd_remap(blockIdx.x, gridDim.x)
                                 : ORDER == 2 ? xcd_group_tile(blockIdx.x, gridDim.x) : blockIdx.x;
    const bool last_lane = (threadIdx.x & 63) == 63;
    for (size_t w = b0; w < nw; w += gridDim.x) {
        u32x4 acc[U];
#pragma unroll
        for (int c = 0; c < U; ++c) {
            const size_t v = (w * U + c) * 64 + threadIdx.x;
            acc[c] = u32x4{0u, 0u, 0u, 0u};
            if (v < nvec) acc[c] = ld16<true>(vr + v);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const unsigned p = ph.p[k];
            const unsigned char* body = sends.p[k] + off;
            u32x4 sv[U];
            if (p == 0) {
#pragma unroll
                for (int c = 0; c < U; ++c) {
                    const size_t v = (w * U + c) * 64 + threadIdx.x;
                    sv[c] = u32x4{0u, 0u, 0u, 0u};
                    if (v < nvec) sv[c] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(body) + v);
                }
            } else {
                const u32x4* va = reinterpret_cast<const u32x4*>(body - p);
                u32x4 lo[U];
#pragma unroll
                for (int c = 0; c < U; ++c) {
                    const size_t v = (w * U + c) * 64 + threadIdx.x;
                    lo[c] = u32x4{0u, 0u, 0u, 0u};
                    if (v <= nvec) lo[c] = __builtin_nontemporal_load(va + v);
                }
                u32x4 ex = {0u, 0u, 0u, 0u};
                const size_t vl = (w * U + U - 1) * 64 + threadIdx.x;
                if (last_lane && vl < nvec) ex = va[vl + 1];
                const unsigned bb = p & 3;
#pragma unroll
                for (int c = 0; c < U; ++c) {
                    const u32x4 nx = c + 1 < U ? from_next_lane(lo[c + 1 < U ? c + 1 : c]) : ex;
                    const u32x4 hi = from_next_lane_or(lo[c], nx);
                    switch (p >> 2) {
                    case 0: sv[c] = shift_q<0>(lo[c], hi, bb); break;
                    case 1: sv[c] = shift_q<1>(lo[c], hi, bb); break;
                    case 2: sv[c] = shift_q<2>(lo[c], hi, bb); break;
                    default: sv[c] = shift_q<3>(lo[c], hi, bb); break;
                    }
                }
            }
#pragma unroll
            for (int c = 0; c < U; ++c) acc[c] = combine16<float, kSum>(acc[c], sv[c]);
        }
#pragma unroll
        for (int c = 0; c < U; ++c) {
            const size_t v = (w * U + c) * 64 + threadIdx.x;
            if (v < nvec) __builtin_nontemporal_store(acc[c], vr + v);
        }
    }
    if (blockIdx.x == 0) {
        for (size_t j = threadIdx.x; j < head + tail; j += blockDim.x) {
            const size_t i = j < head ? j : head + nvec * 4 + (j - head);
            float a = ld_elem<float, true>(recv, i);
#pragma unroll
            for (int k = 0; k < K; ++k) a = Combine<float, kSum>::apply(a, ld_elem<float, true>(sends.p[k], i));
            st_elem<float, true>(recv, i, a);
        }
    }
}
template <int K, int U, int ORDER>
int tune_phased_walk_k(SendList sl, PhaseList ph, unsigned char* r, Split sp, hipStream_t st) {
    size_t grid = ceil_div(sp.nvec, size_t(64 * U));
    if (grid == 0) grid = 1;
    if (grid > kMaxGrid) return DCCL_INVALID_ARGUMENT;
    void* args[] = {&sl, &ph, &r, &sp.head, &sp.nvec, &sp.tail};
    return launch(reinterpret_cast<const void*>(&tune_phased_walk_kernel<K, U, ORDER>), grid, args, st, 64);
}
template <int U, int ORDER>
int tune_phased_walk_u(SendList sl, PhaseList ph, int k, unsigned char* r, Split sp, hipStream_t st) {
    switch (k) {
    case 1: return tune_phased_walk_k<1, U, ORDER>(sl, ph, r, sp, st);
    case 2: return tune_phased_walk_k<2, U, ORDER>(sl, ph, r, sp, st);
    case 4: return tune_phased_walk_k<4, U, ORDER>(sl, ph, r, sp, st);
    case 7: return tune_phased_walk_k<7, U, ORDER>(sl, ph, r, sp, st);
    default: return DCCL_INVALID_ARGUMENT;
    }
}
}  // namespace

// variant: U = 1 << (variant % 3) (1, 2, 4) consecutive tiles per wave, ORDER = variant / 3 (0-2).
extern "C" int dccl_tune_phased_walk_f32_sum(const void* const* sends, int nsend, void* recv, size_t count, int variant,
                                             void* stream) {
    if (sends == nullptr || recv == nullptr || nsend < 1 || nsend > 8 || variant < 0 || variant > 8)
        return DCCL_INVALID_ARGUMENT;
    const uintptr_t ar = reinterpret_cast<uintptr_t>(recv);
    if (ar & 3) return DCCL_INVALID_ARGUMENT;
    SendList sl{};
    for (int k = 0; k < nsend; ++k) {
        if (reinterpret_cast<uintptr_t>(sends[k]) & 3) return DCCL_INVALID_ARGUMENT;
        sl.p[k] = static_cast<const unsigned char*>(sends[k]);
    }
    const Split sp = split_for_vectors<float>(ar, count, 128);
    PhaseList ph{};
    for (int k = 0; k < nsend; ++k) ph.p[k] = phase_word(sl.p[k], sp.head * sizeof(float));
    auto r = static_cast<unsigned char*>(recv);
    const auto st = static_cast<hipStream_t>(stream);
    switch (variant) {
    case 0: return tune_phased_walk_u<1, 0>(sl, ph, nsend, r, sp, st);
    case 1: return tune_phased_walk_u<2, 0>(sl, ph, nsend, r, sp, st);
    case 2: return tune_phased_walk_u<4, 0>(sl, ph, nsend, r, sp, st);
    case 3: return tune_phased_walk_u<1, 1>(sl, ph, nsend, r, sp, st);
    case 4: return tune_phased_walk_u<2, 1>(sl, ph, nsend, r, sp, st);
    case 5: return tune_phased_walk_u<4, 1>(sl, ph, nsend, r, sp, st);
    case 6: return tune_phased_walk_u<1, 2>(sl, ph, nsend, r, sp, st);
    case 7: return tune_phased_walk_u<2, 2>(sl, ph, nsend, r, sp, st);
    default: return tune_phased_walk_u<4, 2>(sl, ph, nsend, r, sp, st);
    }
}

// ---------------------------------------------------------------------------------
// Tuning only: the shipped phased k-way (own == nullptr, recv = dst) and chain kernels with the loads-first
// form (first), the XCD tile order (xcd) and an explicit wave cap (lds_bytes) chosen at run time.
// ---------------------------------------------------------------------------------
namespace {
template <int K, bool X, bool F>
int tune_phased_prod_k(SendList sl, PhaseList ph, const unsigned char* own, unsigned char* d, Split sp, hipStream_t st,
                       size_t lds) {
    size_t grid = ceil_div(sp.nvec, size_t(64));
    if (grid == 0) grid = 1;
    if (own == nullptr) {
        void* args[] = {&sl, &ph, &d, &sp.head, &sp.nvec, &sp.tail};
        return launch(reinterpret_cast<const void*>(&reduce_multi_phased_kernel<float, kSum, K, X, F>), grid, args, st,
                      64, lds);
    }
    void* args[] = {&sl, &ph, &own, &d, &sp.head, &sp.nvec, &sp.tail};
    return launch(reinterpret_cast<const void*>(&reduce_chain_phased_kernel<float, kSum, K, X, F>), grid, args, st, 64,
                  lds);
}
template <bool X, bool F>
int tune_phased_prod_xf(SendList sl, PhaseList ph, int k, const unsigned char* own, unsigned char* d, Split sp,
                        hipStream_t st, size_t lds) {
    switch (k) {
    case 2: return tune_phased_prod_k<2, X, F>(sl, ph, own, d, sp, st, lds);
    case 3: return tune_phased_prod_k<3, X, F>(sl, ph, own, d, sp, st, lds);
    case 4: return tune_phased_prod_k<4, X, F>(sl, ph, own, d, sp, st, lds);
    case 5: return tune_phased_prod_k<5, X, F>(sl, ph, own, d, sp, st, lds);
    case 6: return tune_phased_prod_k<6, X, F>(sl, ph, own, d, sp, st, lds);
    case 7: return tune_phased_prod_k<7, X, F>(sl, ph, own, d, sp, st, lds);
    case 8: return tune_phased_prod_k<8, X, F>(sl, ph, own, d, sp, st, lds);
    default: return DCCL_INVALID_ARGUMENT;
    }
}
}  // namespace

extern "C" int dccl_tune_phased_prod_f32_sum(const void* const* sends, int nsend, const void* own, void* dst,
                                             size_t count, int first, int xcd, size_t lds_bytes, void* stream) {
    if (sends == nullptr || dst == nullptr || nsend < 2 || nsend > 8 || lds_bytes > (64u << 10))
        return DCCL_INVALID_ARGUMENT;
    const uintptr_t ad = reinterpret_cast<uintptr_t>(dst);
    if (ad & 3) return DCCL_INVALID_ARGUMENT;
    SendList sl{};
    for (int k = 0; k < nsend; ++k) sl.p[k] = static_cast<const unsigned char*>(sends[k]);
    const Split sp = split_for_vectors<float>(ad, count, 128);
    PhaseList ph{};
    for (int k = 0; k < nsend; ++k) ph.p[k] = phase_word(sl.p[k], sp.head * sizeof(float));
    const auto o = static_cast<const unsigned char*>(own);
    if (o != nullptr) ph.p[nsend] = phase_word(o, sp.head * sizeof(float));
    auto d = static_cast<unsigned char*>(dst);
    const auto st = static_cast<hipStream_t>(stream);
    if (xcd) return first ? tune_phased_prod_xf<true, true>(sl, ph, nsend, o, d, sp, st, lds_bytes)
                          : tune_phased_prod_xf<true, false>(sl, ph, nsend, o, d, sp, st, lds_bytes);
    return first ? tune_phased_prod_xf<false, true>(sl, ph, nsend, o, d, sp, st, lds_bytes)
                 : tune_phased_prod_xf<false, false>(sl, ph, nsend, o, d, sp, st, lds_bytes);
}

// Tuning only: the shipped shifted-kernel dispatch for an element-aligned recv and a send at another phase
// (or byte offset), under a wave cap of `lds_bytes` of unused dynamic LDS per block (0 = uncapped).
extern "C" int dccl_tune_shift_caps_f32_sum(const void* send, void* recv, size_t count, size_t lds_bytes, void* stream) {
    const auto s = static_cast<const unsigned char*>(send);
    const auto r = static_cast<unsigned char*>(recv);
    const auto st = static_cast<hipStream_t>(stream);
    const uintptr_t as = reinterpret_cast<uintptr_t>(send), ar = reinterpret_cast<uintptr_t>(recv);
    if ((ar & 3) || ((as ^ ar) & 15) == 0 || lds_bytes > (64u << 10)) return DCCL_INVALID_ARGUMENT;
    const Split sp = split_for_vectors<float>(ar, count, 128);
    const uintptr_t a = (as + sp.head * sizeof(float)) & ~uintptr_t(15);
    constexpr int kP = kNtSend | kNtRecv | kNtStore, kPs = kNtRecv | kNtStore;
    if (as & 3)
        return (a & 127) ? launch_shift<float, kSum, kPs, false, 0, false>(s, r, count, st, 128, lds_bytes)
                         : launch_shift<float, kSum, kP, false, 0, false>(s, r, count, st, 128, lds_bytes);
    return (a & 127) ? launch_shift<float, kSum, kPs, false>(s, r, count, st, 128, lds_bytes)
                     : launch_shift<float, kSum, kP, false>(s, r, count, st, 128, lds_bytes);
}

// ---------------------------------------------------------------------------------
// Tuning only: the shipped unaligned k-way (own == nullptr) and chain kernels called directly on any
// operands (the product calls them only for a destination that is not element-aligned), under an
// explicit wave cap: used to try "sources aligned, destination at another phase" tilings.
// ---------------------------------------------------------------------------------
namespace {
template <int K, bool FIRST>
int tune_unaligned_kway_k(SendList sl, PhaseList ph, const unsigned char* own, unsigned char* d, size_t count,
                          hipStream_t st, size_t lds, int order) {
    size_t nvec = count / 4;
    const size_t grid = ceil_div(ceil_div(nvec, size_t(64)), size_t(8)) * 8;
    if (own == nullptr) {
        void* args[] = {&sl, &ph, &d, &nvec, &count, &order};
        return launch(reinterpret_cast<const void*>(&reduce_multi_unaligned_kernel<float, kSum, K, FIRST>), grid,
                      args, st, 64, lds);
    }
    void* args[] = {&sl, &ph, &own, &d, &nvec, &count, &order};
    return launch(reinterpret_cast<const void*>(&reduce_chain_unaligned_kernel<float, kSum, K, FIRST>), grid,
                  args, st, 64, lds);
}
template <int K>
int tune_unaligned_kway_form(SendList sl, PhaseList ph, const unsigned char* own, unsigned char* d, size_t count,
                             hipStream_t st, size_t lds, int form) {
    if ((form >> 1) > 4) return DCCL_INVALID_ARGUMENT;
    return (form & 1) ? tune_unaligned_kway_k<K, true>(sl, ph, own, d, count, st, lds, form >> 1)
                      : tune_unaligned_kway_k<K, false>(sl, ph, own, d, count, st, lds, form >> 1);
}
}  // namespace

// form: bit 0 = the loads-first form (reduce_kernels.hpp FIRST), form >> 1 = the tile ORDER (0 XCD-contiguous,
// 1 block order, 2 group-interleaved, 3 runs of 4, 4 runs of 2).
extern "C" int dccl_tune_unaligned_kway_f32_sum(const void* const* sends, int nsend, const void* own, void* dst,
                                                size_t count, size_t lds_bytes, int form, void* stream) {
    if (sends == nullptr || dst == nullptr || nsend < 1 || nsend > 8 || lds_bytes > (64u << 10))
        return DCCL_INVALID_ARGUMENT;
    SendList sl{};
    PhaseList ph{};
    for (int k = 0; k < nsend; ++k) {
        sl.p[k] = static_cast<const unsigned char*>(sends[k]);
        ph.p[k] = phase_word(sl.p[k], 0);
    }
    const auto o = static_cast<const unsigned char*>(own);
    if (o != nullptr) ph.p[nsend] = phase_word(o, 0);
    if (o == nullptr && nsend < 2) return DCCL_INVALID_ARGUMENT;
    auto d = static_cast<unsigned char*>(dst);
    const auto st = static_cast<hipStream_t>(stream);
    return with_k<1, 8>(nsend, [&](auto K) {
        return tune_unaligned_kway_form<K.value>(sl, ph, o, d, count, st, lds_bytes, form);
    });
}

// The pairwise misaligned-recv kernel (reduce_unaligned_kernel) under an explicit cap and tile order (0 XCD-
// contiguous, 1 block order, 2 group-interleaved); recv not element-aligned.
extern "C" int dccl_tune_unaligned_pair_f32_sum(const void* send, void* recv, size_t count, size_t lds_bytes,
                                                int order, void* stream) {
    if ((reinterpret_cast<uintptr_t>(recv) & 3) == 0 || lds_bytes > (64u << 10)) return DCCL_INVALID_ARGUMENT;
    const unsigned char* s = static_cast<const unsigned char*>(send);
    unsigned char* r = static_cast<unsigned char*>(recv);
    size_t nvec = count / 4;
    unsigned p = unsigned(reinterpret_cast<uintptr_t>(send) & 15);
    size_t grid = ceil_div(ceil_div(nvec, size_t(64)), size_t(8)) * 8;
    if (grid == 0) grid = 8;
    if (order < 0 || order > 4) return DCCL_INVALID_ARGUMENT;
    void* args[] = {&s, &p, &r, &nvec, &count, &order};
    return launch(reinterpret_cast<const void*>(&reduce_unaligned_kernel<float, kSum>), grid, args,
                  static_cast<hipStream_t>(stream), 64, lds_bytes);
}

// ---------------------------------------------------------------------------------
// Tuning only (round 3): a persistent work-queue form of the aligned fp32 Sum combine.  `waves` one-wave
// blocks per CU take GRAB consecutive 1 KiB tiles at a time from a device counter (one returning vector
// atomic per grab by lane 0, prefetched one grab ahead), so the chip's access front stays as tight as the
// one-shot grid's without dispatching 1 M workgroups.  PIPE: the next tile's loads are issued before the
// current tile's store.  Every wave leaves the loop once the counter passes the last tile; the last wave
// to finish resets ctr[0..1] for the next launch (stream order makes the reset visible to it).
// ctr: two zero-initialised 64-bit words in device memory, one pair per concurrently running launch.
// ---------------------------------------------------------------------------------
namespace {
__device__ __forceinline__ unsigned long long bcast_lane0(unsigned long long x) {
    const unsigned lo = __builtin_amdgcn_readfirstlane(unsigned(x)), hi = __builtin_amdgcn_readfirstlane(unsigned(x >> 32));
    return (static_cast<unsigned long long>(hi) << 32) | lo;
}

template <int GRAB, bool PIPE>
__global__ __launch_bounds__(64) void tune_wq_kernel(const u32x4* __restrict__ vs, u32x4* __restrict__ vr,
                                                     unsigned long long ntiles, unsigned long long* ctr) {
    unsigned long long t = 0, nt = 0;
    if (threadIdx.x == 0) t = atomicAdd(ctr, static_cast<unsigned long long>(GRAB));
    t = bcast_lane0(t);
    while (t < ntiles) {
        if (threadIdx.x == 0) nt = atomicAdd(ctr, static_cast<unsigned long long>(GRAB));  // the next grab, early
        const unsigned long long end = t + GRAB < ntiles ? t + GRAB : ntiles;
        if constexpr (PIPE) {
            size_t i = size_t(t) * 64 + threadIdx.x;
            u32x4 s = __builtin_nontemporal_load(vs + i), r = __builtin_nontemporal_load(vr + i);
            for (unsigned long long u = t + 1; u <= end; ++u) {
                const size_t j = size_t(u) * 64 + threadIdx.x;
                u32x4 s2{0u, 0u, 0u, 0u}, r2{0u, 0u, 0u, 0u};
                if (u < end) {
                    s2 = __builtin_nontemporal_load(vs + j);
                    r2 = __builtin_nontemporal_load(vr + j);
                }
                __builtin_nontemporal_store(combine16<float, kSum>(r, s), vr + i);
                s = s2;
                r = r2;
                i = j;
            }
        } else {
            for (unsigned long long u = t; u < end; ++u) {
                const size_t i = size_t(u) * 64 + threadIdx.x;
                const u32x4 s = __builtin_nontemporal_load(vs + i), r = __builtin_nontemporal_load(vr + i);
                __builtin_nontemporal_store(combine16<float, kSum>(r, s), vr + i);
            }
        }
        t = bcast_lane0(nt);
    }
    if (threadIdx.x == 0) {
        const unsigned long long d = atomicAdd(ctr + 1, 1ull);
        if (d == gridDim.x - 1) {  // every other wave has left the loop: reset for the next launch
            ctr[0] = 0;
            ctr[1] = 0;
        }
    }
}

template <int GRAB, bool PIPE>
int tune_wq_launch(const u32x4* vs, u32x4* vr, unsigned long long ntiles, unsigned long long* ctr, size_t grid,
                   hipStream_t st) {
    void* args[] = {&vs, &vr, &ntiles, &ctr};
    return launch(reinterpret_cast<const void*>(&tune_wq_kernel<GRAB, PIPE>), grid, args, st, 64);
}
}  // namespace

// variant: grab (tiles per atomic) 1, 2, 4, 8, 16 or 32, plus 100 for the pipelined form; waves per CU 1-32.
// count a multiple of 256 floats, 16-B aligned operands.
extern "C" int dccl_tune_wq_f32_sum(const void* send, void* recv, size_t count, int variant, int waves_per_cu,
                                    void* counter, void* stream) {
    if (count % 256 || waves_per_cu < 1 || waves_per_cu > 32 || counter == nullptr) return DCCL_INVALID_ARGUMENT;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || cus <= 0) cus = 256;
    const auto vs = static_cast<const u32x4*>(send);
    const auto vr = static_cast<u32x4*>(recv);
    const unsigned long long ntiles = count / 256;
    const size_t grid = size_t(cus) * size_t(waves_per_cu);
    auto* ctr = static_cast<unsigned long long*>(counter);
    const auto st = static_cast<hipStream_t>(stream);
    switch (variant) {
    case 1: return tune_wq_launch<1, false>(vs, vr, ntiles, ctr, grid, st);
    case 2: return tune_wq_launch<2, false>(vs, vr, ntiles, ctr, grid, st);
    case 4: return tune_wq_launch<4, false>(vs, vr, ntiles, ctr, grid, st);
    case 8: return tune_wq_launch<8, false>(vs, vr, ntiles, ctr, grid, st);
    case 16: return tune_wq_launch<16, false>(vs, vr, ntiles, ctr, grid, st);
    case 32: return tune_wq_launch<32, false>(vs, vr, ntiles, ctr, grid, st);
    case 104: return tune_wq_launch<4, true>(vs, vr, ntiles, ctr, grid, st);
    case 108: return tune_wq_launch<8, true>(vs, vr, ntiles, ctr, grid, st);
    case 116: return tune_wq_launch<16, true>(vs, vr, ntiles, ctr, grid, st);
    default: return DCCL_INVALID_ARGUMENT;
    }
}

// ---------------------------------------------------------------------------------
// Tuning only (round 3): the phased k-way kernel (sources at other 16-B phases, element-aligned recv) in the
// tile-run orders of run_tile (each XCD walks `run` consecutive tiles in every group of 8 * run blocks;
// run 1 = block order, the shipped order from k = 5), per-operand (FIRST false) or loads-first form.
// ---------------------------------------------------------------------------------
namespace {
template <int K, bool FIRST>
__global__ __launch_bounds__(64) void tune_phased_run_kernel(SendList sends, PhaseList ph, unsigned char* __restrict__ recv,
                                                             size_t head, size_t nvec, size_t tail, unsigned run) {
    const size_t off = head * sizeof(float);
    u32x4* vr = reinterpret_cast<u32x4*>(recv + off);
    const size_t ntiles = (nvec + 63) / 64;
    for (size_t t = run_tile_rt(blockIdx.x, gridDim.x, run); t < ntiles; t += gridDim.x) {
        const size_t v = t * 64 + threadIdx.x;
        u32x4 acc = {0u, 0u, 0u, 0u};
        if constexpr (FIRST) {
            if (v < nvec) acc = ld16<true>(vr + v);
            PhasedLoad x[K];
#pragma unroll
            for (int k = 0; k < K; ++k) x[k] = ld_phased_issue(sends.p[k] + off, ph.p[k], v, nvec);
#pragma unroll
            for (int k = 0; k < K; ++k) acc = combine16<float, kSum>(acc, ld_phased_finish(x[k], ph.p[k]));
        } else {
            u32x4 s[K];
#pragma unroll
            for (int k = 0; k < K; ++k) s[k] = ld_phased(sends.p[k] + off, ph.p[k], v, nvec);
            if (v < nvec) acc = ld16<true>(vr + v);
#pragma unroll
            for (int k = 0; k < K; ++k) acc = combine16<float, kSum>(acc, s[k]);
        }
        if (v < nvec) __builtin_nontemporal_store(acc, vr + v);
    }
    if (blockIdx.x == 0)
        for (size_t j = threadIdx.x; j < head + tail; j += 64) {
            const size_t i = j < head ? j : head + nvec * 4 + (j - head);
            float acc = ld_elem<float, true>(recv, i);
#pragma unroll
            for (int k = 0; k < K; ++k) acc = Combine<float, kSum>::apply(acc, ld_elem<float, false>(sends.p[k], i));
            st_elem<float, true>(recv, i, acc);
        }
}
template <int K>
int tune_phased_run_k(SendList sl, PhaseList ph, unsigned char* r, Split sp, hipStream_t st, size_t lds, bool first,
                      unsigned run) {
    size_t grid = ceil_div(sp.nvec, size_t(64));
    if (grid == 0) grid = 1;
    void* args[] = {&sl, &ph, &r, &sp.head, &sp.nvec, &sp.tail, &run};
    const void* fn = first ? reinterpret_cast<const void*>(&tune_phased_run_kernel<K, true>)
                           : reinterpret_cast<const void*>(&tune_phased_run_kernel<K, false>);
    return launch(fn, grid, args, st, 64, lds);
}
}  // namespace

extern "C" int dccl_tune_phased_run_f32_sum(const void* const* sends, int nsend, void* recv, size_t count,
                                            size_t lds_bytes, int first, unsigned run, void* stream) {
    if (sends == nullptr || recv == nullptr || nsend < 2 || nsend > 8 || lds_bytes > (64u << 10) || run < 1 ||
        (reinterpret_cast<uintptr_t>(recv) & 3))
        return DCCL_INVALID_ARGUMENT;
    const Split sp = split_for_vectors<float>(reinterpret_cast<uintptr_t>(recv), count, 128);
    SendList sl{};
    PhaseList ph{};
    for (int k = 0; k < nsend; ++k) {
        sl.p[k] = static_cast<const unsigned char*>(sends[k]);
        ph.p[k] = phase_word(sl.p[k], sp.head * sizeof(float));
    }
    auto r = static_cast<unsigned char*>(recv);
    const auto st = static_cast<hipStream_t>(stream);
    return with_k<2, 8>(nsend, [&](auto K) {
        return tune_phased_run_k<K.value>(sl, ph, r, sp, st, lds_bytes, first != 0, run);
    });
}

// ---------------------------------------------------------------------------------
// Tuning only (round 3): the product's straddling and phased k-way / chain kernels in the tile-run orders
// (reduce_kernels.hpp run_tile<RUN>, VecCfg::RUN): kind 0 k-way straddling (sources cached), 1 chain
// straddling, 2 k-way phased, 3 chain phased (own = nullptr for the k-way kinds); run 1, 2 or 4; first: the
// phased kernels' loads-first form.  recv / dst element-aligned, sources in its 16-B phase (kinds 0, 1) or
// at any phase (2, 3).
// ---------------------------------------------------------------------------------
namespace {
template <int K, int RUN>
int tune_runs_k(int kind, bool first, SendList sl, PhaseList ph, const unsigned char* own, unsigned char* d, Split sp,
                hipStream_t st, size_t lds) {
    size_t grid = ceil_div(sp.nvec, size_t(64));
    if (grid == 0) grid = 1;
    using C = VecCfg<64, 1, kNtRecv | kNtStore, false, 1, RUN>;
    void* a_multi[] = {&sl, &d, &sp.head, &sp.nvec, &sp.tail};
    void* a_chain[] = {&sl, &own, &d, &sp.head, &sp.nvec, &sp.tail};
    void* a_pm[] = {&sl, &ph, &d, &sp.head, &sp.nvec, &sp.tail};
    void* a_pc[] = {&sl, &ph, &own, &d, &sp.head, &sp.nvec, &sp.tail};
    switch (kind) {
    case 0: return launch(reinterpret_cast<const void*>(&reduce_multi_vec_kernel<float, kSum, K, C>), grid, a_multi, st, 64, lds);
    case 1: return launch(reinterpret_cast<const void*>(&reduce_chain_vec_kernel<float, kSum, K, C>), grid, a_chain, st, 64, lds);
    case 2:
        return launch(first ? reinterpret_cast<const void*>(&reduce_multi_phased_kernel<float, kSum, K, false, true, RUN>)
                            : reinterpret_cast<const void*>(&reduce_multi_phased_kernel<float, kSum, K, false, false, RUN>),
                      grid, a_pm, st, 64, lds);
    default:
        return launch(first ? reinterpret_cast<const void*>(&reduce_chain_phased_kernel<float, kSum, K, false, true, RUN>)
                            : reinterpret_cast<const void*>(&reduce_chain_phased_kernel<float, kSum, K, false, false, RUN>),
                      grid, a_pc, st, 64, lds);
    }
}
}  // namespace

extern "C" int dccl_tune_runs_f32_sum(int kind, const void* const* sends, int nsend, const void* own, void* dst,
                                      size_t count, size_t lds_bytes, int run, int first, void* stream) {
    if (kind < 0 || kind > 3 || sends == nullptr || dst == nullptr || nsend < 1 || nsend > 8 ||
        lds_bytes > (64u << 10) || (reinterpret_cast<uintptr_t>(dst) & 3) || ((kind & 1) != 0) != (own != nullptr))
        return DCCL_INVALID_ARGUMENT;
    if ((kind & 1) == 0 && nsend < 2) return DCCL_INVALID_ARGUMENT;
    const Split sp = split_for_vectors<float>(reinterpret_cast<uintptr_t>(dst), count, 128);
    SendList sl{};
    PhaseList ph{};
    for (int k = 0; k < nsend; ++k) {
        sl.p[k] = static_cast<const unsigned char*>(sends[k]);
        ph.p[k] = phase_word(sl.p[k], sp.head * sizeof(float));
    }
    const auto o = static_cast<const unsigned char*>(own);
    if (o != nullptr) ph.p[nsend] = phase_word(o, sp.head * sizeof(float));
    auto d = static_cast<unsigned char*>(dst);
    const auto st = static_cast<hipStream_t>(stream);
    return with_k<1, 8>(nsend, [&](auto K) {
        switch (run) {
        case 1: return tune_runs_k<K.value, 1>(kind, first != 0, sl, ph, o, d, sp, st, lds_bytes);
        case 2: return tune_runs_k<K.value, 2>(kind, first != 0, sl, ph, o, d, sp, st, lds_bytes);
        case 4: return tune_runs_k<K.value, 4>(kind, first != 0, sl, ph, o, d, sp, st, lds_bytes);
        default: return int(DCCL_INVALID_ARGUMENT);
        }
    });
}

// ---------------------------------------------------------------------------------
// Tuning only (round 3): the pairwise launches in tile-run orders: the shipped dispatch for an element-aligned
// recv and a send at another 16-B phase or byte offset (reduce_shift_kernel, nt or cached send by its line) or
// in phase but off recv's lines (reduce_vec_kernel, StraddleCfg), or aligned (DefaultCfg), with RUN 1, 2, 4, 8.
// ---------------------------------------------------------------------------------
namespace {
template <int RUN>
int tune_pair_run(const unsigned char* s, unsigned char* r, size_t count, hipStream_t st, size_t lds) {
    const uintptr_t as = reinterpret_cast<uintptr_t>(s), ar = reinterpret_cast<uintptr_t>(r);
    const Split sp = split_for_vectors<float>(ar, count, 128);
    const uintptr_t a = (as + sp.head * sizeof(float)) & ~uintptr_t(15);
    constexpr int kP = kNtSend | kNtRecv | kNtStore, kPs = kNtRecv | kNtStore;
    if (as & 3)
        return (a & 127) ? launch_shift<float, kSum, kPs, false, 1, false, RUN>(s, r, count, st, 128, lds)
                         : launch_shift<float, kSum, kP, false, 1, false, RUN>(s, r, count, st, 128, lds);
    if ((as ^ ar) & 15)
        return (a & 127) ? launch_shift<float, kSum, kPs, false, 1, true, RUN>(s, r, count, st, 128, lds)
                         : launch_shift<float, kSum, kP, false, 1, true, RUN>(s, r, count, st, 128, lds);
    if ((as ^ ar) & 127) return launch_vec<float, kSum, VecCfg<64, 1, kPs, false, 1, RUN>>(s, r, sp, st, 0, lds);
    return launch_vec<float, kSum, VecCfg<64, 1, kP, false, 1, RUN>>(s, r, sp, st, 0, lds);
}
}  // namespace

extern "C" int dccl_tune_pair_run_f32_sum(const void* send, void* recv, size_t count, size_t lds_bytes, int run,
                                          void* stream) {
    if ((reinterpret_cast<uintptr_t>(recv) & 3) || lds_bytes > (64u << 10)) return DCCL_INVALID_ARGUMENT;
    const auto s = static_cast<const unsigned char*>(send);
    const auto r = static_cast<unsigned char*>(recv);
    const auto st = static_cast<hipStream_t>(stream);
    switch (run) {
    case 1: return tune_pair_run<1>(s, r, count, st, lds_bytes);
    case 2: return tune_pair_run<2>(s, r, count, st, lds_bytes);
    case 4: return tune_pair_run<4>(s, r, count, st, lds_bytes);
    case 8: return tune_pair_run<8>(s, r, count, st, lds_bytes);
    default: return DCCL_INVALID_ARGUMENT;
    }
}
