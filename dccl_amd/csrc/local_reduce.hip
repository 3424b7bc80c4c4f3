// dccl_amd/csrc/local_reduce.hip — the MI355X (gfx950) local bucket-reduction combine.
//
//   recv[i] = op(recv[i], send[i]),  i in [0, count)
//
// Replaces the reference's single CUDA kernel reduce_kernel<DT> and its launcher
// do_device_reduce (/root/reference/src/core/reduce.cu:9-100).  That kernel moves one
// scalar element per thread per iteration through a runtime op switch on a grid of
// num_SMs x 256 threads; this one is an HBM stream:
//   * 16-byte (global_load_dwordx4 / global_store_dwordx4) accesses of both operands;
//   * the shipped shape (DefaultCfg, chosen by tune_reduce.py@4f20423 on MI355X): one-wave
//     (64-thread) blocks, one 16-B vector per lane and operand, i.e. one 1 KiB tile of each
//     operand per block and ~1M blocks for 1 GiB; every load and the store non-temporal;
//   * dtype and op are template parameters (no per-element switch);
//   * unaligned head / tail elements are folded into block 0 of the same launch;
//   * element-aligned operands with different 16-B phases take the shifted vector kernel
//     (aligned loads of both, a cross-lane funnel shift of send), and so does a send at any byte address
//     against an element-aligned recv; a recv that is not element-aligned takes one 16-B access per lane
//     at the displaced addresses themselves (reduce_unaligned_kernel).
// No LDS and no MFMA: each element is touched once (BASELINE.json north_star).
//
// Roofline: HBM, 3 * count * sizeof(T) algorithmic bytes (read send, read recv, write recv).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "dccl/dccl_reduce.h"
#include "dispatch.hpp"
#include "reduce_kernels.hpp"

namespace dccl_amd {
namespace {

// Default configuration of the shipped kernel.  One-wave blocks, one 16-B vector per lane and operand, every access non-temporal: the
// fastest shape measured on MI355X at 1 GiB (tune_reduce.py@4f20423, profiles/r1_tune.json).
using DefaultCfg = VecCfg<64, 1, kNtSend | kNtRecv | kNtStore, false>;
// When send's 128-B phase differs from recv's, every 1 KiB send tile straddles 9 lines, one of them
// shared with the next tile (a wave on another XCD): send is then loaded through the caches, so the
// shared line is fetched from HBM once (phase_probe.py@4f20423 on MI355X, 1 GiB fp32 Sum: 81.0 % with
// non-temporal send loads, 84.1 % cached; with equal phases non-temporal is 1 % faster).
using StraddleCfg = VecCfg<64, 1, kNtRecv | kNtStore, false>;
// The shifted kernel (operands with different 16-B phases) by the same rule; lane 63's extra send
// vector is always loaded through the caches.
constexpr int ShiftPolicy = kNtSend | kNtRecv | kNtStore;
constexpr int ShiftStraddlePolicy = kNtRecv | kNtStore;
// ... in the group-interleaved tile order (run_tile<8>): the vector lane 63 reads past its tile and the next
// tile's first line then meet in one L2 in 7 of 8 cases while the chip sweeps one front.  1 GiB fp32 Sum,
// pooled layout, two boxes (pair_runs_probe.py@4f20423, profiles/r3_s16_*, r3_s17_*): send + 4 B 83.8 -> 85.2-85.4 %,
// send + 1 B 83.7-83.9 -> 85.3-85.4 %, send + 20 B (cached send loads) 84.1 -> 84.7 %: the aligned kernel's rate.
constexpr int kShiftRun = 8;
// recv is aligned to this many bytes by the head scalars (DCCL_REDUCE_ALIGN, a power of two from 16 to
// 4096; default 128, one line): a recv that straddles lines costs 10-15 % (profiles/r1_s3_phase_probe.json).
size_t recv_align() {
    static const size_t v = [] {
        const char* e = std::getenv("DCCL_REDUCE_ALIGN");
        const unsigned long long x = e ? std::strtoull(e, nullptr, 10) : 128ull;
        return (x >= 16 && x <= 4096 && (x & (x - 1)) == 0) ? static_cast<size_t>(x) : size_t(128);
    }();
    return v;
}
// grid_cap (a multiple of 8; 0 = none): at most this many one-wave blocks, each striding over the tiles.  The
// zero-copy combine of host operands takes it (host_staged.cpp): uncapped, every wave of a PCIe-bound launch
// issues its reads at once and the writes follow in one burst at the end, so the link's two directions work one
// after the other instead of together.
template <typename T, int OP>
int reduce_typed(const void* send, void* recv, size_t count, hipStream_t stream, size_t grid_cap = 0) {
    const auto s = static_cast<const unsigned char*>(send);
    const auto r = static_cast<unsigned char*>(recv);
    const uintptr_t as = reinterpret_cast<uintptr_t>(send), ar = reinterpret_cast<uintptr_t>(recv);
    const size_t align = recv_align();
    if (ar % sizeof(T)) {  // recv's elements straddle its 16-B vectors: one 16-B access per lane at any address
        const size_t nvec = count / Pack<T>::N;
        size_t grid = ceil_div(ceil_div(nvec, size_t(64)), size_t(8)) * 8;  // a multiple of 8 (kMaxGrid is one)
        if (grid == 0) grid = 8;
        if (grid_cap && grid > grid_cap) grid = grid_cap;
        unsigned p = unsigned(as & 15);
        int order = kOrderGroup;  // one front, shared lines in one L2: +4.5 points over the XCD ranges (round 3)
        void* args[] = {const_cast<unsigned char**>(&s), &p, const_cast<unsigned char**>(&r),
                        const_cast<size_t*>(&nvec), &count, &order};
        return launch(reinterpret_cast<const void*>(&reduce_unaligned_kernel<T, OP>), grid, args, stream, 64);
    }
    if (as % sizeof(T)) {  // an element-aligned recv and a send at any byte address: the shifted kernel
        const Split sp = split_for_vectors<T>(ar, count, align);
        const uintptr_t a = (as + sp.head * sizeof(T)) & ~uintptr_t(15);
        return (a & 127) ? launch_shift<T, OP, ShiftStraddlePolicy, false, 0, false, kShiftRun>(s, r, count, stream,
                                                                                                align, 0, grid_cap)
                         : launch_shift<T, OP, ShiftPolicy, false, 0, false, kShiftRun>(s, r, count, stream, align, 0,
                                                                                       grid_cap);
    }
    const Split sp = split_for_vectors<T>(ar, count, align);
    if ((as ^ ar) & 15) {
        const uintptr_t a = (as + sp.head * sizeof(T)) & ~uintptr_t(15);  // the shifted kernel's send vectors
        return (a & 127) ? launch_shift<T, OP, ShiftStraddlePolicy, false, 0, true, kShiftRun>(s, r, count, stream,
                                                                                               align, 0, grid_cap)
                         : launch_shift<T, OP, ShiftPolicy, false, 0, true, kShiftRun>(s, r, count, stream, align, 0,
                                                                                      grid_cap);
    }
    if ((as ^ ar) & 127) return launch_vec<T, OP, StraddleCfg>(s, r, sp, stream, grid_cap);
    return launch_vec<T, OP, DefaultCfg>(s, r, sp, stream, grid_cap);
}

// k-way combine: every resident wave keeps k+1 16-B loads per lane in flight, so the resident waves
// per CU are capped (through unused dynamic LDS, 160 KiB per CU) to keep roughly 50-80 KiB of reads
// outstanding per CU.  Measured optimum per k at 1 GiB per operand on MI355X, fp32 Sum
// (tune_multi.py@4f20423, profiles/r1_tune_multi_waves.json): 4-7 % faster than 32 waves for k >= 2.
// In-phase sources off recv's 128-B line grid (recv is line-aligned past the head): their loads go
// through the caches, so the line two neighbouring tiles share is fetched once (StraddleCfg's rule).
// 1 GiB-class A/B on one MI355X (profiles/r1_s5_kway_straddle_ab.json): k = 1 76.7 -> 85.6 %,
// k = 2 75.5 -> 78.0 %, k = 4 74.4 -> 78.4 %, k = 7 72.3 -> 77.5 % of HBM peak.
inline bool any_straddles(const SendList& sl, int nsend, size_t off) {
    for (int k = 0; k < nsend; ++k)
        if ((reinterpret_cast<uintptr_t>(sl.p[k]) + off) & 127) return true;
    return false;
}

template <typename T, int OP, int K>
int launch_multi_vec(SendList sl, unsigned char* r, Split sp, hipStream_t stream) {
    using C = DefaultCfg;
    size_t grid = ceil_div(sp.nvec, C::TILE);
    if (grid == 0 && (sp.head + sp.tail) > 0) grid = 1;
    void* args[] = {&sl, &r, &sp.head, &sp.nvec, &sp.tail};
    return launch(reinterpret_cast<const void*>(&reduce_multi_vec_kernel<T, OP, K, C>), grid, args, stream, C::BLOCK,
                  caps::lds(caps::kMulti, K, sp.nvec * 16));
}

template <typename T, int OP>
int reduce_multi_typed(const void* const* sends, int nsend, void* recv, size_t count, hipStream_t stream) {
    // One source is the pairwise combine itself: take its tuned dispatch (every alignment class).  The
    // k-way kernel at k = 1 ran at 78.7 % of peak at 1 GiB against 85 % for the pairwise kernel
    // (profiles/r2_kway_pmc.json, traffic exactly 3N in both).
    if (nsend == 1) return reduce_typed<T, OP>(sends[0], recv, count, stream);
    SendList sl{};
    const uintptr_t ar = reinterpret_cast<uintptr_t>(recv);
    bool vec_ok = (ar % sizeof(T)) == 0;
    for (int k = 0; k < nsend; ++k) {
        sl.p[k] = static_cast<const unsigned char*>(sends[k]);
        if ((reinterpret_cast<uintptr_t>(sends[k]) ^ ar) & 15) vec_ok = false;
    }
    auto r = static_cast<unsigned char*>(recv);
    if (ar % sizeof(T)) {  // recv not element-aligned: 16-B accesses at its own address, sources at any phase
        if constexpr (sizeof(T) > 1) {
            PhaseList ph{};
            for (int k = 0; k < nsend; ++k) ph.p[k] = phase_word(sl.p[k], 0);
            return multi_unaligned_typed<T, OP>(sl, ph, nsend, r, count, stream);
        }
    }
    if (!vec_ok) {  // an element-aligned recv and sources at other 16-B (or byte) phases: the phased kernel
        if constexpr (sizeof(T) > 1) {
            if (caps::phased_via_windows(false, nsend, count * sizeof(T), (ar & 15) == 0)) {  // or the windows kernel (caps.hpp)
                PhaseList ph{};
                for (int k = 0; k < nsend; ++k) ph.p[k] = phase_word(sl.p[k], 0);
                return multi_unaligned_typed<T, OP>(sl, ph, nsend, r, count, stream);
            }
        }
        const Split sp = split_for_vectors<T>(ar, count, recv_align());
        PhaseList ph{};
        for (int k = 0; k < nsend; ++k) ph.p[k] = phase_word(sl.p[k], sp.head * sizeof(T));
        return multi_phased_typed<T, OP>(sl, ph, nsend, r, sp, stream);
    }
    const Split sp = split_for_vectors<T>(ar, count, recv_align());
    if (any_straddles(sl, nsend, sp.head * sizeof(T))) return multi_straddle_typed<T, OP>(sl, nsend, r, sp, stream);
    return with_k<2, 8>(nsend, [&](auto K) { return launch_multi_vec<T, OP, K.value>(sl, r, sp, stream); });
}

// ---------------------------------------------------------------------------------
// Multi-source copy (the all-gather half of the direct collectives): pair y copies `bytes`
// from src[y] to dst[y]; every pair in one launch, so reads from up to 8 peers (8 xGMI links)
// are in flight together.  Any byte alignment of src[y] and dst[y].
// ---------------------------------------------------------------------------------
struct CopyList { const unsigned char* src[8]; unsigned char* dst[8]; };

// Pairs are interleaved block by block (block b copies for pair b % npairs), so the blocks the
// dispatcher issues together read from every source at once: with a peer per pair, every xGMI link is
// busy for the whole launch instead of one peer after another (a y-row per pair would be dispatched
// row by row).  dst is walked in aligned 16-B vectors; a source at another 16-B phase is read with
// the phased kernels' cross-lane funnel shift (ld_phased), so every access stays a 16-B vector.
__global__ __launch_bounds__(64) void copy_multi_kernel(CopyList cl, int npairs, size_t bytes) {
    const unsigned y = blockIdx.x % unsigned(npairs);
    const size_t x = blockIdx.x / unsigned(npairs), gx = gridDim.x / unsigned(npairs);
    const unsigned char* s = cl.src[y];
    unsigned char* d = cl.dst[y];
    size_t head = (16 - (reinterpret_cast<uintptr_t>(d) & 15)) & 15;
    if (head > bytes) head = bytes;
    const size_t nvec = (bytes - head) / 16;
    const unsigned p = unsigned((reinterpret_cast<uintptr_t>(s) + head) & 15);  // uniform per block
    u32x4* vd = reinterpret_cast<u32x4*>(d + head);
    for (size_t t = x; t * 64 < nvec; t += gx) {  // uniform per wave: every lane reaches the lane exchange
        const size_t v = t * 64 + threadIdx.x;
        const u32x4 val = ld_phased(s + head, p, v, nvec);
        if (v < nvec) __builtin_nontemporal_store(val, vd + v);
    }
    if (x == 0) {
        for (size_t b = threadIdx.x; b < head; b += 64) d[b] = s[b];
        for (size_t b = head + nvec * 16 + threadIdx.x; b < bytes; b += 64) d[b] = s[b];
    }
}

template <typename T, int OP, int K>
int launch_chain_vec(SendList sl, const unsigned char* own, unsigned char* d, Split sp, hipStream_t stream,
                     size_t grid_cap) {
    using C = DefaultCfg;
    size_t grid = ceil_div(sp.nvec, C::TILE);
    if (grid == 0 && (sp.head + sp.tail) > 0) grid = 1;
    if (grid_cap && grid > grid_cap) grid = grid_cap;
    void* args[] = {&sl, &own, &d, &sp.head, &sp.nvec, &sp.tail};
    return launch(reinterpret_cast<const void*>(&reduce_chain_vec_kernel<T, OP, K, C>), grid, args, stream, C::BLOCK,
                  caps::lds(caps::kChain, K, sp.nvec * 16));
}

// grid_cap: as reduce_typed's, for the zero-copy host chain combine; it applies to the in-phase launches (the host
// staging keeps every operand 256-B aligned), the other alignment classes keep their own grids.
template <typename T, int OP>
int reduce_chain_typed(const void* const* sends, int nsend, const void* own, void* dst, size_t count,
                       hipStream_t stream, size_t grid_cap) {
    // dst = op(own, s0) in place is the pairwise combine recv = op(recv, send) with recv = own = dst
    if (nsend == 1 && own == dst) return reduce_typed<T, OP>(sends[0], dst, count, stream, grid_cap);
    SendList sl{};
    const uintptr_t ad = reinterpret_cast<uintptr_t>(dst), ao = reinterpret_cast<uintptr_t>(own);
    bool src_off = false;  // some source at another 16-B phase than dst
    for (int k = 0; k < nsend; ++k) {
        sl.p[k] = static_cast<const unsigned char*>(sends[k]);
        if ((reinterpret_cast<uintptr_t>(sends[k]) ^ ad) & 15) src_off = true;
    }
    const bool vec_ok = (ad % sizeof(T)) == 0 && ((ad ^ ao) & 15) == 0 && !src_off;
    const auto o = static_cast<const unsigned char*>(own);
    auto d = static_cast<unsigned char*>(dst);
    if (ad % sizeof(T)) {  // dst not element-aligned: 16-B accesses at its own address, operands at any phase
        if constexpr (sizeof(T) > 1) {
            PhaseList ph{};
            for (int k = 0; k < nsend; ++k) ph.p[k] = phase_word(sl.p[k], 0);
            ph.p[nsend] = phase_word(o, 0);
            return chain_unaligned_typed<T, OP>(sl, ph, nsend, o, d, count, stream);
        }
    }
    if (!vec_ok) {  // an element-aligned dst and operands at other 16-B (or byte) phases: the phased kernel
        if constexpr (sizeof(T) > 1) {
            // or the windows kernel (caps.hpp), whose off-phase forms were measured with sources off phase (not
            // with `own` alone off phase: that launch keeps the phased kernels)
            if (src_off && caps::phased_via_windows(true, nsend, count * sizeof(T), (ad & 15) == 0)) {
                PhaseList ph{};
                for (int k = 0; k < nsend; ++k) ph.p[k] = phase_word(sl.p[k], 0);
                ph.p[nsend] = phase_word(o, 0);
                return chain_unaligned_typed<T, OP>(sl, ph, nsend, o, d, count, stream);
            }
        }
        const Split sp = split_for_vectors<T>(ad, count, recv_align());
        PhaseList ph{};
        for (int k = 0; k < nsend; ++k) ph.p[k] = phase_word(sl.p[k], sp.head * sizeof(T));
        ph.p[nsend] = phase_word(o, sp.head * sizeof(T));
        return chain_phased_typed<T, OP>(sl, ph, nsend, o, d, sp, stream);
    }
    const Split sp = split_for_vectors<T>(ad, count, recv_align());
    if (any_straddles(sl, nsend, sp.head * sizeof(T))) return chain_straddle_typed<T, OP>(sl, nsend, o, d, sp, stream);
    return with_k<1, 8>(nsend,
                        [&](auto K) { return launch_chain_vec<T, OP, K.value>(sl, o, d, sp, stream, grid_cap); });
}

struct ReduceChainFn {
    template <typename T, int OP>
    static int run(const void* const* sends, int nsend, const void* own, void* dst, size_t count, hipStream_t stream,
                   size_t grid_cap) {
        return reduce_chain_typed<T, OP>(sends, nsend, own, dst, count, stream, grid_cap);
    }
};

struct ReduceFn {
    template <typename T, int OP>
    static int run(const void* send, void* recv, size_t count, hipStream_t stream, size_t grid_cap) {
        return reduce_typed<T, OP>(send, recv, count, stream, grid_cap);
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

namespace dccl_amd {
// dccl_local_reduce with at most grid_cap one-wave blocks (a multiple of 8; 0 = none): the zero-copy combine of
// host operands (host_staged.cpp).  Hidden: not part of the library's ABI.
__attribute__((visibility("hidden"))) int local_reduce_capped(const void* send, void* recv, int dtype, size_t count, int op, hipStream_t stream,
                        size_t grid_cap) {
    const int v = validate(dtype, op);
    if (v != DCCL_SUCCESS) return v;
    if (count == 0) return DCCL_SUCCESS;
    if (send == nullptr || recv == nullptr) return DCCL_INVALID_ARGUMENT;
    if (partial_overlap(send, recv, count * size_of_dtype(dtype))) return DCCL_INVALID_ARGUMENT;
    return dispatch<ReduceFn>(dtype, op, send, recv, count, stream, grid_cap / 8 * 8);
}
}  // namespace dccl_amd

extern "C" int dccl_local_reduce(const void* send, void* recv, int dtype, size_t count, int op, void* stream) {
    return local_reduce_capped(send, recv, dtype, count, op, static_cast<hipStream_t>(stream), 0);
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
    if (sources_overlap_destination(sends, nsend, nullptr, recv, count * size_of_dtype(dtype)))
        return DCCL_INVALID_ARGUMENT;
    return dispatch<ReduceMultiFn>(dtype, op, sends, nsend, recv, count, static_cast<hipStream_t>(stream));
}

namespace dccl_amd {
// dccl_local_reduce_chain with the in-phase launches capped at grid_cap one-wave blocks (a multiple of 8; 0 =
// none): the zero-copy host chain combine (host_staged.cpp).  Hidden: not part of the library's ABI.
__attribute__((visibility("hidden"))) int local_reduce_chain_capped(const void* const* sends, int nsend, const void* own, void* dst, int dtype,
                              size_t count, int op, hipStream_t stream, size_t grid_cap) {
    const int v = validate(dtype, op);
    if (v != DCCL_SUCCESS) return v;
    if (nsend < 1 || nsend > 8 || sends == nullptr) return DCCL_INVALID_ARGUMENT;
    if (count == 0) return DCCL_SUCCESS;
    if (own == nullptr || dst == nullptr) return DCCL_INVALID_ARGUMENT;
    for (int k = 0; k < nsend; ++k)
        if (sends[k] == nullptr) return DCCL_INVALID_ARGUMENT;
    if (sources_overlap_destination(sends, nsend, own, dst, count * size_of_dtype(dtype)))
        return DCCL_INVALID_ARGUMENT;
    return dispatch<ReduceChainFn>(dtype, op, sends, nsend, own, dst, count, stream, grid_cap / 8 * 8);
}
}  // namespace dccl_amd

extern "C" int dccl_local_reduce_chain(const void* const* sends, int nsend, const void* own, void* dst, int dtype,
                                       size_t count, int op, void* stream) {
    return local_reduce_chain_capped(sends, nsend, own, dst, dtype, count, op, static_cast<hipStream_t>(stream), 0);
}

extern "C" int dccl_copy_multi(const void* const* srcs, void* const* dsts, int npairs, size_t bytes, void* stream) {
    if (npairs < 0 || npairs > 8 || (npairs > 0 && (srcs == nullptr || dsts == nullptr))) return DCCL_INVALID_ARGUMENT;
    if (npairs == 0 || bytes == 0) return DCCL_SUCCESS;
    CopyList cl{};
    for (int y = 0; y < npairs; ++y) {
        if (srcs[y] == nullptr || dsts[y] == nullptr) return DCCL_INVALID_ARGUMENT;
        cl.src[y] = static_cast<const unsigned char*>(srcs[y]);
        cl.dst[y] = static_cast<unsigned char*>(dsts[y]);
    }
    // a pair's dst may be its own src (a no-op copy); it may share no other byte with any src or dst
    for (int y = 0; y < npairs; ++y)
        for (int z = 0; z < npairs; ++z) {
            if (z == y ? partial_overlap(srcs[z], dsts[y], bytes) : (partial_overlap(srcs[z], dsts[y], bytes) ||
                                                                     srcs[z] == dsts[y]))
                return DCCL_INVALID_ARGUMENT;
            if (z > y && (partial_overlap(dsts[z], dsts[y], bytes) || dsts[z] == dsts[y])) return DCCL_INVALID_ARGUMENT;
        }
    const auto st = static_cast<hipStream_t>(stream);
    size_t gx = ceil_div(bytes / 16 + 1, 64);
    if (gx > (size_t(1) << 20)) gx = size_t(1) << 20;
    void* args[] = {&cl, &npairs, &bytes};
    return hipLaunchKernel(reinterpret_cast<const void*>(&copy_multi_kernel), dim3(unsigned(gx * size_t(npairs))),
                           dim3(64), args, 0, st) == hipSuccess
               ? DCCL_SUCCESS
               : DCCL_UNHANDLED_DEVICE_ERROR;
}
