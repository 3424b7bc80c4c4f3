// dccl_amd/csrc/unaligned_multi.hip — the k-way and chain combines into a destination that is not
// element-aligned (reduce_windows_kernel, and the round-3 forms for k <= 2, in reduce_kernels.hpp), and the
// phased launches that caps::phased_via_windows routes here (element-aligned destination).
// Instantiated for every (T, OP) with sizeof(T) > 1 (a one-byte element is always aligned), in a
// translation unit of its own, so the build compiles it beside local_reduce.hip.
#include <hip/hip_runtime.h>

#include "dispatch.hpp"
#include "reduce_kernels.hpp"

namespace dccl_amd {
namespace {

// A grid that is a multiple of 8 (the kernels' XCD / group tile maps); kMaxGrid is one.
size_t unaligned_grid(size_t nvec) {
    const size_t g = ceil_div(ceil_div(nvec, size_t(64)), size_t(8)) * 8;
    return g == 0 ? 8 : g;
}

// Tile order (1 GiB fp32 Sum, destination + 2 B, tools/ab_unaligned.py, profiles/r4_s3_ab_unaligned.json):
// with every source at 16-B phase 0 one front for the chip wins, the group-interleaved order up to k = 2
// and block order above (k = 4 78.9 %, k = 8 79.8 %); sources at other phases want consecutive tiles in one
// L2 (the lane-63 extra vector is the next tile's first): XCD ranges up to k = 4 (76.2 %), the
// group-interleaved order above (k = 8 75.2 % against 72.0 % with XCD ranges).
int unaligned_order(const PhaseList& ph, int nsend) {
    for (int k = 0; k < nsend; ++k)
        if (ph.p[k] != 0) return nsend <= 4 ? kOrderXcd : kOrderGroup;
    return nsend <= 2 ? kOrderGroup : kOrderBlock;
}

// k <= 2 with every source at 16-B phase 0: the round-3 kernels (reduce_kernels.hpp), 2.5-4.3 points faster
// there; everything else: reduce_windows_kernel.
bool round3_form(const PhaseList& ph, int nsend) {
    if (nsend > 2) return false;
    for (int k = 0; k < nsend; ++k)
        if (ph.p[k] != 0) return false;
    return true;
}

template <typename T, int OP, int K, bool CHAIN>
int launch_round3(SendList sl, PhaseList ph, const unsigned char* own, unsigned char* d, size_t count,
                  hipStream_t stream) {
    size_t nvec = count / Pack<T>::N;
    int order = unaligned_order(ph, K);
    if constexpr (CHAIN) {
        void* args[] = {&sl, &ph, &own, &d, &nvec, &count, &order};
        return launch(reinterpret_cast<const void*>(&reduce_chain_unaligned_kernel<T, OP, K>), unaligned_grid(nvec),
                      args, stream, 64);
    } else {
        void* args[] = {&sl, &ph, &d, &nvec, &count, &order};
        return launch(reinterpret_cast<const void*>(&reduce_multi_unaligned_kernel<T, OP, K>), unaligned_grid(nvec),
                      args, stream, 64);
    }
}

template <typename T, int OP, int K, bool CHAIN, bool FIRST, int ORDER>
int launch_form(WindowArgs A, hipStream_t stream, size_t lds) {
    void* args[] = {&A};
    return launch(reinterpret_cast<const void*>(&reduce_windows_kernel<T, OP, K, CHAIN, ORDER, FIRST>),
                  unaligned_grid(A.nvec), args, stream, 64, lds);
}

// The tuned form of operand class C at K (caps.hpp kWindow): one kernel per (class, K).
template <typename T, int OP, int K, bool CHAIN, int C>
int launch_tuned(const WindowArgs& A, hipStream_t stream) {
    constexpr caps::WindowForm f = caps::window_form(caps::WindowClass(C), K);
    return launch_form<T, OP, K, CHAIN, f.first != 0, int(f.order)>(A, stream, caps::lds_for_waves(f.waves));
}

template <typename T, int OP, int K, bool CHAIN>
int launch_windows(const SendList& sl, const PhaseList& ph, const unsigned char* own, unsigned char* d, size_t count,
                   hipStream_t stream) {
    WindowArgs A{};
    bool off = false;
    for (int k = 0; k < K; ++k) {
        A.p[k] = ph.p[k];
        A.a[k] = reinterpret_cast<const u32x4*>(sl.p[k] - ph.p[k]);
        A.src[k] = sl.p[k];
        off = off || ph.p[k] != 0;
    }
    const unsigned char* w = CHAIN ? own : d;  // the last window: own (chain) or the destination's own (k-way)
    A.p[K] = phase_word(w, 0);
    A.a[K] = reinterpret_cast<const u32x4*>(w - A.p[K]);
    A.own = w;
    A.dst = d;
    A.nvec = count / Pack<T>::N;
    A.count = count;
    if (count * sizeof(T) >= caps::kWindowTunedBytes)
        return off ? launch_tuned<T, OP, K, CHAIN, caps::kWinOffPhase>(A, stream)
                   : launch_tuned<T, OP, K, CHAIN, caps::kWinInPhase>(A, stream);
    if (off && caps::window_mid(CHAIN, K, count * sizeof(T))) {
        constexpr caps::WindowForm f = (CHAIN && K == 3) ? caps::kWindowMidChain3 : caps::kWindowMid;
        return launch_form<T, OP, K, CHAIN, f.first != 0, int(f.order)>(A, stream, caps::lds_for_waves(f.waves));
    }
    switch (unaligned_order(ph, K)) {  // smaller launches: the per-operand form, uncapped
    case kOrderXcd: return launch_form<T, OP, K, CHAIN, false, kOrderXcd>(A, stream, 0);
    case kOrderBlock: return launch_form<T, OP, K, CHAIN, false, kOrderBlock>(A, stream, 0);
    default: return launch_form<T, OP, K, CHAIN, false, kOrderGroup>(A, stream, 0);
    }
}

}  // namespace

template <typename T, int OP>
int multi_unaligned_typed(SendList sl, PhaseList ph, int nsend, unsigned char* r, size_t count, hipStream_t stream) {
    if (round3_form(ph, nsend))
        return with_k<2, 2>(nsend, [&](auto K) {
            return launch_round3<T, OP, K.value, false>(sl, ph, nullptr, r, count, stream);
        });
    return with_k<2, 8>(nsend, [&](auto K) {
        return launch_windows<T, OP, K.value, false>(sl, ph, nullptr, r, count, stream);
    });
}

template <typename T, int OP>
int chain_unaligned_typed(SendList sl, PhaseList ph, int nsend, const unsigned char* own, unsigned char* d,
                          size_t count, hipStream_t stream) {
    if (round3_form(ph, nsend))
        return with_k<1, 2>(nsend, [&](auto K) {
            return launch_round3<T, OP, K.value, true>(sl, ph, own, d, count, stream);
        });
    return with_k<1, 8>(nsend, [&](auto K) {
        return launch_windows<T, OP, K.value, true>(sl, ph, own, d, count, stream);
    });
}

#define DCCL_UNALIGNED_INST_OP(T, OP)                                                                             \
    template int multi_unaligned_typed<T, OP>(SendList, PhaseList, int, unsigned char*, size_t, hipStream_t);      \
    template int chain_unaligned_typed<T, OP>(SendList, PhaseList, int, const unsigned char*, unsigned char*, size_t, \
                                              hipStream_t);
#define DCCL_UNALIGNED_INST(T)              \
    DCCL_UNALIGNED_INST_OP(T, kSum)         \
    DCCL_UNALIGNED_INST_OP(T, kProd)        \
    DCCL_UNALIGNED_INST_OP(T, kMax)         \
    DCCL_UNALIGNED_INST_OP(T, kMin)
DCCL_UNALIGNED_INST(int32_t)
DCCL_UNALIGNED_INST(uint32_t)
DCCL_UNALIGNED_INST(int64_t)
DCCL_UNALIGNED_INST(uint64_t)
DCCL_UNALIGNED_INST(f16_bits)
DCCL_UNALIGNED_INST(float)
DCCL_UNALIGNED_INST(double)
DCCL_UNALIGNED_INST(bf16_bits)
#undef DCCL_UNALIGNED_INST
#undef DCCL_UNALIGNED_INST_OP

}  // namespace dccl_amd
