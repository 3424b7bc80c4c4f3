// dccl_amd/csrc/phased_chain.hip — the chain combine dst = op(own, op(s{K-1}, ... op(s1, s0))) (the ring order) for element-aligned
// operands whose 16-B phases differ from the destination's (reduce_chain_phased_kernel in
// reduce_kernels.hpp).  Instantiated for every (T, OP) here, in a translation unit of its own, so the
// build compiles it beside local_reduce.hip.
#include <hip/hip_runtime.h>


#include "dispatch.hpp"
#include "reduce_kernels.hpp"

namespace dccl_amd {
namespace {

template <typename T, int OP, int K>
int launch_phased(SendList sl, PhaseList ph, const unsigned char* own, unsigned char* d, Split sp, hipStream_t stream) {
    size_t grid = ceil_div(sp.nvec, size_t(64));
    if (grid == 0 && (sp.head + sp.tail) > 0) grid = 1;
    void* args[] = {&sl, &ph, &own, &d, &sp.head, &sp.nvec, &sp.tail};
    // the per-operand form uncapped (with the XCD order up to kPhasedXcdMaxK), or the loads-first form under
    // its own cap (caps::kChainPhasedFirst, caps.hpp)
    if constexpr (caps::phased_loads_first(true, K))
        return launch(reinterpret_cast<const void*>(
                          &reduce_chain_phased_kernel<T, OP, K, false, true, caps::tile_run(caps::kChainPhasedFirst, K)>),
                      grid, args, stream, 64, caps::lds(caps::kChainPhasedFirst, K, sp.nvec * 16));
    return launch(reinterpret_cast<const void*>(&reduce_chain_phased_kernel<T, OP, K, (K <= kPhasedXcdMaxK)>), grid, args, stream, 64);
}

using StraddleKwayCfg = VecCfg<64, 1, kNtRecv | kNtStore, false>;

template <typename T, int OP, int K>
int launch_straddle(SendList sl, const unsigned char* own, unsigned char* d, Split sp, hipStream_t stream) {
    size_t grid = ceil_div(sp.nvec, size_t(64));
    if (grid == 0 && (sp.head + sp.tail) > 0) grid = 1;
    void* args[] = {&sl, &own, &d, &sp.head, &sp.nvec, &sp.tail};
    // the chain kernel's line-straddle caps by operand size (caps::kChainStraddle, caps.hpp)
    return launch(reinterpret_cast<const void*>(&reduce_chain_vec_kernel<T, OP, K, StraddleKwayCfg>), grid, args, stream, 64,
                  caps::lds(caps::kChainStraddle, K, sp.nvec * 16));
}

}  // namespace

template <typename T, int OP>
int chain_phased_typed(SendList sl, PhaseList ph, int nsend, const unsigned char* own, unsigned char* d, Split sp, hipStream_t stream) {
    return with_k<1, 8>(nsend, [&](auto K) { return launch_phased<T, OP, K.value>(sl, ph, own, d, sp, stream); });
}

template <typename T, int OP>
int chain_straddle_typed(SendList sl, int nsend, const unsigned char* own, unsigned char* d, Split sp, hipStream_t stream) {
    return with_k<1, 8>(nsend, [&](auto K) { return launch_straddle<T, OP, K.value>(sl, own, d, sp, stream); });
}

#define DCCL_PHASED_INST(T)                                                       \
    template int chain_straddle_typed<T, kSum>(SendList sl, int nsend, const unsigned char* own, unsigned char* d, Split sp, hipStream_t stream); \
    template int chain_straddle_typed<T, kProd>(SendList sl, int nsend, const unsigned char* own, unsigned char* d, Split sp, hipStream_t stream); \
    template int chain_straddle_typed<T, kMax>(SendList sl, int nsend, const unsigned char* own, unsigned char* d, Split sp, hipStream_t stream); \
    template int chain_straddle_typed<T, kMin>(SendList sl, int nsend, const unsigned char* own, unsigned char* d, Split sp, hipStream_t stream); \
    template int chain_phased_typed<T, kSum>(SendList sl, PhaseList ph, int nsend, const unsigned char* own, unsigned char* d, Split sp, hipStream_t stream);  \
    template int chain_phased_typed<T, kProd>(SendList sl, PhaseList ph, int nsend, const unsigned char* own, unsigned char* d, Split sp, hipStream_t stream); \
    template int chain_phased_typed<T, kMax>(SendList sl, PhaseList ph, int nsend, const unsigned char* own, unsigned char* d, Split sp, hipStream_t stream);  \
    template int chain_phased_typed<T, kMin>(SendList sl, PhaseList ph, int nsend, const unsigned char* own, unsigned char* d, Split sp, hipStream_t stream);
DCCL_PHASED_INST(int8_t)
DCCL_PHASED_INST(uint8_t)
DCCL_PHASED_INST(int32_t)
DCCL_PHASED_INST(uint32_t)
DCCL_PHASED_INST(int64_t)
DCCL_PHASED_INST(uint64_t)
DCCL_PHASED_INST(f16_bits)
DCCL_PHASED_INST(float)
DCCL_PHASED_INST(double)
DCCL_PHASED_INST(bf16_bits)
#undef DCCL_PHASED_INST

}  // namespace dccl_amd
