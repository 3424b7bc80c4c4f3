// dccl_amd/csrc/phased_multi.hip — the k-way combine recv = op(...op(recv, s0)..., s{K-1}) for element-aligned
// operands whose 16-B phases differ from the destination's (reduce_multi_phased_kernel in
// reduce_kernels.hpp).  Instantiated for every (T, OP) here, in a translation unit of its own, so the
// build compiles it beside local_reduce.hip.
#include <hip/hip_runtime.h>


#include "dispatch.hpp"
#include "reduce_kernels.hpp"

namespace dccl_amd {
namespace {

template <typename T, int OP, int K>
int launch_phased(SendList sl, PhaseList ph, unsigned char* r, Split sp, hipStream_t stream) {
    size_t grid = ceil_div(sp.nvec, size_t(64));
    if (grid == 0 && (sp.head + sp.tail) > 0) grid = 1;
    void* args[] = {&sl, &ph, &r, &sp.head, &sp.nvec, &sp.tail};
    // the per-operand form uncapped (with the XCD order up to kPhasedXcdMaxK), or the loads-first form under
    // its own cap (caps::kMultiPhasedFirst, caps.hpp)
    if constexpr (caps::phased_loads_first(false, K))
        return launch(reinterpret_cast<const void*>(
                          &reduce_multi_phased_kernel<T, OP, K, false, true, caps::tile_run(caps::kMultiPhasedFirst, K)>),
                      grid, args, stream, 64, caps::lds(caps::kMultiPhasedFirst, K, sp.nvec * 16));
    return launch(reinterpret_cast<const void*>(&reduce_multi_phased_kernel<T, OP, K, (K <= kPhasedXcdMaxK)>), grid, args, stream, 64);
}

// sources through the caches, in the tile-run order of caps::kRun
template <int K>
using StraddleKwayCfg = VecCfg<64, 1, kNtRecv | kNtStore, false, 0, caps::tile_run(caps::kMultiStraddle, K)>;

template <typename T, int OP, int K>
int launch_straddle(SendList sl, unsigned char* r, Split sp, hipStream_t stream) {
    size_t grid = ceil_div(sp.nvec, size_t(64));
    if (grid == 0 && (sp.head + sp.tail) > 0) grid = 1;
    void* args[] = {&sl, &r, &sp.head, &sp.nvec, &sp.tail};
    return launch(reinterpret_cast<const void*>(&reduce_multi_vec_kernel<T, OP, K, StraddleKwayCfg<K>>), grid, args, stream, 64,
                  caps::lds(caps::kMultiStraddle, K, sp.nvec * 16));
}

}  // namespace

template <typename T, int OP>
int multi_phased_typed(SendList sl, PhaseList ph, int nsend, unsigned char* r, Split sp, hipStream_t stream) {
    return with_k<2, 8>(nsend, [&](auto K) { return launch_phased<T, OP, K.value>(sl, ph, r, sp, stream); });
}

template <typename T, int OP>
int multi_straddle_typed(SendList sl, int nsend, unsigned char* r, Split sp, hipStream_t stream) {
    return with_k<2, 8>(nsend, [&](auto K) { return launch_straddle<T, OP, K.value>(sl, r, sp, stream); });
}

#define DCCL_PHASED_INST(T)                                                       \
    template int multi_straddle_typed<T, kSum>(SendList sl, int nsend, unsigned char* r, Split sp, hipStream_t stream); \
    template int multi_straddle_typed<T, kProd>(SendList sl, int nsend, unsigned char* r, Split sp, hipStream_t stream); \
    template int multi_straddle_typed<T, kMax>(SendList sl, int nsend, unsigned char* r, Split sp, hipStream_t stream); \
    template int multi_straddle_typed<T, kMin>(SendList sl, int nsend, unsigned char* r, Split sp, hipStream_t stream); \
    template int multi_phased_typed<T, kSum>(SendList sl, PhaseList ph, int nsend, unsigned char* r, Split sp, hipStream_t stream);  \
    template int multi_phased_typed<T, kProd>(SendList sl, PhaseList ph, int nsend, unsigned char* r, Split sp, hipStream_t stream); \
    template int multi_phased_typed<T, kMax>(SendList sl, PhaseList ph, int nsend, unsigned char* r, Split sp, hipStream_t stream);  \
    template int multi_phased_typed<T, kMin>(SendList sl, PhaseList ph, int nsend, unsigned char* r, Split sp, hipStream_t stream);
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
