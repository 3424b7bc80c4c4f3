// dccl_amd/csrc/unaligned_multi.hip — the k-way and chain combines into a destination that is not
// element-aligned (reduce_multi_unaligned_kernel / reduce_chain_unaligned_kernel in reduce_kernels.hpp).
// Instantiated for every (T, OP) with sizeof(T) > 1 (a one-byte element is always aligned), in a
// translation unit of its own, so the build compiles it beside local_reduce.hip.
#include <hip/hip_runtime.h>

#include "dispatch.hpp"
#include "reduce_kernels.hpp"

namespace dccl_amd {
namespace {

// A grid that is a multiple of 8 (the kernels' XCD tile map); kMaxGrid is one.
size_t unaligned_grid(size_t nvec) {
    const size_t g = ceil_div(ceil_div(nvec, size_t(64)), size_t(8)) * 8;
    return g == 0 ? 8 : g;
}

// Tile order: with every source at 16-B phase 0 (plain vector loads) one front for the chip wins, the
// group-interleaved order up to k = 2 and block order above; sources at other phases keep consecutive tiles
// on one XCD, where the vector lane 63 reads past its tile meets the next tile's first line in one L2.
// 1 GiB fp32 Sum, destination + 2 B, one box (unaligned_forms_probe.py@4f20423, profiles/r3_s4_*): aligned sources
// k = 2 80.0 -> 83.4 % (group), k = 4 74.6 -> 78.0 %, k = 8 71.7 -> 76.4 % (block); the chain the same.
int unaligned_order(const PhaseList& ph, int nsend) {
    for (int k = 0; k < nsend; ++k)
        if (ph.p[k] != 0) return kOrderXcd;
    return nsend <= 2 ? kOrderGroup : kOrderBlock;
}

template <typename T, int OP, int K>
int launch_multi(SendList sl, PhaseList ph, unsigned char* r, size_t count, hipStream_t stream) {
    size_t nvec = count / Pack<T>::N;
    int order = unaligned_order(ph, K);
    void* args[] = {&sl, &ph, &r, &nvec, &count, &order};
    return launch(reinterpret_cast<const void*>(&reduce_multi_unaligned_kernel<T, OP, K>), unaligned_grid(nvec), args,
                  stream, 64);
}

template <typename T, int OP, int K>
int launch_chain(SendList sl, PhaseList ph, const unsigned char* own, unsigned char* d, size_t count,
                 hipStream_t stream) {
    size_t nvec = count / Pack<T>::N;
    int order = unaligned_order(ph, K);  // the sources' phases decide; own is the destination's window
    void* args[] = {&sl, &ph, &own, &d, &nvec, &count, &order};
    return launch(reinterpret_cast<const void*>(&reduce_chain_unaligned_kernel<T, OP, K>), unaligned_grid(nvec), args,
                  stream, 64);
}

}  // namespace

template <typename T, int OP>
int multi_unaligned_typed(SendList sl, PhaseList ph, int nsend, unsigned char* r, size_t count, hipStream_t stream) {
    return with_k<2, 8>(nsend, [&](auto K) { return launch_multi<T, OP, K.value>(sl, ph, r, count, stream); });
}

template <typename T, int OP>
int chain_unaligned_typed(SendList sl, PhaseList ph, int nsend, const unsigned char* own, unsigned char* d,
                          size_t count, hipStream_t stream) {
    return with_k<1, 8>(nsend, [&](auto K) { return launch_chain<T, OP, K.value>(sl, ph, own, d, count, stream); });
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
