// dccl_amd/csrc/misaligned.hip — production instantiations of the combine for a recv that is not
// element-aligned (misaligned.hpp: a boundary pass, then a vector pass that writes every recv vector whole
// from one wave).  Shape: 4 vectors per lane (4 KiB tiles), send loaded through the caches — chosen by
// tools/misaligned_ab.py on MI355X.
#include <hip/hip_runtime.h>

#include "dispatch.hpp"
#include "misaligned.hpp"
#include "reduce_kernels.hpp"

namespace dccl_amd {

template <typename T, int OP>
int reduce_misaligned_typed(const unsigned char* s, unsigned char* r, size_t count, hipStream_t stream) {
    return mis::launch_misaligned<T, OP, 4, false>(s, r, count, stream);
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
