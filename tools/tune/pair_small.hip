// tools/tune/pair_small.hip — block-shape variants of the aligned pairwise combine for mid-size launches
// (8-128 MiB per operand, DCCL's ring-step chunks of a 256 MiB all-reduce), fp32 Sum only.
// Tools only: never linked into the product.
//
// The product launch (DefaultCfg: one-wave blocks, one 16-B vector per lane and operand) dispatches one
// workgroup per KiB of recv: 8 192 workgroups for 8 MiB, whose dispatch and drain show as the ramp and tail
// of a 5-us kernel.  The variants trade workgroups for waves per workgroup or vectors per lane:
//   variant 0: 64 threads x 1 vector (the product shape)     1: 128 x 1     2: 256 x 1     3: 512 x 1
//           4: 64 x 2                                        5: 64 x 4      6: 256 x 2     7: 1024 x 1
// and tile orders of the product shape for separately allocated operands (DCCL's scratchpad + user chunk,
// tools/pair_layout.py): 8: XCD ranges (eight fronts)   9, 10, 11: runs of 2 / 4 / 8 tiles per XCD.
//
//   extern "C" int ps_combine(int variant, size_t lds, const void* send, void* recv, size_t count, void* stream)
#include <hip/hip_runtime.h>

#include "reduce_kernels.hpp"

namespace dccl_amd {
namespace ps {

constexpr int kAllNt = kNtSend | kNtRecv | kNtStore;

template <int BLOCK, int UNROLL, bool XCD = false, int RUN = 1>
int run(const unsigned char* s, unsigned char* r, size_t count, hipStream_t st, size_t lds) {
    using C = VecCfg<BLOCK, UNROLL, kAllNt, XCD, 1, RUN>;
    const Split sp = split_for_vectors<float>(reinterpret_cast<uintptr_t>(r), count, 128);
    return launch_vec<float, kSum, C>(s, r, sp, st, 0, lds);
}

}  // namespace ps
}  // namespace dccl_amd

using namespace dccl_amd;

extern "C" int ps_combine(int variant, size_t lds, const void* send, void* recv, size_t count, void* stream) {
    const auto s = static_cast<const unsigned char*>(send);
    const auto r = static_cast<unsigned char*>(recv);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if ((reinterpret_cast<uintptr_t>(s) ^ reinterpret_cast<uintptr_t>(r)) & 127) return DCCL_INVALID_ARGUMENT;
    switch (variant) {
    case 0: return ps::run<64, 1>(s, r, count, st, lds);
    case 1: return ps::run<128, 1>(s, r, count, st, lds);
    case 2: return ps::run<256, 1>(s, r, count, st, lds);
    case 3: return ps::run<512, 1>(s, r, count, st, lds);
    case 4: return ps::run<64, 2>(s, r, count, st, lds);
    case 5: return ps::run<64, 4>(s, r, count, st, lds);
    case 6: return ps::run<256, 2>(s, r, count, st, lds);
    case 7: return ps::run<1024, 1>(s, r, count, st, lds);
    case 8: return ps::run<64, 1, true>(s, r, count, st, lds);      // XCD ranges: 8 fronts, one per XCD
    case 9: return ps::run<64, 1, false, 2>(s, r, count, st, lds);  // tile runs of 2 / 4 / 8 per XCD
    case 10: return ps::run<64, 1, false, 4>(s, r, count, st, lds);
    case 11: return ps::run<64, 1, false, 8>(s, r, count, st, lds);
    default: return DCCL_INVALID_ARGUMENT;
    }
}
