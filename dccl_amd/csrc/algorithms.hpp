// dccl_amd/csrc/algorithms.hpp — collective algorithms (see algorithms.cpp).
#pragma once

#include <functional>

#include "comm.hpp"
#include "dispatch.hpp"

namespace dccl_amd {

// rank_converter_t of /root/reference/src/core/algorithms.hpp
using RankMap = std::function<uint32_t(uint32_t)>;

ncclResult_t reduce_scatter_ring(dccl::dcclComm* c, void* buffer, void* scratch, size_t count, int dtype, int op,
                                 bool device, hipStream_t st, const RankMap& to_new, const RankMap& to_old);
ncclResult_t all_gather_ring(dccl::dcclComm* c, void* buffer, size_t slot_elems, int dtype, bool device,
                             hipStream_t st, const RankMap& to_new, const RankMap& to_old);
ncclResult_t all_reduce_ring(dccl::dcclComm* c, void* buffer, void* scratch, size_t count, int dtype, int op,
                             bool device, hipStream_t st);
// DCCL_ALLREDUCE_ALGORITHM=rabenseifner: fold to 2^k ranks, recursive halving RS, recursive doubling AG.
ncclResult_t all_reduce_rabenseifner(dccl::dcclComm* c, void* buffer, void* scratch, size_t count, int dtype, int op,
                                     bool device, hipStream_t st);

}  // namespace dccl_amd
