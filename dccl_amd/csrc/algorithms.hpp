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
// Grouped forms for the RCCL transport (device buffers): every contribution to the slot this rank owns
// arrives in ONE grouped exchange (W - 1 xGMI links at once), then ONE chain combine applies them in the
// ring's order, so results are bit-identical to reduce_scatter_ring with the same maps.  `shift`: rank r owns
// slot (r + shift) % W; 1 = all_reduce_ring's identity maps, 0 = ncclReduceScatter's maps.  `in` (count
// elements) is only read; the owned slot's result goes to `dst`.
ncclResult_t reduce_scatter_grouped(dccl::dcclComm* c, const void* in, void* dst, size_t count, int dtype, int op,
                                    hipStream_t st, uint32_t shift);
// reduce_scatter_grouped(shift 1) from `send` into recv's owned slot, then one grouped all-gather of the
// reduced slots into `recv` (send == recv allowed).
ncclResult_t all_reduce_grouped(dccl::dcclComm* c, const void* send, void* recv, size_t count, int dtype, int op,
                                hipStream_t st);
// DCCL_ALLREDUCE_ALGORITHM=rabenseifner: fold to 2^k ranks, recursive halving RS, recursive doubling AG.
ncclResult_t all_reduce_rabenseifner(dccl::dcclComm* c, void* buffer, void* scratch, size_t count, int dtype, int op,
                                     bool device, hipStream_t st);

}  // namespace dccl_amd
