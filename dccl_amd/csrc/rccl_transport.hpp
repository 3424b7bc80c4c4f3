// dccl_amd/csrc/rccl_transport.hpp — RCCL (over xGMI) as the rank-to-rank transport of the
// namespace-dccl collectives, for ranks in different processes (one process per GPU).
//
// Only point-to-point RCCL calls are used (ncclSend / ncclRecv inside ncclGroupStart/End): the
// reduction itself stays the build's gfx950 combine kernel, exactly as the reference keeps its own
// combine behind Derecho's OOB transport (reduce_scatter_ring.cpp:75-94).  librccl is opened with
// dlopen at first use, so the C-ABI library has no link-time RCCL dependency and shares the copy a
// host process (e.g. PyTorch) already loaded.  Kept in its own translation unit: rccl.h's global
// ncclResult_t / ncclComm_t never meet namespace dccl's.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace dccl_amd {

constexpr size_t kRcclUniqueIdBytes = 128;  // NCCL_UNIQUE_ID_BYTES

// All functions return ncclResult_t values (numerically identical in RCCL and DCCL).
int rccl_available();  // 1 if librccl could be opened and bound
int rccl_get_unique_id(void* out128);
int rccl_comm_init(void** rcomm, uint32_t world, uint32_t rank, const void* id128);
int rccl_comm_destroy(void* rcomm);
// One grouped exchange: send `send_bytes` from `sendbuf` to `to`, receive `recv_bytes` into
// `recvbuf` from `from` (either side may be skipped with a null buffer), enqueued on `stream`.
int rccl_exchange(void* rcomm, const void* sendbuf, size_t send_bytes, uint32_t to, void* recvbuf,
                  size_t recv_bytes, uint32_t from, hipStream_t stream);
// The root's side of a one-to-all (send) or all-to-one (receive) step in ONE group: `bytes` to / from every
// rank p != self at bufs[p], enqueued on `stream`, so the root's transfers to its W - 1 peers run together
// (broadcast; the gather to the root of ncclReduce, dccl.cpp:803-840) instead of one after another.
int rccl_fan(void* rcomm, bool send, void* const* bufs, size_t bytes, uint32_t world, uint32_t self,
             hipStream_t stream);
// Every pairwise transfer of one step in ONE group: `bytes` from sendbufs[p] to rank p and from rank p into
// recvbufs[p], for every p != self (a null buffer skips that side), enqueued on `stream`: on the fully
// connected xGMI mesh the W - 1 peers' transfers use W - 1 links at once (the grouped collectives of
// algorithms.hpp).
int rccl_exchange_all(void* rcomm, const void* const* sendbufs, void* const* recvbufs, size_t bytes, uint32_t world,
                      uint32_t self, hipStream_t stream);

}  // namespace dccl_amd
