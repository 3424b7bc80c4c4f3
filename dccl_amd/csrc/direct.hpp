// dccl_amd/csrc/direct.hpp — direct (peer-read) collectives for one node of MI355X GPUs.
//
// The reference moves every chunk around a ring, one neighbour and one chunk per step
// (reduce_scatter_ring.cpp:73-101, all_gather_ring.cpp:44-64): on the fully connected xGMI mesh
// of an MI355X node that keeps one of a GPU's 7 links busy at a time.  Here each rank reads its
// peers' buffers directly, mapped into its address space:
//   reduce-scatter  one dccl_local_reduce_chain launch per owned chunk reads that chunk from all
//                   W-1 peers at once (all links) and applies the ring's combines in the ring's
//                   order, so results are bit-identical to the reference ring;
//   all-gather      one dccl_copy_multi launch pulls every other chunk from its owner.
// Peers are synchronised with barriers between the phases: after each rank's stream has drained
// (inputs written / own chunk reduced) and before anyone may overwrite what peers still read.
//
// Two ways to see peer buffers:
//   * in-process ranks (threads; comm.hpp): pointers are published through the Group;
//   * the IPC transport (DCCL_TRANSPORT=ipc; one process per GPU): each communicator's scratch is exported
//     with hipIpcGetMemHandle (dmabuf) under serials the exporter never reuses, published in a POSIX
//     shared-memory segment and opened once by each peer (its token verified); an export ends only by a
//     retirement written into that segment (ipc_cache.hpp).  Every input is copied into the scratch.
//     Barriers spin on counters in the same segment and watch the peers' processes.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "comm.hpp"

namespace dccl_amd {

constexpr uint32_t kDirectMaxWorld = 8;  // one 8-GPU node; <= 8 copy pairs / chain sends per launch

// Cross-process IPC transport: join (rank 0 creates the segment and publishes its name through a
// file in DCCL_BOOTSTRAP_DIR keyed by DCCL_BOOTSTRAP_TAG / MASTER_PORT) and leave.
ncclResult_t ipc_join(dccl::dcclComm* c, uint32_t world, uint32_t rank);
ncclResult_t ipc_leave(dccl::dcclComm* c);
// dcclRegisterCacheMemory / dcclDeregisterCacheMemory of device memory on an IPC communicator: validated and
// tracked only (peers read every input through the communicator's scratch).
ncclResult_t ipc_register(void* buffer, size_t size);
ncclResult_t ipc_deregister(void* buffer);
// The process's IPC counters (dccl_ipc_stats, include/dccl/dccl_comm.h): fills min(n, count) of them and
// returns how many there are.
int ipc_stats(uint64_t* out, int n);

// True when the collectives of `c` on device buffers take the direct algorithms: always on the
// IPC transport; on the in-process transport (W <= 8) unless DCCL_ALLREDUCE_ALGORITHM is ring or
// rabenseifner.
bool direct_selected(const dccl::dcclComm* c);

ncclResult_t direct_all_reduce(dccl::dcclComm* c, const void* send, void* recv, size_t count, int dtype, int op,
                               hipStream_t st);

// Host buffers of an in-process group: the direct all_reduce with the chain combine staged through the
// GPU (dccl_local_reduce_chain_host, staged in double-buffered pieces) and the all-gather by memcpy from
// the owners' buffers.  Selected like direct_selected().
bool host_direct_selected(const dccl::dcclComm* c, size_t slot_bytes);
ncclResult_t direct_all_reduce_host(dccl::dcclComm* c, const void* send, void* recv, size_t count, int dtype,
                                    int op);
ncclResult_t direct_reduce_scatter_host(dccl::dcclComm* c, const void* send, void* recv, size_t recvcount,
                                        int dtype, int op);
ncclResult_t direct_reduce_scatter(dccl::dcclComm* c, const void* send, void* recv, size_t recvcount, int dtype,
                                   int op, hipStream_t st);
ncclResult_t direct_reduce(dccl::dcclComm* c, const void* send, void* recv, size_t count, int dtype, int op,
                           uint32_t root, hipStream_t st);
ncclResult_t direct_all_gather(dccl::dcclComm* c, const void* send, void* recv, size_t sendcount, int dtype,
                               hipStream_t st);
ncclResult_t direct_broadcast(dccl::dcclComm* c, const void* send, void* recv, size_t count, int dtype,
                              uint32_t root, hipStream_t st);

}  // namespace dccl_amd
