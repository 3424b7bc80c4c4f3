/*
 * include/dccl/dccl_comm.h — C-ABI of the collectives built around the combine, for FFI callers
 * (the C++ surface is include/dccl/dccl.hpp).  Communicators are opaque `void*`; integer enums
 * and results are the ncclDataType_t / ncclRedOp_t / ncclResult_t values.
 *
 *   dccl_comm_init_rank   in-process group: one communicator per thread, blocks until all
 *                         `world` ranks joined (dcclCommInitRank)
 *   dccl_get_unique_id /  cross-process group over the RCCL (xGMI) transport, one process per
 *   dccl_comm_init_rccl   GPU; the 128-byte id travels out of band (dcclCommInitRccl)
 *   dccl_comm_init_p2p    a group over a point-to-point transport the caller plugs in: one exchange
 *                         call sends one buffer to a rank and receives one from a rank (either side may
 *                         be skipped with NULL), complete on return for host buffers and ordered on
 *                         `stream` for device buffers; `memory` = 1 host buffers, 2 device buffers,
 *                         3 both.  This is where the reference's own transport plugs in: Derecho's OOB
 *                         send / recv / wait (/root/reference/src/core/internal_common.hpp:698-792)
 *                         wrapped as one exchange.  The ring collectives
 *                         (reduce_scatter_ring.cpp:73-101, all_gather_ring.cpp:44-64) then run on it,
 *                         with the gfx950 combine after every receive.
 *   dccl_comm_init_ipc    cross-process group over the IPC peer-read transport (one process per GPU
 *                         on one node; rendezvous through DCCL_BOOTSTRAP_DIR, dcclCommInitIpc).  A failed
 *                         collective aborts the group, like an aborted NCCL communicator: every later
 *                         collective returns ncclRemoteError (6) until dccl_comm_finalize, which still
 *                         returns and releases the shared segment and the peers' mappings.  (The
 *                         in-process transport agrees per collective and stays usable after a failure.)
 *                         Inputs are first copied (on the collective's stream) into the communicator's
 *                         scratch, one library-owned allocation exported once, whose token every peer
 *                         checks through its new mapping; peers never read user memory.  A peer whose
 *                         process dies ends every other rank's wait with ncclRemoteError within ~0.1 s; a
 *                         live peer may take any time between collectives (no limit unless
 *                         DCCL_IPC_TIMEOUT_S sets one; 300 s when peers' processes are not visible, e.g.
 *                         another pid namespace, which turns the liveness check off).  Communicators of one
 *                         process share one mapping cache under one mutex: collectives driven from several
 *                         threads at once serialise while they map peer buffers (a failing open retries
 *                         for up to ~0.5 s under it); a collective releases its mappings once its stream
 *                         has drained, before its last barrier.
 *   dccl_comm_register /  dcclRegisterCacheMemory / dcclDeregisterCacheMemory (/root/reference/src/core/
 *   dccl_comm_deregister  dccl.cpp:503-549): 64-byte aligned address and size.  Host memory is page-locked.
 *                         Device memory: validated (an IPC communicator checks it is a device allocation
 *                         of this process and the range lies inside it) and tracked, nothing exported
 *                         (registering a start address again counts; deregister as often).
 *   dccl_ipc_stats        the process's IPC transport counters, in this order: exports made, exports
 *                         retired, (0), scratch copies, scratch bytes copied, scratch grows, (0),
 *                         mappings opened, mappings reused, mappings closed on retirement, retirement-log
 *                         overflows, mappings trimmed, alias evictions, alias errors, open retries, size
 *                         mismatches, mappings open, bytes mapped, exports with recycled handle bytes (never
 *                         published), (0), new scratch mappings whose token did not read back.  The (0)
 *                         slots counted the registered in-place path removed in round 5.  Fills min(n,
 *                         count) values; returns count.
 *   dccl_bootstrap_unique_id  single-node exchange of the RCCL id through DCCL_BOOTSTRAP_DIR: rank 0
 *                         creates and publishes it, the others wait (DCCL_BOOTSTRAP_TIMEOUT_S, default
 *                         120 s) for a file published by a LIVE rank 0 of the same world size, so a
 *                         file an earlier job left behind is never taken (what ncclCommInit does
 *                         with DCCL_TRANSPORT=rccl).  A second call under the same tag waits for a new
 *                         publication: a rank never takes the id it already took, and the file is removed
 *                         as soon as every reader rank took it, so a process started later never takes a
 *                         formed group's id (even without dccl_bootstrap_done)
 *   dccl_bootstrap_done   rank 0 removes the published id once dccl_comm_init_rccl returned (every rank
 *                         has read it then), as ncclCommInit does; other ranks: no-op
 *   dccl_all_reduce       ncclAllReduce       (/root/reference/include/dccl/dccl.hpp:206-207)
 *   dccl_reduce_scatter   ncclReduceScatter   (/root/reference/include/dccl/dccl.hpp:243-244)
 *   dccl_all_gather       ncclAllGather       (/root/reference/include/dccl/dccl.hpp:392-393)
 *   dccl_reduce           ncclReduce          (/root/reference/include/dccl/dccl.hpp:346-347)
 *   dccl_broadcast        ncclBroadcast       (/root/reference/include/dccl/dccl.hpp:289-290)
 * A null / finalized communicator returns ncclInvalidArgument (4) instead of throwing.
 */
#ifndef DCCL_COMM_H_
#define DCCL_COMM_H_
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* returns 0 on success, else an ncclResult_t value (the collective returns it) */
typedef int (*dccl_p2p_exchange_fn)(void* ctx, const void* sendbuf, size_t send_bytes, uint32_t to, void* recvbuf,
                                    size_t recv_bytes, uint32_t from, void* stream);
int dccl_comm_init_rank(void** comm, uint32_t world, uint32_t rank);
int dccl_get_unique_id(void* unique_id_128);
int dccl_comm_init_rccl(void** comm, uint32_t world, uint32_t rank, const void* unique_id_128);
int dccl_comm_init_ipc(void** comm, uint32_t world, uint32_t rank);
int dccl_comm_init_p2p(void** comm, uint32_t world, uint32_t rank, dccl_p2p_exchange_fn exchange, void* ctx,
                       int memory);
int dccl_bootstrap_unique_id(uint32_t rank, uint32_t world, void* unique_id_128);
int dccl_bootstrap_done(uint32_t rank, uint32_t world);
int dccl_comm_finalize(void* comm);
int dccl_all_reduce(const void* send, void* recv, size_t count, int dtype, int op, void* comm, void* stream);
int dccl_reduce_scatter(const void* send, void* recv, size_t recvcount, int dtype, int op, void* comm,
                        void* stream);
int dccl_all_gather(const void* send, void* recv, size_t sendcount, int dtype, void* comm, void* stream);
int dccl_reduce(const void* send, void* recv, size_t count, int dtype, int op, int root, void* comm,
                void* stream);
int dccl_broadcast(const void* send, void* recv, size_t count, int dtype, int root, void* comm, void* stream);
int dccl_rccl_available(void);
int dccl_comm_register(void* comm, void* buffer, size_t size);
int dccl_comm_deregister(void* comm, void* buffer);
int dccl_ipc_stats(uint64_t* out, int n);
#ifdef __cplusplus
}
#endif
#endif
