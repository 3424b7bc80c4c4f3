// include/dccl/dccl.hpp — NCCL-compatible DCCL surface of the MI355X build.
//
// Source-compatible with the reference's public header (/root/reference/include/dccl/dccl.hpp):
// same namespace (dccl), C++ linkage, same enum names and values (results 0-8, dtypes 0-9,
// ops 0-5; :59-112) and the same function names and argument meaning.  Differences, all
// deliberate and documented in INTEGRATION.md:
//   * the stream parameter is a hipStream_t (the reference's is cudaStream_t, :11-22);
//     nullptr still means "host buffers" (:188-201);
//   * ncclBfloat16 = 9 is always present (the reference gates it on CUDA bf16, :81-86);
//   * ncclCommInit joins an in-process group (one communicator per thread, rank = join
//     order, world size from DCCL_WORLD_SIZE) instead of a Derecho subgroup; the transport
//     between ranks is host memcpy / device-to-device (xGMI peer) copies, stream-ordered.
//     dcclCommInitRank() picks the rank explicitly.
// The element-wise combine behind ncclAllReduce / ncclReduceScatter is the gfx950 HIP kernel
// of include/dccl/dccl_reduce.h.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

/** Option key (environment variable here, derecho.cfg in the reference, dccl.hpp:38). */
#define DCCL_ALLREDUCE_ALGORITHM_CONFSTR "DCCL_ALLREDUCE_ALGORITHM"
#define DCCL_ALLREDUCE_RING "ring"
#define DCCL_ALLREDUCE_RABENSEIFNER "rabenseifner"

namespace dccl {

typedef enum {
    ncclSuccess = 0,
    ncclUnhandledCudaError = 1,  // a HIP runtime failure on this build
    ncclSystemError = 2,
    ncclInternalError = 3,
    ncclInvalidArgument = 4,
    ncclInvalidUsage = 5,
    ncclRemoteError = 6,
    ncclInProgress = 7,
    ncclNumResults = 8
} ncclResult_t;

typedef enum {
    ncclInt8 = 0, ncclChar = 0,
    ncclUint8 = 1,
    ncclInt32 = 2, ncclInt = 2,
    ncclUint32 = 3,
    ncclInt64 = 4,
    ncclUint64 = 5,
    ncclFloat16 = 6, ncclHalf = 6,
    ncclFloat32 = 7, ncclFloat = 7,
    ncclFloat64 = 8, ncclDouble = 8,
    ncclBfloat16 = 9,
    ncclNumTypes = 10
} ncclDataType_t;

typedef enum { ncclNumOps_dummy = 5 } ncclRedOp_dummy_t;

typedef enum {
    ncclSum = 0,
    ncclProd = 1,
    ncclMax = 2,
    ncclMin = 3,
    ncclAvg = 4,
    ncclNumOps = 5,
    ncclMaxRedOp = 0x7fffffff >> (32 - 8 * sizeof(ncclRedOp_dummy_t))
} ncclRedOp_t;

struct dcclComm;
typedef struct dcclComm* ncclComm_t;

/** Join the process's DCCL group; blocks until DCCL_WORLD_SIZE (default 1) ranks joined. */
ncclResult_t ncclCommInit(ncclComm_t* comm);
/** MI355X-build extension: join the process's group at an explicit rank. */
ncclResult_t dcclCommInitRank(ncclComm_t* comm, uint32_t world_size, uint32_t rank);
/** MI355X-build extension: cross-process communicator on the RCCL (xGMI) transport, one process
 *  per GPU (the current HIP device).  `unique_id` is 128 bytes from dcclGetUniqueId on one rank.
 *  ncclCommInit selects this transport itself when DCCL_TRANSPORT=rccl (rank/world from
 *  RANK/WORLD_SIZE, id exchanged through a file in DCCL_BOOTSTRAP_DIR). Device buffers only. */
ncclResult_t dcclGetUniqueId(void* unique_id);
ncclResult_t dcclCommInitRccl(ncclComm_t* comm, uint32_t world_size, uint32_t rank, const void* unique_id);
/** MI355X-build extension: cross-process communicator on the IPC peer-read transport, one process
 *  per GPU of one node (the current HIP device).  Collectives read peers' buffers directly over
 *  xGMI.  ncclCommInit selects it when DCCL_TRANSPORT=ipc (rank/world from
 *  RANK/WORLD_SIZE, rendezvous through DCCL_BOOTSTRAP_DIR).  Device buffers only, world <= 8
 *  for the collectives, no ncclSend/ncclRecv. */
ncclResult_t dcclCommInitIpc(ncclComm_t* comm, uint32_t world_size, uint32_t rank);
ncclResult_t ncclCommFinalize(ncclComm_t comm);

/** Page-lock host memory for direct DMA.  Device memory: validated (on an IPC communicator: a device
 *  allocation of this process, the range inside it) and tracked; peers read every input through the
 *  communicator's scratch, never user memory. */
ncclResult_t dcclRegisterCacheMemory(ncclComm_t comm, void* buffer, size_t size);
ncclResult_t dcclDeregisterCacheMemory(ncclComm_t comm, void* buffer, size_t size = 0UL);

ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                           ncclRedOp_t op, ncclComm_t comm, hipStream_t stream);
ncclResult_t ncclReduceScatter(const void* sendbuff, void* recvbuff, size_t recvcount,
                               ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm, hipStream_t stream);
ncclResult_t ncclBroadcast(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype, int root,
                           ncclComm_t comm, hipStream_t stream);
ncclResult_t ncclBcast(void* buff, size_t count, ncclDataType_t datatype, int root, ncclComm_t comm,
                       hipStream_t stream);
ncclResult_t ncclReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                        ncclRedOp_t op, int root, ncclComm_t comm, hipStream_t stream);
ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t datatype,
                           ncclComm_t comm, hipStream_t stream);
ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream);
ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream);

uint32_t dcclGetWorldSize(ncclComm_t comm);
uint32_t dcclGetMyRank(ncclComm_t comm);

/** Host cache line used for the alignment advisories (CACHELINE_SIZE of the reference). */
constexpr size_t kCachelineSize = 64;
/** GPU line size for the device-side alignment advisories. */
constexpr size_t kDeviceCachelineSize = 128;

}  // namespace dccl
