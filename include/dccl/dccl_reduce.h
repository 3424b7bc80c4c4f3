/*
 * include/dccl/dccl_reduce.h — the C-ABI drop-in boundary of the DCCL local
 * bucket-reduction combine on MI355X (gfx950).
 *
 * Every entry point is `extern "C"`, takes plain pointers, sizes and integer
 * enum values (numerically identical to dccl::ncclDataType_t / ncclRedOp_t /
 * ncclResult_t of include/dccl/dccl.hpp and of the reference's
 * /root/reference/include/dccl/dccl.hpp:59-112), and never throws.
 *
 * Semantics: recv[i] = op(recv[i], send[i]) for
 * i in [0, count).  Sum/Prod wrap for integers, Max/Min are compare-and-select
 * (`if (r < s) r = s` / `if (r > s) r = s`: NaN or +-0 ties keep recv),
 * fp16/bf16 widen to fp32 and round back to nearest-even.  Avg returns
 * ncclInvalidUsage (5), any other op or an unknown dtype ncclInvalidArgument (4),
 * a HIP failure ncclUnhandledCudaError (1).  count == 0 is a successful no-op.
 *
 * Aliasing (SURVEY.md §8(b) "Ownership"), the same rule at every combine entry point below:
 *   - an operand may BE the destination (send == recv; a k-way source == recv; a chain source or
 *     own == dst): every combine is element-wise, so each output depends only on its own index;
 *   - an operand whose count*sizeof(dtype) bytes PARTIALLY overlap the destination's (shared bytes,
 *     different start) returns ncclInvalidArgument (4) before anything is launched.  The reference's
 *     one-thread ascending loop (/root/reference/src/core/internal_common.hpp:550-560) gives such a call
 *     an order-dependent answer that no parallel kernel reproduces.
 *   Sources may overlap each other freely (they are only read).  dccl_copy_multi: a pair's dst may equal
 *   its own src; no dst may share a byte with another pair's src or dst.
 */
#ifndef DCCL_REDUCE_H_
#define DCCL_REDUCE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Result codes (ncclResult_t values). */
#define DCCL_SUCCESS 0
#define DCCL_UNHANDLED_DEVICE_ERROR 1
#define DCCL_SYSTEM_ERROR 2
#define DCCL_INTERNAL_ERROR 3
#define DCCL_INVALID_ARGUMENT 4
#define DCCL_INVALID_USAGE 5

/*
 * Device combine, asynchronous and stream-ordered.
 *
 * Replaces the reference's GPU boundary
 *   dccl::do_device_reduce(const void*, void*, ncclDataType_t, size_t,
 *                          ncclRedOp_t, cudaStream_t)
 *   (/root/reference/src/core/internal_common.hpp:613-618, definition
 *    /root/reference/src/core/reduce.cu:40-100)
 * and its template shim do_device_reduce<DT>
 *   (/root/reference/src/core/internal_common.hpp:644-691).
 *
 * `send` and `recv` are device pointers of the device that owns `stream`
 * (a hipStream_t; NULL = that device's null stream).  Returns after the kernel
 * is enqueued; errors of the launch itself are reported, not asynchronous faults.
 */
int dccl_local_reduce(const void* send, void* recv, int dtype, size_t count, int op, void* stream);

/*
 * k-way device combine: recv[i] = op(...op(op(recv[i], sends[0][i]), sends[1][i])..., sends[k-1][i]),
 * applied in that order, one read of recv and one write.  Bit-identical to k
 * successive dccl_local_reduce calls (same association order).  1 <= nsend <= 8.
 * Serves the multi-arrival callers: recursive halving
 *   (/root/reference/src/core/reduce_scatter_recursive_halving.cpp:66-111) and the
 * Rabenseifner fold (/root/reference/src/core/all_reduce_recursive_halving_and_doubling.cpp:72-151).
 */
int dccl_local_reduce_multi(const void* const* sends, int nsend, void* recv, int dtype, size_t count,
                            int op, void* stream);

/*
 * Chain combine: the whole combine sequence of the ring reduce-scatter for one chunk, in one pass:
 *   dst[i] = op(own[i], op(sends[k-1][i], ... op(sends[1][i], sends[0][i])))
 * Each step is op(recv = next rank's data, send = partial so far), exactly as the ring applies it
 * (/root/reference/src/core/reduce_scatter_ring.cpp:73-101: rank c+j combines its own chunk c with
 * the partial received from rank c+j-1), so the result is bit-identical to W-1 ring steps when
 * sends[j] is rank c+j's chunk and `own` is the last rank's.  `own` may equal `dst`.
 * 1 <= nsend <= 8.  Used by the direct (xGMI peer-read) collectives, DESIGN.md §7.3.
 */
int dccl_local_reduce_chain(const void* const* sends, int nsend, const void* own, void* dst, int dtype,
                            size_t count, int op, void* stream);

/*
 * Multi-source device copy: dsts[y][0..bytes) = srcs[y][0..bytes) for y < npairs (<= 8), in one
 * launch, so the reads of several peers' chunks use several xGMI links at once (the all-gather
 * half of the direct collectives; replaces W-1 ring all-gather steps,
 * /root/reference/src/core/all_gather_ring.cpp:44-64).
 */
int dccl_copy_multi(const void* const* srcs, void* const* dsts, int npairs, size_t bytes, void* stream);

/*
 * Host combine, synchronous: `send` and `recv` are host pointers (the RDMA
 * receive buffers of the reference's host path).  Replaces the reference's CPU
 * boundary do_host_reduce<DT>
 *   (/root/reference/src/core/internal_common.hpp:496-586),
 * called by the ring reduce-scatter at /root/reference/src/core/reduce_scatter_ring.cpp:91-94.
 * The combine runs on the calling thread's current HIP device: chunks are staged
 * through pinned buffers in a copy/compute pipeline (H2D || combine || D2H).
 * Pointers registered with dccl_register_host_memory() are DMA'd directly.
 */
int dccl_local_reduce_host(const void* send, void* recv, int dtype, size_t count, int op);

/*
 * Host chain combine, synchronous: dccl_local_reduce_chain on host pointers (the direct all_reduce of
 * in-process ranks on host buffers).  Operands are staged through pinned memory and
 * combined by zero-copy kernels on the calling thread's current HIP device, in pieces whose staging
 * overlaps the previous piece's kernel; registered operands are read in place.
 */
int dccl_local_reduce_chain_host(const void* const* sends, int nsend, const void* own, void* dst, int dtype,
                                 size_t count, int op);

/*
 * Routing hint for host-resident chunks: the payload size (bytes per operand) from which
 * dccl_local_reduce_host beats the reference's own one-thread CPU loop do_host_reduce<DT>
 * (/root/reference/src/core/internal_common.hpp:496-586) on MI355X, measured by bench.py's
 * `host_crossover` leg on buffers registered with dccl_register_host_memory against one core on the
 * buffers' NUMA node.  A caller keeps do_host_reduce below it; pageable
 * chunks never beat that loop.  0 for dtypes the reference's host loop cannot combine (bf16; fp16 has host
 * operators only in CUDA builds), an unknown dtype included: the GPU path is then the only one.
 * DCCL_HOST_GPU_MIN_BYTES overrides the measured value for every dtype the reference's loop supports.  This
 * is advice for the caller: the library itself never combines on the CPU.
 */
size_t dccl_host_reduce_gpu_min_bytes(int dtype);

/* Page-lock a host range for direct DMA by dccl_local_reduce_host
 * (the role of dcclRegisterCacheMemory, /root/reference/src/core/dccl.cpp:503-549). */
int dccl_register_host_memory(void* buffer, size_t size);
int dccl_deregister_host_memory(void* buffer);

/* Size in bytes of a dtype, 0 if unknown (size_of_type, internal_common.hpp:314-335,
 * with bf16 always present). */
size_t dccl_size_of_type(int dtype);

/* Human-readable result string. */
const char* dccl_result_string(int result);

/* Library version, major*10000 + minor*100 + patch. */
int dccl_version(void);

#ifdef __cplusplus
}
#endif

#endif /* DCCL_REDUCE_H_ */
