/* include/dccl/dccl_synth.h — counter-based synthetic operands for the combine benchmarks.
 *
 * SURVEY.md §8(d) "Synthetic inputs": element i of buffer `buffer_id` is derived from
 *     x_i = splitmix64(seed ^ (buffer_id << 40) ^ i)
 * so any slice of a 1 GiB operand can be regenerated on the host (oracle/host_reduce.c,
 * oracle_synth_fill) and checked bit-exactly against what the GPU combined.  The reference has
 * no counterpart: its benchmarks memset by rank (src/application/cli.cpp:421-424).
 *
 * Value mapping (exact: no rounding anywhere, so host and device agree bit for bit):
 *   integer types             the low sizeof(T) bytes of x_i (full range: wrap is exercised)
 *   float, op != ncclProd     uniform on [-1, 1):  m * 2^-p with m = (x_i >> (64-p-1)) - 2^p,
 *                             p = 23 (fp32), 52 (fp64), 10 (fp16), 7 (bf16)
 *   float, op == ncclProd     [0.5, 2): random mantissa, exponent 2^-1 or 2^0 from the top bit
 *                             (repeated products stay finite)
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/** Fill `count` elements of `dtype` at device pointer `dst`, asynchronously on `hip_stream`.
 *  `op` selects the float value range (ncclProd vs the rest; any op value 0-4 is accepted).
 *  Returns DCCL_SUCCESS, DCCL_INVALID_ARGUMENT (dtype, NULL dst with count > 0) or
 *  DCCL_UNHANDLED_DEVICE_ERROR. */
int dccl_synth_fill(void* dst, int dtype, size_t count, int op, uint64_t seed, uint64_t buffer_id,
                    void* hip_stream);

/** Elements [first, first + count) of the same operand: a slice of a larger buffer, e.g. to rebuild
 *  the inputs of a sampled range of a combine for checking. */
int dccl_synth_fill_range(void* dst, int dtype, size_t count, int op, uint64_t seed, uint64_t buffer_id,
                          size_t first, void* hip_stream);

#ifdef __cplusplus
}
#endif
