/*
 * include/dccl/dccl_reduce_tuning.h — benchmark/tuning hook, NOT part of the drop-in
 * boundary.  Launches the fp32 Sum combine with an explicit kernel variant so the
 * tuner (tools/tune_reduce.py) can A/B variants in one process on MI355X.
 *
 *   unroll   : 16-B vectors per thread per operand in flight (1, 2, 4, 8)
 *   policy   : bit 0 = non-temporal send loads, bit 1 = non-temporal recv loads,
 *              bit 2 = non-temporal recv stores (allowed values 0, 1, 3, 5, 7)
 *   grid_cap : 0 = one block per tile (default shape), else a persistent grid of
 *              at most grid_cap blocks striding over the tiles.
 */
#ifndef DCCL_REDUCE_TUNING_H_
#define DCCL_REDUCE_TUNING_H_
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif
int dccl_tune_reduce_f32_sum(const void* send, void* recv, size_t count, int unroll, int policy,
                             size_t grid_cap, void* stream);
#ifdef __cplusplus
}
#endif
#endif
