/*
 * tools/tune/dccl_reduce_tuning.h — benchmark/tuning hook, NOT part of the drop-in boundary:
 * built into tools/lib/libdccl_amd_tune.so, never into the product library libdccl_amd.so.  Launches the fp32 Sum combine with an explicit kernel variant so the
 * tuner (tools/tune_reduce.py) can A/B variants in one process on MI355X.
 *
 * A variant is (block threads, unroll = 16-B vectors per thread per operand in flight,
 * policy bits: 1 = non-temporal send loads, 2 = non-temporal recv loads, 4 = non-temporal
 * recv stores, xcd = XCD-contiguous block remap); grid_cap 0 = one block per tile,
 * else a persistent grid of at most grid_cap blocks striding over the tiles.
 */
#ifndef DCCL_REDUCE_TUNING_H_
#define DCCL_REDUCE_TUNING_H_
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif
int dccl_tune_num_variants(void);
int dccl_tune_variant_info(int variant, int* block, int* unroll, int* policy, int* xcd);
/* One-wave blocks, one vector per lane, cache bits in inline asm; flavor 0-6 (see tune_kernels.hip). */
int dccl_tune_asm_f32_sum(const void* send, void* recv, size_t count, int flavor, void* stream);
int dccl_tune_reduce_f32_sum(const void* send, void* recv, size_t count, int variant, size_t grid_cap,
                             void* stream);
/* Same, with `lds_bytes` of (unused) dynamic LDS per block to cap waves per CU. */
int dccl_tune_reduce_f32_sum_lds(const void* send, void* recv, size_t count, int variant, size_t grid_cap,
                                 size_t lds_bytes, void* stream);
/* Block of `waves` one-wave tiles; each wave pairs recv tile w with send tile (w+skew)%waves,
 * exchanging send through LDS (tests address-pair decorrelation). */
int dccl_tune_skew_f32_sum(const void* send, void* recv, size_t count, int waves, int skew, void* stream);
/* k-way fp32 Sum (the dccl_local_reduce_multi kernel) in shape `variant` 0-7 (see tune_kernels.hip),
 * with `lds_bytes` (<= 64 KiB) of unused dynamic LDS per block to cap resident blocks per CU. */
/* the in-phase chain kernel (dccl_local_reduce_chain) with `lds_bytes` of unused LDS per one-wave block */
int dccl_tune_chain_f32_sum(const void* const* sends, int nsend, const void* own, void* dst, size_t count,
                            size_t lds_bytes, void* stream);
/* the misaligned-recv combine in shape `variant` 0-9 (see tune_kernels.hip) */
int dccl_tune_group_f32_sum(const void* send, void* recv, size_t count, size_t lds_bytes, void* stream);
int dccl_tune_misaligned_f32_sum(const void* send, void* recv, size_t count, int variant, void* stream);
int dccl_tune_multi_f32_sum(const void* const* sends, int nsend, void* recv, size_t count, int variant,
                            size_t lds_bytes, void* stream);
/* HBM ceiling probes (see tune_kernels.hip): kind 0 read send, 1 read send+recv, 2 write recv,
 * 3 copy send->recv, 4 the fp32 Sum combine, all in the shipped shape; 5 read send+recv and
 * 6 write recv in 256-thread x 4-vector blocks; 7 empty workgroups on the shipped grid;
 * 8 the combine with the recv load issued first.
 * count_f32 % 4096 == 0, 16-B aligned operands. */
int dccl_tune_ceiling(int kind, const void* send, void* recv, size_t count_f32, void* stream);
/* Write-only streaming probe: variant -> (block, vectors per lane, store policy 0 plain / 1 nt / 2 sc1);
 * stream == (void*)~0 only reports the shape.  count_f32 % 32768 == 0. */
// The shifted kernel for operands with different 16-B phases (fp32 Sum; both element-aligned, phases
// different), by cache policy bits (1 send, 2 recv, 4 store, 8 lane 63's extra send load) and block order.
int dccl_tune_shift_num_variants(void);
int dccl_tune_shift_f32_sum(const void* send, void* recv, size_t count, int variant, int* policy, int* xcd,
                            void* stream);
/* Persistent one-wave blocks with a software pipeline (loads of `depth` tiles ahead in flight), fp32 Sum,
 * 16-B aligned operands, count a multiple of 256, `grid` blocks. */
int dccl_tune_pipelined_f32_sum(const void* send, void* recv, size_t count, int depth, size_t grid, void* stream);
int dccl_tune_write_num_variants(void);
int dccl_tune_write_probe(int variant, void* recv, size_t count_f32, int* block, int* unroll, int* policy,
                          void* stream);
/* the phased k-way combine (k = 1-8) in shape `variant` 0-4 (see tune_kernels.hip) */
int dccl_tune_phased_f32_sum(const void* const* sends, int nsend, void* recv, size_t count, int variant,
                             size_t lds_bytes, void* stream);

/* the phased chain combine (k = 1-5, 7) with the XCD tile order on (xcd 1) or off */
int dccl_tune_chain_phased_f32_sum(const void* const* sends, int nsend, const void* own, void* dst, size_t count,
                                   int xcd, void* stream);

/* the phased k-way combine (k = 1, 2, 4, 7) walking U tiles per wave: variant = 3 * order + log2(U) */
int dccl_tune_phased_walk_f32_sum(const void* const* sends, int nsend, void* recv, size_t count, int variant,
                                  void* stream);

/* the chain kernel with cache policy 7 (all non-temporal) or 6 (sources cached) and an explicit wave cap */
int dccl_tune_chain_policy_f32_sum(const void* const* sends, int nsend, const void* own, void* dst, size_t count,
                                   size_t lds_bytes, int policy, void* stream);

/* the shipped phased k-way (own NULL) / chain kernels: loads-first form, XCD order and wave cap chosen at run time */
int dccl_tune_phased_prod_f32_sum(const void* const* sends, int nsend, const void* own, void* dst, size_t count,
                                  int first, int xcd, size_t lds_bytes, void* stream);

/* the shipped shifted-kernel dispatch under an explicit wave cap (lds_bytes of unused LDS per block) */
int dccl_tune_shift_caps_f32_sum(const void* send, void* recv, size_t count, size_t lds_bytes, void* stream);

/* the unaligned k-way (own NULL) / chain kernels called directly on any operands, under a wave cap; form bit 0:
 * the loads-first form, form >> 1: the tile order (0 XCD-contiguous, 1 block order, 2 group-interleaved) */
int dccl_tune_unaligned_kway_f32_sum(const void* const* sends, int nsend, const void* own, void* dst, size_t count,
                                     size_t lds_bytes, int form, void* stream);
/* the pairwise misaligned-recv kernel under a wave cap and tile order */
int dccl_tune_unaligned_pair_f32_sum(const void* send, void* recv, size_t count, size_t lds_bytes, int order,
                                     void* stream);

/* the phased k-way combine (sources at other 16-B phases) in the tile-run orders (run 1 = block order) */
int dccl_tune_phased_run_f32_sum(const void* const* sends, int nsend, void* recv, size_t count, size_t lds_bytes,
                                 int first, unsigned run, void* stream);
/* the product's straddling / phased k-way (kind 0 / 2) and chain (1 / 3) kernels in tile-run orders 1, 2, 4 */
int dccl_tune_runs_f32_sum(int kind, const void* const* sends, int nsend, const void* own, void* dst, size_t count,
                           size_t lds_bytes, int run, int first, void* stream);
/* the pairwise launches (aligned, send off its lines, send at another 16-B phase or byte offset) in tile runs */
int dccl_tune_pair_run_f32_sum(const void* send, void* recv, size_t count, size_t lds_bytes, int run, void* stream);
/* the persistent work-queue combine (fp32 Sum, aligned): variant = tiles per grab (1-32) or 100 + grab for the
 * pipelined form; waves_per_cu one-wave blocks per CU; counter = two zeroed 64-bit words (reset by the kernel) */
int dccl_tune_wq_f32_sum(const void* send, void* recv, size_t count, int variant, int waves_per_cu, void* counter,
                         void* stream);

#ifdef __cplusplus
}
#endif
#endif
