// dccl_amd/csrc/grouped.cpp — the grouped reduce-scatter / all-reduce of the RCCL transport (algorithms.hpp).
// A translation unit of its own: the CPU harness of the ring's p2p branch (tests/native/ring_p2p_harness.cpp)
// links algorithms.cpp alone, and links this file with a fake grouped exchange and a CPU chain combine.
#include <vector>

#include "algorithms.hpp"
#include "dccl/dccl_reduce.h"
#include "rccl_transport.hpp"

namespace dccl_amd {

namespace {
inline uint32_t mod(int64_t a, uint32_t w) { return static_cast<uint32_t>(((a % w) + w) % w); }
}  // namespace

// Grouped reduce-scatter / all-reduce over RCCL.  The ring moves one chunk per step to one neighbour and
// combines it pairwise: W - 1 transfers on one xGMI link in turn and W - 1 launches of 3 * slot bytes each,
// at the mid-size ring-step shapes where a launch runs at 57-76 % of HBM peak.  Here the
// W - 1 contributions to this rank's slot travel in one RCCL group into W - 1 scratch slots, and one chain
// launch reads them with the rank's own slot ((W + 1) * slot bytes) in the ring's association order.
ncclResult_t reduce_scatter_grouped(dccl::dcclComm* c, const void* in, void* dst, size_t count, int dtype, int op,
                                    hipStream_t st, uint32_t shift) {
    const uint32_t W = c->world, r = c->rank;
    if (c->rccl == nullptr || W < 2) return dccl::ncclInvalidUsage;
    if (count < W || count % W) return dccl::ncclInvalidArgument;
    const size_t slot_elems = count / W, slot = slot_elems * size_of_dtype(dtype);
    ncclResult_t rc = ensure_scratch(c, (W - 1) * slot, true);
    if (rc != dccl::ncclSuccess) return rc;
    auto* base = static_cast<const unsigned char*>(in);
    auto* pad = static_cast<unsigned char*>(c->dev_scratch);
    std::vector<const void*> sends(W, nullptr);
    std::vector<void*> recvs(W, nullptr);
    for (uint32_t p = 0; p < W; ++p) {
        if (p == r) continue;
        sends[p] = base + size_t((p + shift) % W) * slot;            // this rank's part of the slot p owns
        recvs[p] = pad + size_t(mod(int64_t(p) - r - 1, W)) * slot;  // chain position of p's part
    }
    rc = static_cast<ncclResult_t>(rccl_exchange_all(c->rccl, sends.data(), recvs.data(), slot, W, r, st));
    if (rc != dccl::ncclSuccess) return rc;
    // the ring's order for the slot this rank owns: ranks r+1, r+2, ..., r-1, then this rank's own part
    std::vector<const void*> chain(W - 1);
    for (uint32_t j = 0; j + 1 < W; ++j) chain[j] = pad + size_t(j) * slot;
    return static_cast<ncclResult_t>(dccl_local_reduce_chain(chain.data(), int(W - 1),
                                                             base + size_t((r + shift) % W) * slot, dst, dtype,
                                                             slot_elems, op, static_cast<void*>(st)));
}

ncclResult_t all_reduce_grouped(dccl::dcclComm* c, const void* send, void* recv, size_t count, int dtype, int op,
                                hipStream_t st) {
    const uint32_t W = c->world, r = c->rank;
    const size_t slot = count / W * size_of_dtype(dtype);
    auto* out = static_cast<unsigned char*>(recv);
    // slot p + 1 lives on rank p (all_reduce_ring's ownership); no in-place copy: the sends read `send`
    ncclResult_t rc = reduce_scatter_grouped(c, send, out + size_t((r + 1) % W) * slot, count, dtype, op, st, 1);
    if (rc != dccl::ncclSuccess) return rc;
    std::vector<const void*> sends(W, nullptr);
    std::vector<void*> recvs(W, nullptr);
    for (uint32_t p = 0; p < W; ++p) {
        if (p == r) continue;
        sends[p] = out + size_t((r + 1) % W) * slot;
        recvs[p] = out + size_t((p + 1) % W) * slot;
    }
    return static_cast<ncclResult_t>(rccl_exchange_all(c->rccl, sends.data(), recvs.data(), slot, W, r, st));
}

}  // namespace dccl_amd
