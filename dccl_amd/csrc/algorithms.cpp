// dccl_amd/csrc/algorithms.cpp — ring collectives around the gfx950 combine.
//
// Choreography follows the reference:
//   reduce_scatter_ring  /root/reference/src/core/reduce_scatter_ring.cpp:8-106
//   all_gather_ring      /root/reference/src/core/all_gather_ring.cpp:8-69
//   all_reduce_ring      /root/reference/src/core/all_reduce_ring.cpp:8-79
// with the same chunk addressing (slot i of the buffer, indices taken mod W), the same rank
// maps, the same count % W == 0 constraint, and the same order of combines, so results are
// bit-identical to the reference's for every dtype (floating point included).  Two changes:
//   * device steps are stream-ordered end to end: no host stream synchronisation per step
//     (the reference syncs after every device combine, reduce_scatter_ring.cpp:88, and that
//     sync overwrites the combine's return code — SURVEY.md A.3 #5);
//   * by default the receive of a reduce-scatter step is fused with the combine: the combine reads
//     the peer's chunk in place (scratch == nullptr); DCCL_RS_SCRATCH=1 keeps the reference's
//     land-in-scratchpad-then-combine shape (same results, one extra write + read of the chunk);
//   * the send of a step is posted before its receive (the in-process transport's receive
//     blocks until the matching post exists; the reference posts recv first in the all-gather,
//     all_gather_ring.cpp:46-49, which is equivalent for a non-blocking RDMA post).
#include <functional>

#include "algorithms.hpp"
#include "rccl_transport.hpp"

namespace dccl_amd {

namespace {
inline uint32_t mod(int64_t a, uint32_t w) { return static_cast<uint32_t>(((a % w) + w) % w); }
}  // namespace

ncclResult_t reduce_scatter_ring(dccl::dcclComm* c, void* buffer, void* scratch, size_t count, int dtype, int op,
                                 bool device, hipStream_t st, const RankMap& to_new, const RankMap& to_old) {
    const uint32_t W = c->world;
    if (count < W || count % W) return dccl::ncclInvalidArgument;  // reduce_scatter_ring.cpp:53-58
    const size_t esz = size_of_dtype(dtype);
    const size_t slot_elems = count / W, slot_bytes = slot_elems * esz;
    const uint32_t r = to_new(c->rank);
    auto data = [&](int64_t i) { return static_cast<unsigned char*>(buffer) + slot_bytes * mod(i, W); };
    const uint32_t to = to_old(mod(int64_t(r) + 1, W)), from = to_old(mod(int64_t(r) - 1, W));
    if (c->rccl != nullptr) {  // cross-process: RCCL p2p into the scratchpad, then the combine
        ncclResult_t rc = ensure_scratch(c, slot_bytes, true);
        for (uint32_t s = 0; s + 1 < W && rc == dccl::ncclSuccess; ++s) {
            rc = static_cast<ncclResult_t>(rccl_exchange(c->rccl, data(int64_t(r) - s), slot_bytes, to,
                                                         c->dev_scratch, slot_bytes, from, st));
            if (rc == dccl::ncclSuccess)
                rc = combine(c->dev_scratch, data(int64_t(r) - s - 1), dtype, slot_elems, op, true, st);
        }
        return rc;
    }
    for (uint32_t s = 0; s + 1 < W; ++s) {
        ncclResult_t rc = xport_send(c, to, data(int64_t(r) - s), slot_bytes, device, st);
        if (rc == dccl::ncclSuccess) {
            if (scratch != nullptr) {  // reference shape: land in the scratchpad, then combine
                rc = xport_recv(c, from, scratch, slot_bytes, device, st);
                if (rc == dccl::ncclSuccess)
                    rc = combine(scratch, data(int64_t(r) - s - 1), dtype, slot_elems, op, device, st);
            } else {  // fused: combine straight from the peer's chunk
                rc = xport_recv_combine(c, from, data(int64_t(r) - s - 1), slot_elems, dtype, op, device, st);
            }
        }
        const ncclResult_t rw = xport_wait_send(c, to, device, st);
        if (rc == dccl::ncclSuccess) rc = rw;
        if (rc != dccl::ncclSuccess) return rc;
    }
    return dccl::ncclSuccess;
}

ncclResult_t all_gather_ring(dccl::dcclComm* c, void* buffer, size_t slot_elems, int dtype, bool device,
                             hipStream_t st, const RankMap& to_new, const RankMap& to_old) {
    const uint32_t W = c->world;
    const size_t slot_bytes = slot_elems * size_of_dtype(dtype);
    const uint32_t r = to_new(c->rank);
    auto data = [&](int64_t i) { return static_cast<unsigned char*>(buffer) + slot_bytes * mod(i, W); };
    const uint32_t to = to_old(mod(int64_t(r) + 1, W)), from = to_old(mod(int64_t(r) - 1, W));
    if (c->rccl != nullptr) {
        for (uint32_t s = 0; s + 1 < W; ++s) {
            const int rc = rccl_exchange(c->rccl, data(int64_t(r) - s), slot_bytes, to, data(int64_t(r) - s - 1),
                                         slot_bytes, from, st);
            if (rc != 0) return static_cast<ncclResult_t>(rc);
        }
        return dccl::ncclSuccess;
    }
    for (uint32_t s = 0; s + 1 < W; ++s) {
        ncclResult_t rc = xport_send(c, to, data(int64_t(r) - s), slot_bytes, device, st);
        if (rc == dccl::ncclSuccess) rc = xport_recv(c, from, data(int64_t(r) - s - 1), slot_bytes, device, st);
        const ncclResult_t rw = xport_wait_send(c, to, device, st);
        if (rc == dccl::ncclSuccess) rc = rw;
        if (rc != dccl::ncclSuccess) return rc;
    }
    return dccl::ncclSuccess;
}

ncclResult_t all_reduce_ring(dccl::dcclComm* c, void* buffer, void* scratch, size_t count, int dtype, int op,
                             bool device, hipStream_t st) {
    const uint32_t W = c->world;
    if (count < W || count % W) return dccl::ncclInvalidArgument;  // all_reduce_ring.cpp:51-55
    const RankMap id = [](uint32_t x) { return x; };
    ncclResult_t rc = reduce_scatter_ring(c, buffer, scratch, count, dtype, op, device, st, id, id);
    if (rc != dccl::ncclSuccess) return rc;
    // all_reduce_ring.cpp:70-72: new rank = r + 1, so rank r starts from the slot it reduced
    return all_gather_ring(c, buffer, count / W, dtype, device, st,
                           [W](uint32_t x) { return (x + 1) % W; },
                           [W](uint32_t x) { return (x + W - 1) % W; });
}

}  // namespace dccl_amd
