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

namespace dccl_amd {

namespace {
inline uint32_t mod(int64_t a, uint32_t w) { return static_cast<uint32_t>(((a % w) + w) % w); }

// Take the acknowledgements of `posted` sends to `peer` (every posted message is acknowledged, even
// after a failed step, so the channel stays in step); the first error wins.
ncclResult_t collect_acks(dccl::dcclComm* c, uint32_t peer, uint32_t posted, bool device, hipStream_t st,
                          ncclResult_t rc) {
    for (uint32_t i = 0; i < posted; ++i) {
        const ncclResult_t rw = xport_wait_send(c, peer, device, st);
        if (rc == dccl::ncclSuccess) rc = rw;
    }
    return rc;
}
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
    if (c->p2p != nullptr) {  // cross-process (RCCL or a plugged-in transport): into the scratchpad, then combine
        ncclResult_t rc = ensure_scratch(c, slot_bytes, device);
        void* pad = device ? c->dev_scratch : c->host_scratch;
        for (uint32_t s = 0; s + 1 < W && rc == dccl::ncclSuccess; ++s) {
            rc = p2p_exchange(c, data(int64_t(r) - s), slot_bytes, to, pad, slot_bytes, from, st);
            if (rc == dccl::ncclSuccess) rc = combine(pad, data(int64_t(r) - s - 1), dtype, slot_elems, op, device, st);
        }
        return rc;
    }
    // A chunk this rank sends at step s (slot r-s) is never written again by this rank during the
    // reduce-scatter (it writes slots r-1 ... r+1, each before sending it), so the acknowledgements
    // are collected once, after the last step, instead of after every step: a step's critical path
    // then holds one cross-stream hand-off (the peer's chunk is ready) instead of two.
    ncclResult_t rc = dccl::ncclSuccess;
    uint32_t posted = 0;
    for (uint32_t s = 0; s + 1 < W && rc == dccl::ncclSuccess; ++s) {
        rc = xport_send(c, to, data(int64_t(r) - s), slot_bytes, device, st);
        if (rc != dccl::ncclSuccess) break;
        ++posted;
        if (scratch != nullptr) {  // reference shape: land in the scratchpad, then combine
            rc = xport_recv(c, from, scratch, slot_bytes, device, st);
            if (rc == dccl::ncclSuccess)
                rc = combine(scratch, data(int64_t(r) - s - 1), dtype, slot_elems, op, device, st);
        } else {  // fused: combine straight from the peer's chunk
            rc = xport_recv_combine(c, from, data(int64_t(r) - s - 1), slot_elems, dtype, op, device, st);
        }
    }
    return collect_acks(c, to, posted, device, st, rc);
}

ncclResult_t all_gather_ring(dccl::dcclComm* c, void* buffer, size_t slot_elems, int dtype, bool device,
                             hipStream_t st, const RankMap& to_new, const RankMap& to_old) {
    const uint32_t W = c->world;
    const size_t slot_bytes = slot_elems * size_of_dtype(dtype);
    const uint32_t r = to_new(c->rank);
    auto data = [&](int64_t i) { return static_cast<unsigned char*>(buffer) + slot_bytes * mod(i, W); };
    const uint32_t to = to_old(mod(int64_t(r) + 1, W)), from = to_old(mod(int64_t(r) - 1, W));
    if (c->p2p != nullptr) {
        for (uint32_t s = 0; s + 1 < W; ++s) {
            const ncclResult_t rc =
                p2p_exchange(c, data(int64_t(r) - s), slot_bytes, to, data(int64_t(r) - s - 1), slot_bytes, from, st);
            if (rc != dccl::ncclSuccess) return rc;
        }
        return dccl::ncclSuccess;
    }
    // As in the reduce-scatter, a slot is written (received) once and only then forwarded, so the
    // acknowledgements are collected after the last step.
    ncclResult_t rc = dccl::ncclSuccess;
    uint32_t posted = 0;
    for (uint32_t s = 0; s + 1 < W && rc == dccl::ncclSuccess; ++s) {
        rc = xport_send(c, to, data(int64_t(r) - s), slot_bytes, device, st);
        if (rc != dccl::ncclSuccess) break;
        ++posted;
        rc = xport_recv(c, from, data(int64_t(r) - s - 1), slot_bytes, device, st);
    }
    return collect_acks(c, to, posted, device, st, rc);
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

// ------------------------------------------------------------------------------------------
// Rabenseifner all-reduce (DCCL_ALLREDUCE_ALGORITHM=rabenseifner):
//   /root/reference/src/core/all_reduce_recursive_halving_and_doubling.cpp:8-201
//   /root/reference/src/core/reduce_scatter_recursive_halving.cpp:12-116
//   /root/reference/src/core/all_gather_recursive_doubling.cpp:12-92
// Same fold of a non-power-of-two world onto 2^k ranks, same halving order and the same
// op(recv = own part, send = peer's part) at every step, so every reduced block is bit-identical to
// the reference's.  One deliberate fix: the reference's recursive-doubling all-gather sends one slice
// per step (its step_bsize doubling sits inside a comment, all_gather_recursive_doubling.cpp:85), so
// with a subworld of 4 or more ranks some blocks never arrive; here step s moves 2^s slices and every
// rank ends with the whole result.
// ------------------------------------------------------------------------------------------
namespace {

inline uint32_t floor_log2(uint32_t n) {
    uint32_t k = 0;
    while ((n >> (k + 1)) != 0) ++k;
    return k;
}

inline uint32_t reverse_low_bits(uint32_t x, uint32_t nbits) {
    uint32_t r = 0;
    for (uint32_t b = 0; b < nbits; ++b) r = (r << 1) | ((x >> b) & 1u);
    return r;
}

// Send [sbuf, sbytes) to `peer` (skipped if sbuf is null) and receive `rbytes` from it into rbuf
// (skipped if rbuf is null).
ncclResult_t swap(dccl::dcclComm* c, uint32_t peer, const void* sbuf, size_t sbytes, void* rbuf, size_t rbytes,
                  bool device, hipStream_t st) {
    if (c->p2p != nullptr) return p2p_exchange(c, sbuf, sbytes, peer, rbuf, rbytes, peer, st);
    ncclResult_t rc = dccl::ncclSuccess;
    if (sbuf != nullptr) rc = xport_send(c, peer, sbuf, sbytes, device, st);
    if (rc == dccl::ncclSuccess && rbuf != nullptr) rc = xport_recv(c, peer, rbuf, rbytes, device, st);
    if (sbuf != nullptr) {
        const ncclResult_t rw = xport_wait_send(c, peer, device, st);
        if (rc == dccl::ncclSuccess) rc = rw;
    }
    return rc;
}

// Send [sbuf, elems) to `peer` and combine what it sends into dst: dst = op(dst, peer's part).
ncclResult_t swap_combine(dccl::dcclComm* c, uint32_t peer, const void* sbuf, void* dst, size_t elems, int dtype,
                          int op, void* scratch, bool device, hipStream_t st) {
    const size_t bytes = elems * size_of_dtype(dtype);
    if (c->p2p != nullptr) {
        ncclResult_t rc = ensure_scratch(c, bytes, device);
        void* pad = device ? c->dev_scratch : c->host_scratch;
        if (rc == dccl::ncclSuccess) rc = p2p_exchange(c, sbuf, bytes, peer, pad, bytes, peer, st);
        return rc == dccl::ncclSuccess ? combine(pad, dst, dtype, elems, op, device, st) : rc;
    }
    ncclResult_t rc = xport_send(c, peer, sbuf, bytes, device, st);
    if (rc == dccl::ncclSuccess) {
        if (scratch != nullptr) {  // the reference's shape: land in the scratchpad, then combine
            rc = xport_recv(c, peer, scratch, bytes, device, st);
            if (rc == dccl::ncclSuccess) rc = combine(scratch, dst, dtype, elems, op, device, st);
        } else {
            rc = xport_recv_combine(c, peer, dst, elems, dtype, op, device, st);
        }
    }
    const ncclResult_t rw = xport_wait_send(c, peer, device, st);
    return rc == dccl::ncclSuccess ? rw : rc;
}

}  // namespace

ncclResult_t all_reduce_rabenseifner(dccl::dcclComm* c, void* buffer, void* scratch, size_t count, int dtype, int op,
                                     bool device, hipStream_t st) {
    const uint32_t W = c->world, me = c->rank;
    const uint32_t k = floor_log2(W), sub = 1u << k, rem = W - sub;
    if (count % sub) return dccl::ncclInvalidArgument;  // all_reduce_recursive_halving_and_doubling.cpp:50-54
    if (W == 1) return dccl::ncclSuccess;
    const size_t esz = size_of_dtype(dtype), total = count * esz, half = total / 2;
    auto* base = static_cast<unsigned char*>(buffer);
    // fold: ranks below 2*rem pair up as (leader 2i, follower 2i+1) -> new rank i; the rest shift down
    auto to_new = [rem](uint32_t o) { return o < 2 * rem ? o / 2 : o - rem; };
    auto to_old = [rem](uint32_t n) { return n < rem ? n * 2 : n + rem; };
    const bool leader = me < 2 * rem && me % 2 == 0, follower = me < 2 * rem && me % 2 == 1;
    ncclResult_t rc = dccl::ncclSuccess;
    if (leader) {  // keep the first half: first = op(mine, follower's); get the second half back reduced
        rc = swap_combine(c, me + 1, base + half, base, count / 2, dtype, op, scratch, device, st);
        if (rc == dccl::ncclSuccess) rc = swap(c, me + 1, nullptr, 0, base + half, half, device, st);
    } else if (follower) {  // reduce the second half: second = op(mine, leader's); hand it to the leader
        rc = swap_combine(c, me - 1, base, base + half, count / 2, dtype, op, scratch, device, st);
        if (rc == dccl::ncclSuccess) rc = swap(c, me - 1, base + half, half, nullptr, 0, device, st);
    }
    if (rc != dccl::ncclSuccess) return rc;
    if (!follower) {
        const uint32_t my = to_new(me);
        // recursive halving reduce-scatter (reduce_scatter_recursive_halving.cpp:68-110)
        unsigned char* region = base;
        size_t bytes = total;
        for (uint32_t s = 0; s < k && rc == dccl::ncclSuccess; ++s) {
            const uint32_t peer = to_old(my ^ (1u << s));
            bytes /= 2;
            unsigned char* keep = ((my >> s) & 1u) ? region + bytes : region;
            unsigned char* give = ((my >> s) & 1u) ? region : region + bytes;
            rc = swap_combine(c, peer, give, keep, bytes / esz, dtype, op, scratch, device, st);
            region = keep;
        }
        // recursive doubling all-gather (all_gather_recursive_doubling.cpp:48-76), 2^s slices at step s
        const size_t slice = total / sub;
        uint32_t block = reverse_low_bits(my, k);
        for (uint32_t s = 0; s < k && rc == dccl::ncclSuccess; ++s) {
            const uint32_t peer = to_old(my ^ (1u << (k - s - 1)));
            block &= ~((1u << s) - 1u);
            const uint32_t rblock = block ^ (1u << s);
            const size_t len = slice << s;
            rc = swap(c, peer, base + size_t(block) * slice, len, base + size_t(rblock) * slice, len, device, st);
        }
    }
    if (rc != dccl::ncclSuccess) return rc;
    if (leader) return swap(c, me + 1, base, total, nullptr, 0, device, st);  // :182-188
    if (follower) return swap(c, me - 1, nullptr, 0, base, total, device, st);  // :189-195
    return dccl::ncclSuccess;
}

}  // namespace dccl_amd
