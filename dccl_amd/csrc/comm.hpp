// dccl_amd/csrc/comm.hpp — communicator and rank-to-rank transport of the MI355X build.
//
// The reference moves chunks between ranks with Derecho's out-of-band RDMA
// (dccl_oob_send / dccl_oob_recv / wait, /root/reference/src/core/internal_common.hpp:698-792):
// a send posts a buffer, the peer's recv lands it in the peer's buffer, and both sides wait.
// Here the ranks of a group are threads of one process (one per GPU on a node, or several
// on one GPU for tests) and the same four verbs are implemented as:
//   send(peer, buf)    post {buf, ready-event recorded on the sender's stream} to peer
//   recv(peer, dst)    take the matching post; device: the receiver's stream waits on the
//                      ready event and copies D2D (an xGMI peer copy across GPUs); host: memcpy;
//                      then acknowledge with a done-event
//   wait_send(peer)    take the acknowledgement; device: the sender's stream waits on the
//                      done event, so later writes to the buffer are ordered after the copy
//   wait_recv(peer)    nothing left to do: the copy is already stream-ordered
// No host-side stream synchronisation happens between ring steps (the reference syncs the
// stream after every device combine, reduce_scatter_ring.cpp:88 — SURVEY.md §8(f) row 2).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <vector>

#include "dccl/dccl.hpp"

namespace dccl_amd {

// Point-to-point transport of ranks in different processes: one exchange = send `send_bytes` from
// `sendbuf` to rank `to` and receive `recv_bytes` from rank `from` into `recvbuf` (either side skipped
// with a null buffer), ordered on `stream` for device buffers, complete on return for host buffers.
// RCCL's grouped ncclSend/ncclRecv over xGMI is one (rccl_transport.hpp); a host may plug in its own,
// e.g. Derecho's OOB send/recv (dccl_comm_init_p2p, include/dccl/dccl_comm.h).
using P2PExchangeFn = int (*)(void* ctx, const void* sendbuf, size_t send_bytes, uint32_t to, void* recvbuf,
                              size_t recv_bytes, uint32_t from, void* stream);

struct Message {
    const void* ptr = nullptr;
    size_t bytes = 0;
    bool device = false;
    hipEvent_t ready = nullptr;  // recorded on the sender's stream (device messages)
};

struct Ack {
    hipEvent_t done = nullptr;  // recorded on the receiver's stream after its copy
};

// One directed channel src -> dst: messages flow forward, acknowledgements back.
struct Channel {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Message> msgs;
    std::deque<Ack> acks;
};

class Group {
public:
    explicit Group(uint32_t world);
    uint32_t world() const { return world_; }
    Channel& channel(uint32_t src, uint32_t dst) { return *chan_[src * world_ + dst]; }
    // Rendezvous: blocks until every rank arrived (init / finalize / the direct collectives' phase
    // points).  It also agrees on success: returns true iff every rank arrived with ok == true, so a rank
    // whose step failed still meets the others and they all learn of it at the same point.
    bool barrier(bool ok = true);
    // HIP device of each rank (-1: none), filled at join; used to enable peer access.
    std::vector<int> devices;
    // Buffer addresses each rank publishes for the direct (peer-read) collectives, direct.cpp.
    std::vector<const void*> pub_in;
    std::vector<void*> pub_out;

    // join bookkeeping (guarded by the registry mutex)
    std::vector<bool> taken;
    uint32_t joined = 0;
    uint32_t left = 0;

private:
    uint32_t world_;
    std::vector<std::unique_ptr<Channel>> chan_;
    std::mutex bmu_;
    std::condition_variable bcv_;
    uint32_t barrier_count_ = 0;
    bool barrier_bad_ = false;           // some rank of the open generation arrived with ok == false
    bool barrier_ok_[2] = {true, true};  // outcome of each generation, indexed by its parity
    std::atomic<uint64_t> barrier_gen_{0};  // written under bmu_, polled without it
};

}  // namespace dccl_amd

// The opaque communicator of include/dccl/dccl.hpp.
struct dccl::dcclComm {
    std::shared_ptr<dccl_amd::Group> group;
    uint32_t rank = 0;
    uint32_t world = 1;
    int device = -1;  // HIP device current at init
    void* rccl = nullptr;  // the RCCL communicator this comm owns (DCCL_TRANSPORT=rccl), destroyed at finalize
    // Cross-process p2p transport (RCCL, or a plugged-in one): when set, the ring algorithms move chunks
    // with p2p(p2p_ctx, ...) instead of the in-process channels.
    dccl_amd::P2PExchangeFn p2p = nullptr;
    void* p2p_ctx = nullptr;
    bool p2p_host = false;    // the p2p transport moves host memory (RCCL: no)
    bool p2p_device = true;   // the p2p transport moves device memory (RCCL: yes)
    void* ipc = nullptr;   // non-null: cross-process IPC peer-read transport (direct.hpp), device buffers only
    // Events of the stream-ordered device transport: a ring of `event_ring` per peer, indexed by the
    // channel's message count, so that no event is recorded again before every wait on its previous
    // record has been enqueued.  A ring phase posts at most W-1 messages to one peer before it
    // collects their acknowledgements (algorithms.cpp), and the acknowledgement of a message is
    // posted only after the receiver enqueued its wait, hence a ring of W-1 suffices.  (With one event
    // per peer a receiver could end up waiting on the sender's NEXT record, and with every rank doing
    // so the streams would wait on each other in a cycle.)
    uint32_t event_ring = 1;
    std::vector<hipEvent_t> ready_events;  // [destination rank * event_ring + message % event_ring]
    std::vector<hipEvent_t> done_events;   // [source rank * event_ring + message % event_ring]
    std::vector<uint64_t> sent;            // messages posted to each peer
    std::vector<uint64_t> received;        // messages taken from each peer
    // Scratchpads (the reference keeps thread_local ones, /root/reference/src/core/dccl.cpp:57-84)
    void* dev_scratch = nullptr;
    size_t dev_scratch_bytes = 0;
    void* host_scratch = nullptr;
    size_t host_scratch_bytes = 0;
    void* dev_work = nullptr;  // full-size work buffer (ReduceScatter's copy of sendbuff)
    size_t dev_work_bytes = 0;
    void* host_work = nullptr;
    size_t host_work_bytes = 0;
};

namespace dccl_amd {

using dccl::ncclResult_t;

// Transport verbs (see the file comment).  `stream` is used for device messages only.
ncclResult_t xport_send(dccl::dcclComm* c, uint32_t peer, const void* buf, size_t bytes, bool device,
                        hipStream_t stream);
ncclResult_t xport_recv(dccl::dcclComm* c, uint32_t peer, void* dst, size_t bytes, bool device,
                        hipStream_t stream);
ncclResult_t xport_wait_send(dccl::dcclComm* c, uint32_t peer, bool device, hipStream_t stream);
// Fused receive + combine: instead of landing the peer's chunk in a scratchpad and combining
// from there (reduce_scatter_ring.cpp:77-94), the combine reads the peer's buffer directly
// (same process; an xGMI peer read when the peer is another GPU):
//     dst[i] = op(dst[i], peer_chunk[i]),  i < count
// One HBM/xGMI read of the peer chunk instead of read + write + read.
ncclResult_t xport_recv_combine(dccl::dcclComm* c, uint32_t peer, void* dst, size_t count, int dtype, int op,
                                bool device, hipStream_t stream);

// One exchange through c->p2p (see P2PExchangeFn).
inline ncclResult_t p2p_exchange(dccl::dcclComm* c, const void* sendbuf, size_t send_bytes, uint32_t to, void* recvbuf,
                                 size_t recv_bytes, uint32_t from, hipStream_t stream) {
    return static_cast<ncclResult_t>(c->p2p(c->p2p_ctx, sendbuf, send_bytes, to, recvbuf, recv_bytes, from, stream));
}

// Scratch management (grown on demand, page/line rounded; never shrinks until finalize).
ncclResult_t ensure_scratch(dccl::dcclComm* c, size_t bytes, bool device);
ncclResult_t ensure_work(dccl::dcclComm* c, size_t bytes, bool device);

// Test-only fault injection: DCCL_FAULT_INJECT=<site>:<rank> makes `site` fail on that rank, so the
// tests can check that one rank's failure reaches every member of the group (as an error) instead of
// leaving peers blocked in a barrier.  Sites: join_events (group formation, dccl_api.cpp),
// direct_combine (the combine step of the direct collectives, direct.cpp).  Read once per process.
bool fault_injected(const char* site, uint32_t rank);

// Local combine on either side of the host/device boundary.
ncclResult_t combine(const void* send, void* recv, int dtype, size_t count, int op, bool device,
                     hipStream_t stream);

}  // namespace dccl_amd
