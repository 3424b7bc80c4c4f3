// dccl_amd/csrc/comm.cpp — in-process group, stream-ordered transport, scratchpads.
// See comm.hpp for the protocol.  Replaces the reference's Derecho OOB wrappers
// (/root/reference/src/core/internal_common.hpp:698-792) for ranks that share a process.
#include "comm.hpp"

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

#include "dccl/dccl_reduce.h"
#include "dispatch.hpp"

namespace dccl_amd {

Group::Group(uint32_t world)
    : devices(world, -1), pub_in(world, nullptr), pub_out(world, nullptr), taken(world, false), world_(world) {
    chan_.reserve(size_t(world) * world);
    for (size_t i = 0; i < size_t(world) * world; ++i) chan_.push_back(std::make_unique<Channel>());
}

// Ranks of a collective arrive within microseconds of each other: poll the generation for up to 2 ms
// (with the pause hint) before blocking on the condition variable, whose wake-up costs tens of
// microseconds on the critical path of every direct collective (ipc_latency.py@4f20423).
bool Group::barrier(bool ok) {
    std::unique_lock<std::mutex> lk(bmu_);
    const uint64_t gen = barrier_gen_.load(std::memory_order_relaxed);
    if (!ok) barrier_bad_ = true;
    if (++barrier_count_ == world_) {
        // Generation gen+2 cannot complete before every rank of gen has read this slot: each of them must
        // arrive at gen+1 first, so indexing the outcome by parity is safe.
        const bool all = !barrier_bad_;
        barrier_ok_[gen & 1] = all;
        barrier_count_ = 0;
        barrier_bad_ = false;
        barrier_gen_.store(gen + 1, std::memory_order_release);
        bcv_.notify_all();
        return all;
    }
    lk.unlock();
    const auto start = std::chrono::steady_clock::now();
    for (uint32_t i = 1; barrier_gen_.load(std::memory_order_acquire) == gen; ++i) {
        if ((i & 1023) == 0) {
            if (std::chrono::steady_clock::now() - start > std::chrono::milliseconds(2)) break;
            std::this_thread::yield();  // a rank without a core of its own gets one
        }
        __builtin_ia32_pause();
    }
    lk.lock();
    bcv_.wait(lk, [&] { return barrier_gen_.load(std::memory_order_acquire) != gen; });
    return barrier_ok_[gen & 1];
}

namespace {
inline ncclResult_t hip_ok(hipError_t e) {
    return e == hipSuccess ? dccl::ncclSuccess : dccl::ncclUnhandledCudaError;
}

// Wait for `ready()` on channel `ch`: spin briefly (ring steps hand off every few microseconds;
// a futex sleep/wake costs as much), then block on the condition variable.
template <typename Pred>
void channel_wait(Channel& ch, std::unique_lock<std::mutex>& lk, Pred ready) {
    for (int i = 0; i < 2000 && !ready(); ++i) {
        lk.unlock();
        std::this_thread::yield();
        lk.lock();
    }
    ch.cv.wait(lk, ready);
}
}  // namespace

ncclResult_t xport_send(dccl::dcclComm* c, uint32_t peer, const void* buf, size_t bytes, bool device,
                        hipStream_t stream) {
    Message m{buf, bytes, device, nullptr};
    if (device) {
        m.ready = c->ready_events[size_t(peer) * c->event_ring + c->sent[peer] % c->event_ring];
        if (hipEventRecord(m.ready, stream) != hipSuccess) return dccl::ncclUnhandledCudaError;
    }
    ++c->sent[peer];
    Channel& ch = c->group->channel(c->rank, peer);
    {
        std::lock_guard<std::mutex> lk(ch.mu);
        ch.msgs.push_back(m);
    }
    ch.cv.notify_all();
    return dccl::ncclSuccess;
}

ncclResult_t xport_recv(dccl::dcclComm* c, uint32_t peer, void* dst, size_t bytes, bool device,
                        hipStream_t stream) {
    Channel& ch = c->group->channel(peer, c->rank);
    Message m;
    {
        std::unique_lock<std::mutex> lk(ch.mu);
        channel_wait(ch, lk, [&] { return !ch.msgs.empty(); });
        m = ch.msgs.front();
        ch.msgs.pop_front();
    }
    const uint64_t n_taken = c->received[peer]++;
    ncclResult_t rc = dccl::ncclSuccess;
    Ack a;
    if (m.bytes != bytes || m.device != device) {
        rc = dccl::ncclInvalidUsage;  // mismatched send/recv pairing
    } else if (device) {
        a.done = c->done_events[size_t(peer) * c->event_ring + n_taken % c->event_ring];
        rc = hip_ok(hipStreamWaitEvent(stream, m.ready, 0));
        if (rc == dccl::ncclSuccess) rc = hip_ok(hipMemcpyAsync(dst, m.ptr, bytes, hipMemcpyDeviceToDevice, stream));
        if (rc == dccl::ncclSuccess) rc = hip_ok(hipEventRecord(a.done, stream));
    } else {
        std::memcpy(dst, m.ptr, bytes);
    }
    {
        std::lock_guard<std::mutex> lk(ch.mu);  // always acknowledge: the sender must not hang
        ch.acks.push_back(a);
    }
    ch.cv.notify_all();
    return rc;
}

ncclResult_t xport_recv_combine(dccl::dcclComm* c, uint32_t peer, void* dst, size_t count, int dtype, int op,
                                bool device, hipStream_t stream) {
    Channel& ch = c->group->channel(peer, c->rank);
    Message m;
    {
        std::unique_lock<std::mutex> lk(ch.mu);
        channel_wait(ch, lk, [&] { return !ch.msgs.empty(); });
        m = ch.msgs.front();
        ch.msgs.pop_front();
    }
    const uint64_t n_taken = c->received[peer]++;
    ncclResult_t rc = dccl::ncclSuccess;
    Ack a;
    if (m.bytes != count * size_of_dtype(dtype) || m.device != device) {
        rc = dccl::ncclInvalidUsage;
    } else if (device) {
        a.done = c->done_events[size_t(peer) * c->event_ring + n_taken % c->event_ring];
        rc = hip_ok(hipStreamWaitEvent(stream, m.ready, 0));
        if (rc == dccl::ncclSuccess) rc = combine(m.ptr, dst, dtype, count, op, true, stream);
        // the done event must exist in the stream even after a failed combine: the sender waits on it
        const ncclResult_t re = hip_ok(hipEventRecord(a.done, stream));
        if (rc == dccl::ncclSuccess) rc = re;
    } else {
        rc = combine(m.ptr, dst, dtype, count, op, false, stream);
    }
    {
        std::lock_guard<std::mutex> lk(ch.mu);
        ch.acks.push_back(a);
    }
    ch.cv.notify_all();
    return rc;
}

ncclResult_t xport_wait_send(dccl::dcclComm* c, uint32_t peer, bool device, hipStream_t stream) {
    Channel& ch = c->group->channel(c->rank, peer);
    Ack a;
    {
        std::unique_lock<std::mutex> lk(ch.mu);
        channel_wait(ch, lk, [&] { return !ch.acks.empty(); });
        a = ch.acks.front();
        ch.acks.pop_front();
    }
    if (device && a.done) return hip_ok(hipStreamWaitEvent(stream, a.done, 0));
    return dccl::ncclSuccess;
}

namespace {
constexpr size_t kScratchMin = size_t(64) << 20;  // initial size, as the reference (dccl.cpp:61-66)
inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

ncclResult_t grow(void** p, size_t* have, size_t need, bool device) {
    if (*have >= need) return dccl::ncclSuccess;
    size_t sz = need < kScratchMin ? kScratchMin : round_up(need, size_t(2) << 20);
    if (device) {
        if (*p && hipFree(*p) != hipSuccess) return dccl::ncclUnhandledCudaError;  // hipFree synchronises
        *p = nullptr;
        *have = 0;
        if (hipMalloc(p, sz) != hipSuccess) return dccl::ncclUnhandledCudaError;
    } else {
        if (*p) {
            (void)hipHostUnregister(*p);
            std::free(*p);
        }
        *p = nullptr;
        *have = 0;
        if (posix_memalign(p, 4096, sz) != 0) return dccl::ncclSystemError;
        // page-lock the host scratchpad so staging DMAs it directly (the reference registers
        // its scratchpad with Derecho, dccl.cpp:129-141)
        if (hipHostRegister(*p, sz, hipHostRegisterDefault) != hipSuccess) (void)hipGetLastError();
    }
    *have = sz;
    return dccl::ncclSuccess;
}
}  // namespace

ncclResult_t ensure_scratch(dccl::dcclComm* c, size_t bytes, bool device) {
    return device ? grow(&c->dev_scratch, &c->dev_scratch_bytes, bytes, true)
                  : grow(&c->host_scratch, &c->host_scratch_bytes, bytes, false);
}

ncclResult_t ensure_work(dccl::dcclComm* c, size_t bytes, bool device) {
    return device ? grow(&c->dev_work, &c->dev_work_bytes, bytes, true)
                  : grow(&c->host_work, &c->host_work_bytes, bytes, false);
}

bool fault_injected(const char* site, uint32_t rank) {
    // read once per process (the tests set it per child process): no getenv on the collectives' steps
    static const std::string spec = [] {
        const char* e = std::getenv("DCCL_FAULT_INJECT");
        return std::string(e ? e : "");
    }();
    if (spec.empty()) return false;
    const char* f = spec.c_str();
    const size_t n = std::strlen(site);
    return std::strncmp(f, site, n) == 0 && f[n] == ':' && std::strtoul(f + n + 1, nullptr, 10) == rank;
}

ncclResult_t combine(const void* send, void* recv, int dtype, size_t count, int op, bool device,
                     hipStream_t stream) {
    const int rc = device ? dccl_local_reduce(send, recv, dtype, count, op, stream)
                          : dccl_local_reduce_host(send, recv, dtype, count, op);
    return static_cast<ncclResult_t>(rc);
}

}  // namespace dccl_amd
