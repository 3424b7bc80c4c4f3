// dccl_amd/csrc/host_staged.cpp — the combine for host-resident chunks.
//
// In the reference the ring reduce-scatter combines chunks that live in host memory
// (Derecho's RDMA receive scratchpad, /root/reference/src/core/dccl.cpp:102-150) with the
// single-threaded CPU loop do_host_reduce<DT> (/root/reference/src/core/internal_common.hpp:496-586,
// called at /root/reference/src/core/reduce_scatter_ring.cpp:91-94).  Here the same call runs
// on the MI355X: the operands are cut into chunks and pushed through a three-stage pipeline
//     copy-in stream : H2D(send chunk), H2D(recv chunk)
//     compute stream : dccl_local_reduce on the staged chunk
//     copy-out stream: D2H(recv chunk)
// over NSLOT device slots, so PCIe in both directions and the HBM combine overlap
// (SURVEY.md §8(f) row 1).  Page-locked user buffers (dccl_register_host_memory, the
// analogue of dcclRegisterCacheMemory, dccl.cpp:503-549) are DMA'd directly; pageable ones
// are bounced through per-thread pinned staging buffers by the calling thread and a small pool of
// copy threads (DCCL_HOST_COPY_THREADS; one bounce core is slower than the PCIe link).
//
// Page-locked operands (and pageable ones up to 16 MiB, bounced) skip the DMA pipeline: one kernel
// loads and stores the host memory directly over PCIe; the pipeline serves large pageable operands.
//
// Per-thread state (like the reference's thread_local scratchpads, dccl.cpp:67-83): no
// locks, no global mutable state; each thread owns its streams and slots per device.
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "dccl/dccl_reduce.h"
#include "dispatch.hpp"

namespace dccl_amd {

// dccl_local_reduce / dccl_local_reduce_chain under a cap on their one-wave blocks (local_reduce.hip; hidden)
__attribute__((visibility("hidden"))) int local_reduce_capped(const void* send, void* recv, int dtype, size_t count,
                                                              int op, hipStream_t stream, size_t grid_cap);
__attribute__((visibility("hidden"))) int local_reduce_chain_capped(const void* const* sends, int nsend,
                                                                    const void* own, void* dst, int dtype,
                                                                    size_t count, int op, hipStream_t stream,
                                                                    size_t grid_cap);

namespace {

constexpr int kSlots = 3;
constexpr size_t kChunkBytes = size_t(16) << 20;  // per operand per slot
constexpr size_t kParallelCopyMin = size_t(1) << 20;  // smaller bounces stay on the calling thread

// Bounce copies of pageable operands, split into contiguous 64-B aligned slices over the calling
// thread and n-1 workers.  One copy at a time: a Stager, and so its pool, belongs to one thread.
// DCCL_HOST_COPY_THREADS sets n (default 4; 1 = the calling thread alone).
class CopyPool {
public:
    explicit CopyPool(int n) : n_(n < 1 ? 1 : n) {
        for (int i = 1; i < n_; ++i) workers_.emplace_back([this, i] { loop(i); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            ++gen_;
        }
        go_.notify_all();
        for (std::thread& t : workers_) t.join();
    }
    void copy(void* dst, const void* src, size_t bytes) {
        if (n_ == 1 || bytes < kParallelCopyMin) {
            std::memcpy(dst, src, bytes);
            return;
        }
        {
            std::lock_guard<std::mutex> g(m_);
            dst_ = static_cast<unsigned char*>(dst);
            src_ = static_cast<const unsigned char*>(src);
            bytes_ = bytes;
            pending_ = n_ - 1;
            ++gen_;
        }
        go_.notify_all();
        slice(0);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return pending_ == 0; });
    }

private:
    void slice(int i) const {
        const size_t per = (bytes_ / size_t(n_)) & ~size_t(63);
        const size_t b = per * size_t(i), e = (i == n_ - 1) ? bytes_ : b + per;
        std::memcpy(dst_ + b, src_ + b, e - b);
    }
    void loop(int i) {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
            go_.wait(lk, [&] { return gen_ != seen; });
            seen = gen_;
            if (stop_) return;
            lk.unlock();
            slice(i);
            lk.lock();
            if (--pending_ == 0) done_.notify_one();
        }
    }

    const int n_;
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable go_, done_;
    uint64_t gen_ = 0;
    bool stop_ = false;
    int pending_ = 0;
    unsigned char* dst_ = nullptr;
    const unsigned char* src_ = nullptr;
    size_t bytes_ = 0;
};

int copy_threads() {
    const char* e = std::getenv("DCCL_HOST_COPY_THREADS");
    const int n = e ? std::atoi(e) : 4;
    return n < 1 ? 1 : (n > 64 ? 64 : n);
}

struct Slot {
    void* d_send = nullptr;
    void* d_recv = nullptr;
    void* h_send = nullptr;  // pinned bounce buffers, used only for pageable user memory
    void* h_recv = nullptr;
    hipEvent_t in_done = nullptr, comp_done = nullptr, out_done = nullptr;
    size_t pending_bytes = 0;    // bytes of an unfinished D2H into h_recv
    unsigned char* pending_dst = nullptr;
};

class Stager {
public:
    explicit Stager(int device) : device_(device) {}
    ~Stager() { release(); }

    int init() {
        if (ready_) return DCCL_SUCCESS;
        if (hipSetDevice(device_) != hipSuccess) return DCCL_UNHANDLED_DEVICE_ERROR;
        for (hipStream_t* s : {&in_, &comp_, &out_})
            if (hipStreamCreateWithFlags(s, hipStreamNonBlocking) != hipSuccess) return fail();
        for (Slot& sl : slots_) {
            if (hipMalloc(&sl.d_send, kChunkBytes) != hipSuccess) return fail();
            if (hipMalloc(&sl.d_recv, kChunkBytes) != hipSuccess) return fail();
            if (hipHostMalloc(&sl.h_send, kChunkBytes, hipHostMallocDefault) != hipSuccess) return fail();
            if (hipHostMalloc(&sl.h_recv, kChunkBytes, hipHostMallocDefault) != hipSuccess) return fail();
            for (hipEvent_t* e : {&sl.in_done, &sl.comp_done, &sl.out_done})
                if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return fail();
        }
        for (hipEvent_t& e : chain_ev_)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail();
        ready_ = true;
        return DCCL_SUCCESS;
    }

    int run(const unsigned char* send, unsigned char* recv, int dtype, size_t count, int op);
    int run_zero_copy(const unsigned char* send, unsigned char* recv, void* dsend, void* drecv, int dtype,
                      size_t count, int op);
    int run_chain(const void* const* sends, int nsend, const void* own, void* dst, int dtype, size_t count, int op);

private:
    int fail() { release(); return DCCL_UNHANDLED_DEVICE_ERROR; }
    void release() {
        for (Slot& sl : slots_) {
            if (sl.d_send) (void)hipFree(sl.d_send);
            if (sl.d_recv) (void)hipFree(sl.d_recv);
            if (sl.h_send) (void)hipHostFree(sl.h_send);
            if (sl.h_recv) (void)hipHostFree(sl.h_recv);
            for (hipEvent_t e : {sl.in_done, sl.comp_done, sl.out_done})
                if (e) (void)hipEventDestroy(e);
            sl = Slot{};
        }
        if (chain_h_) (void)hipHostFree(chain_h_);
        chain_h_ = nullptr;
        chain_cap_ = 0;
        for (hipEvent_t& e : chain_ev_) {
            if (e) (void)hipEventDestroy(e);
            e = nullptr;
        }
        for (hipStream_t s : {in_, comp_, out_})
            if (s) (void)hipStreamDestroy(s);
        in_ = comp_ = out_ = nullptr;
        ready_ = false;
    }
    int drain_slot(Slot& sl) {  // finish a bounced D2H: wait, then copy to user memory
        if (!sl.pending_dst) return DCCL_SUCCESS;
        if (hipEventSynchronize(sl.out_done) != hipSuccess) return DCCL_UNHANDLED_DEVICE_ERROR;
        bounce(sl.pending_dst, sl.h_recv, sl.pending_bytes);
        sl.pending_dst = nullptr;
        sl.pending_bytes = 0;
        return DCCL_SUCCESS;
    }
    void bounce(void* dst, const void* src, size_t bytes) {  // pageable <-> pinned staging copy
        if (!pool_) pool_ = std::make_unique<CopyPool>(copy_threads());
        pool_->copy(dst, src, bytes);
    }

    int device_;
    bool ready_ = false;
    hipStream_t in_ = nullptr, comp_ = nullptr, out_ = nullptr;
    Slot slots_[kSlots];
    std::unique_ptr<CopyPool> pool_;  // created at the first pageable bounce
    void* chain_h_ = nullptr;         // pinned staging of the host chain combine (two halves), grown on demand
    size_t chain_cap_ = 0;
    hipEvent_t chain_ev_[2] = {};     // last kernel reading each half
};

// Page-locked host memory: returns the device-side alias the GPU can load/store through
// (nullptr for pageable memory).
void* pinned_device_alias(const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();  // unregistered pageable memory reports an error: clear it
        return nullptr;
    }
    if (attr.type != hipMemoryTypeHost) return nullptr;
    // attributes describe the allocation: offset the alias to `p`
    const auto host_base = static_cast<const unsigned char*>(attr.hostPointer);
    auto dev_base = static_cast<unsigned char*>(attr.devicePointer);
    if (host_base == nullptr || dev_base == nullptr) return nullptr;
    return dev_base + (static_cast<const unsigned char*>(p) - host_base);
}

// Operands up to this many bytes take the zero-copy path (one kernel loading and storing the
// page-locked host memory over PCIe, no DMA staging).  Measured on MI355X it beats the 3-stream
// DMA pipeline at every size for page-locked operands (1 MiB: 13.4 vs 7.9 GiB/s; 256 MiB: 24.8
// vs 24.0 GiB/s), so the default is unlimited; DCCL_HOST_ZEROCOPY_MAX overrides (0 disables).
// Pageable operands are bounced through a 16 MiB pinned slot, so they qualify only up to that.
size_t zero_copy_max() {
    const char* e = std::getenv("DCCL_HOST_ZEROCOPY_MAX");
    return e ? static_cast<size_t>(std::strtoull(e, nullptr, 10)) : ~size_t(0);
}

// One-wave blocks of a zero-copy combine, each striding over the 1 KiB tiles.  The device combine's grid (one block
// per tile) issues every read of a PCIe-bound launch at once and leaves its writes to a burst at the end, so the
// link's host->device and device->host directions take turns; a few hundred striding waves keep both busy
// together.  dccl_local_reduce_host per call on MI355X, fp32 Sum, registered / hipHostMalloc operands, best of
// three (profiles/r6_zero_copy_waves.json): 512 waves against one block per tile, 4 MiB 220 -> 196 us, 16 MiB
// 733 -> 682 us, 1 GiB 40.2 -> 37.5 ms (57 GB/s host->device); flat from 320 to 768 waves, slower at 128 and
// from 1024.  DCCL_HOST_ZEROCOPY_WAVES overrides (0: one block per tile).
size_t zero_copy_waves() {
    static const size_t v = [] {
        const char* e = std::getenv("DCCL_HOST_ZEROCOPY_WAVES");
        return e ? static_cast<size_t>(std::strtoull(e, nullptr, 10)) : size_t(512);
    }();
    return v;
}

int Stager::run_zero_copy(const unsigned char* send, unsigned char* recv, void* dsend, void* drecv, int dtype,
                          size_t count, int op) {
    const size_t bytes = count * size_of_dtype(dtype);
    Slot& sl = slots_[0];
    if ((dsend == nullptr || drecv == nullptr) && bytes > kChunkBytes) return DCCL_INTERNAL_ERROR;  // bounce size
    if (dsend == nullptr) {  // pageable: bounce through the slot's pinned buffer
        bounce(sl.h_send, send, bytes);
        if (hipHostGetDevicePointer(&dsend, sl.h_send, 0) != hipSuccess) return DCCL_UNHANDLED_DEVICE_ERROR;
    }
    const bool bounce_recv = drecv == nullptr;
    if (bounce_recv) {
        bounce(sl.h_recv, recv, bytes);
        if (hipHostGetDevicePointer(&drecv, sl.h_recv, 0) != hipSuccess) return DCCL_UNHANDLED_DEVICE_ERROR;
    }
    int rc = local_reduce_capped(dsend, drecv, dtype, count, op, comp_, zero_copy_waves());
    if (hipStreamSynchronize(comp_) != hipSuccess && rc == DCCL_SUCCESS) rc = DCCL_UNHANDLED_DEVICE_ERROR;
    if (rc == DCCL_SUCCESS && bounce_recv) bounce(recv, sl.h_recv, bytes);
    return rc;
}

int Stager::run(const unsigned char* send, unsigned char* recv, int dtype, size_t count, int op) {
    const size_t esz = size_of_dtype(dtype);
    const size_t per_chunk = kChunkBytes / esz;
    void* const dsend = pinned_device_alias(send);
    void* const drecv = pinned_device_alias(recv);
    const size_t bytes = count * esz;
    if (bytes <= zero_copy_max() && ((dsend != nullptr && drecv != nullptr) || bytes <= kChunkBytes))
        return run_zero_copy(send, recv, dsend, drecv, dtype, count, op);
    const bool send_pinned = dsend != nullptr, recv_pinned = drecv != nullptr;
    int rc = DCCL_SUCCESS;
    size_t k = 0;
    for (size_t off = 0; off < count && rc == DCCL_SUCCESS; off += per_chunk, ++k) {
        const size_t n = (count - off < per_chunk) ? count - off : per_chunk;
        const size_t bytes = n * esz;
        Slot& sl = slots_[k % kSlots];
        // Slot reuse: the previous occupant's D2H must be done (and unbounced).
        if ((rc = drain_slot(sl)) != DCCL_SUCCESS) break;
        if (hipStreamWaitEvent(in_, sl.out_done, 0) != hipSuccess) { rc = DCCL_UNHANDLED_DEVICE_ERROR; break; }
        const unsigned char* src_s = send + off * esz;
        const unsigned char* src_r = recv + off * esz;
        if (!send_pinned) { bounce(sl.h_send, src_s, bytes); src_s = static_cast<unsigned char*>(sl.h_send); }
        if (!recv_pinned) {
            // h_recv is also the D2H landing zone of this slot: its previous use was drained above.
            bounce(sl.h_recv, src_r, bytes);
            src_r = static_cast<unsigned char*>(sl.h_recv);
        }
        if (hipMemcpyAsync(sl.d_send, src_s, bytes, hipMemcpyHostToDevice, in_) != hipSuccess ||
            hipMemcpyAsync(sl.d_recv, src_r, bytes, hipMemcpyHostToDevice, in_) != hipSuccess ||
            hipEventRecord(sl.in_done, in_) != hipSuccess ||
            hipStreamWaitEvent(comp_, sl.in_done, 0) != hipSuccess) {
            rc = DCCL_UNHANDLED_DEVICE_ERROR;
            break;
        }
        if ((rc = dccl_local_reduce(sl.d_send, sl.d_recv, dtype, n, op, comp_)) != DCCL_SUCCESS) break;
        unsigned char* dst = recv + off * esz;
        if (hipEventRecord(sl.comp_done, comp_) != hipSuccess ||
            hipStreamWaitEvent(out_, sl.comp_done, 0) != hipSuccess ||
            hipMemcpyAsync(recv_pinned ? dst : sl.h_recv, sl.d_recv, bytes, hipMemcpyDeviceToHost, out_) !=
                hipSuccess ||
            hipEventRecord(sl.out_done, out_) != hipSuccess) {
            rc = DCCL_UNHANDLED_DEVICE_ERROR;
            break;
        }
        if (!recv_pinned) { sl.pending_dst = dst; sl.pending_bytes = bytes; }
        // With pageable send, the CPU memcpy of the next chunk into this slot's h_send must not
        // race the in-flight H2D: wait for the copy-in of the slot we are about to reuse.
        if (!send_pinned || !recv_pinned) {
            Slot& next = slots_[(k + 1) % kSlots];
            if (hipEventSynchronize(next.in_done) != hipSuccess) { rc = DCCL_UNHANDLED_DEVICE_ERROR; break; }
        }
    }
    // Always drain: no slot may be left with work in flight, even after an error.
    for (Slot& sl : slots_) {
        const int d = drain_slot(sl);
        if (rc == DCCL_SUCCESS) rc = d;
    }
    if (hipStreamSynchronize(out_) != hipSuccess && rc == DCCL_SUCCESS) rc = DCCL_UNHANDLED_DEVICE_ERROR;
    if (hipStreamSynchronize(comp_) != hipSuccess && rc == DCCL_SUCCESS) rc = DCCL_UNHANDLED_DEVICE_ERROR;
    return rc;
}

// One-wave blocks of a zero-copy chain combine (zero_copy_waves' rule; in-phase launches only).  Per call on MI355X,
// fp32 Sum, k = 1 / 3 / 7 sources of 64 MiB, 256 waves against one block per tile (profiles/r6_chain_host_waves.json):
// registered operands 2742 -> 2457, 5223 -> 4770, 10531 -> 9458 us; staged pageable ones 4057 -> 3586, 6260 -> 5796,
// 11391 -> 10793 us; 512 and 1024 waves within noise of 256 for registered operands.  DCCL_HOST_CHAIN_WAVES
// overrides (0: one block per tile).
size_t chain_waves() {
    static const size_t v = [] {
        const char* e = std::getenv("DCCL_HOST_CHAIN_WAVES");
        return e ? static_cast<size_t>(std::strtoull(e, nullptr, 10)) : size_t(256);
    }();
    return v;
}

// Host chain combine, the host twin of dccl_local_reduce_chain.  Operands that are not page-locked are
// bounced into pinned staging and one zero-copy chain kernel per piece reads them over PCIe in the
// ring's order; the result is copied back.  Pieces alternate between two halves of the staging area, so
// the bounce of piece j overlaps the kernel of piece j-1.  Page-locked operands are read in place.
constexpr size_t kChainHalfBytes = size_t(32) << 20;

int Stager::run_chain(const void* const* sends, int nsend, const void* own, void* dst, int dtype, size_t count,
                      int op) {
    const size_t esz = size_of_dtype(dtype);
    const void* as[8];
    bool all_pinned = true;
    for (int k = 0; k < nsend; ++k)
        if ((as[k] = pinned_device_alias(sends[k])) == nullptr) all_pinned = false;
    void* a_own = pinned_device_alias(own);
    void* a_dst = pinned_device_alias(dst);
    const bool stage_own = a_own == nullptr || a_dst == nullptr;
    int rc = DCCL_SUCCESS;
    if (all_pinned && !stage_own) {  // everything page-locked: one kernel, nothing staged
        rc = local_reduce_chain_capped(as, nsend, a_own, a_dst, dtype, count, op, comp_, chain_waves());
        if (hipStreamSynchronize(comp_) != hipSuccess && rc == DCCL_SUCCESS) rc = DCCL_UNHANDLED_DEVICE_ERROR;
        return rc;
    }
    const size_t slot_max = kChainHalfBytes / size_t(nsend + 1) / 256 * 256;  // bytes per operand per half
    const size_t piece = count * esz <= slot_max ? count : slot_max / esz;    // elements
    const size_t npieces = (count + piece - 1) / piece;
    const size_t ps = (piece * esz + 255) / 256 * 256, half = ps * size_t(nsend + 1);
    const size_t need = npieces > 1 ? 2 * half : half;
    if (chain_cap_ < need) {
        if (chain_h_) (void)hipHostFree(chain_h_);
        chain_h_ = nullptr;
        chain_cap_ = 0;
        const size_t cap = need < (size_t(1) << 20) ? size_t(1) << 20 : need;
        if (hipHostMalloc(&chain_h_, cap, hipHostMallocDefault) != hipSuccess) return DCCL_UNHANDLED_DEVICE_ERROR;
        chain_cap_ = cap;
    }
    void* dbase = nullptr;
    if (hipHostGetDevicePointer(&dbase, chain_h_, 0) != hipSuccess) return DCCL_UNHANDLED_DEVICE_ERROR;
    auto* h = static_cast<unsigned char*>(chain_h_);
    auto* d = static_cast<unsigned char*>(dbase);
    auto elems = [&](size_t j) { return j + 1 == npieces ? count - j * piece : piece; };
    // wait for piece j's kernel, then copy its result back to dst
    auto finish = [&](size_t j) {
        if (hipEventSynchronize(chain_ev_[j % 2]) != hipSuccess) return DCCL_UNHANDLED_DEVICE_ERROR;
        if (stage_own)
            bounce(static_cast<unsigned char*>(dst) + j * piece * esz, h + (j % 2) * half + size_t(nsend) * ps,
                   elems(j) * esz);
        return DCCL_SUCCESS;
    };
    size_t launched = 0, returned = 0;
    for (size_t j = 0; j < npieces && rc == DCCL_SUCCESS; ++j) {
        if (j >= 2 && (rc = finish(returned++)) != DCCL_SUCCESS) break;  // frees this half
        const size_t o = j * piece * esz, n = elems(j), hb = (j % 2) * half;
        const void* ds[8];
        for (int k = 0; k < nsend; ++k) {
            if (as[k] != nullptr) {
                ds[k] = static_cast<const unsigned char*>(as[k]) + o;
                continue;
            }
            bounce(h + hb + size_t(k) * ps, static_cast<const unsigned char*>(sends[k]) + o, n * esz);
            ds[k] = d + hb + size_t(k) * ps;
        }
        const void* down;
        void* ddst;
        if (stage_own) {  // own is staged and the kernel writes the result over it (own may alias dst)
            bounce(h + hb + size_t(nsend) * ps, static_cast<const unsigned char*>(own) + o, n * esz);
            down = ddst = d + hb + size_t(nsend) * ps;
        } else {
            down = static_cast<const unsigned char*>(a_own) + o;
            ddst = static_cast<unsigned char*>(a_dst) + o;
        }
        rc = local_reduce_chain_capped(ds, nsend, down, ddst, dtype, n, op, comp_, chain_waves());
        if (rc == DCCL_SUCCESS && hipEventRecord(chain_ev_[j % 2], comp_) != hipSuccess)
            rc = DCCL_UNHANDLED_DEVICE_ERROR;
        if (rc == DCCL_SUCCESS) launched = j + 1;
    }
    // no kernel may still read the staging area after return, even after an error
    if (hipStreamSynchronize(comp_) != hipSuccess && rc == DCCL_SUCCESS) rc = DCCL_UNHANDLED_DEVICE_ERROR;
    while (rc == DCCL_SUCCESS && returned < launched) rc = finish(returned++);
    return rc;
}

struct ThreadStagers {
    std::vector<std::unique_ptr<Stager>> per_device;
    Stager* get(int dev) {
        if (dev < 0) return nullptr;
        if (static_cast<size_t>(dev) >= per_device.size()) per_device.resize(dev + 1);
        if (!per_device[dev]) per_device[dev] = std::make_unique<Stager>(dev);
        return per_device[dev].get();
    }
};

thread_local ThreadStagers t_stagers;

}  // namespace
}  // namespace dccl_amd

using namespace dccl_amd;

extern "C" int dccl_local_reduce_host(const void* send, void* recv, int dtype, size_t count, int op) {
    const int v = validate(dtype, op);
    if (v != DCCL_SUCCESS) return v;
    if (count == 0) return DCCL_SUCCESS;
    if (send == nullptr || recv == nullptr) return DCCL_INVALID_ARGUMENT;
    if (partial_overlap(send, recv, count * size_of_dtype(dtype))) return DCCL_INVALID_ARGUMENT;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) return DCCL_UNHANDLED_DEVICE_ERROR;
    Stager* st = t_stagers.get(dev);
    if (st == nullptr) return DCCL_UNHANDLED_DEVICE_ERROR;
    int rc = st->init();
    if (rc != DCCL_SUCCESS) return rc;
    rc = st->run(static_cast<const unsigned char*>(send), static_cast<unsigned char*>(recv), dtype, count, op);
    (void)hipSetDevice(dev);
    return rc;
}

extern "C" int dccl_local_reduce_chain_host(const void* const* sends, int nsend, const void* own, void* dst,
                                            int dtype, size_t count, int op) {
    const int v = validate(dtype, op);
    if (v != DCCL_SUCCESS) return v;
    if (nsend < 1 || nsend > 8 || sends == nullptr) return DCCL_INVALID_ARGUMENT;
    if (count == 0) return DCCL_SUCCESS;
    if (own == nullptr || dst == nullptr) return DCCL_INVALID_ARGUMENT;
    for (int k = 0; k < nsend; ++k)
        if (sends[k] == nullptr) return DCCL_INVALID_ARGUMENT;
    if (sources_overlap_destination(sends, nsend, own, dst, count * size_of_dtype(dtype)))
        return DCCL_INVALID_ARGUMENT;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) return DCCL_UNHANDLED_DEVICE_ERROR;
    Stager* st = t_stagers.get(dev);
    if (st == nullptr) return DCCL_UNHANDLED_DEVICE_ERROR;
    int rc = st->init();
    if (rc != DCCL_SUCCESS) return rc;
    rc = st->run_chain(sends, nsend, own, dst, dtype, count, op);
    (void)hipSetDevice(dev);
    return rc;
}

extern "C" int dccl_register_host_memory(void* buffer, size_t size) {
    if (buffer == nullptr || size == 0) return DCCL_INVALID_ARGUMENT;
    return hipHostRegister(buffer, size, hipHostRegisterDefault) == hipSuccess ? DCCL_SUCCESS
                                                                               : DCCL_UNHANDLED_DEVICE_ERROR;
}

extern "C" int dccl_deregister_host_memory(void* buffer) {
    if (buffer == nullptr) return DCCL_INVALID_ARGUMENT;
    return hipHostUnregister(buffer) == hipSuccess ? DCCL_SUCCESS : DCCL_UNHANDLED_DEVICE_ERROR;
}

// The measured crossover of dccl_local_reduce_host against the reference's one-thread loop on a core of the
// buffers' NUMA node (bench.py `host_crossover`, registered fp32 Sum operands, cold caches;
// profiles/r6_host_crossover.json).  The loop's rate is in bytes for every dtype it vectorises, so one byte
// threshold serves them all.
constexpr size_t kHostGpuMinBytes = size_t(64) << 20;

extern "C" size_t dccl_host_reduce_gpu_min_bytes(int dtype) {
    if (dtype == kFloat16 || dtype == kBfloat16 || size_of_dtype(dtype) == 0) return 0;  // no reference CPU loop
    static const size_t v = [] {
        const char* e = std::getenv("DCCL_HOST_GPU_MIN_BYTES");
        return e ? static_cast<size_t>(std::strtoull(e, nullptr, 10)) : kHostGpuMinBytes;
    }();
    return v;
}

extern "C" size_t dccl_size_of_type(int dtype) { return size_of_dtype(dtype); }

extern "C" const char* dccl_result_string(int result) {
    switch (result) {
    case 0: return "ncclSuccess";
    case 1: return "ncclUnhandledCudaError (HIP runtime failure)";
    case 2: return "ncclSystemError";
    case 3: return "ncclInternalError";
    case 4: return "ncclInvalidArgument";
    case 5: return "ncclInvalidUsage";
    case 6: return "ncclRemoteError";
    case 7: return "ncclInProgress";
    default: return "unknown result";
    }
}

extern "C" int dccl_version(void) { return 1 * 10000 + 0 * 100 + 0; }
