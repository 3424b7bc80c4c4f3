// dccl_amd/csrc/direct.cpp — see direct.hpp.
#include "direct.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <iterator>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "bootstrap.hpp"
#include "dccl/dccl_reduce.h"
#include "dispatch.hpp"

namespace dccl_amd {
namespace {

using dccl::dcclComm;

constexpr uint64_t kMagic = 0x3143504943434344ull;  // "DCCIPC1"
constexpr uint32_t kMaxRanks = 64;
constexpr size_t kHandleBytes = sizeof(hipIpcMemHandle_t);
// Peer mappings are kept for later calls, in one cache per process (below); the oldest unused one is
// closed beyond this many, or beyond this many bytes of peer memory: a mapping keeps the peer's allocation
// alive after the peer freed it, so the cache must not hold more than a bounded amount of it.
constexpr size_t kMaxOpenMappings = 256;
constexpr size_t kMaxOpenBytes = size_t(64) << 30;

struct ShmSlot {
    unsigned char h_in[kHandleBytes];
    unsigned char h_out[kHandleBytes];
    uint64_t off_in, off_out;
    uint64_t serial_in, serial_out;  // the exporter's serial of each handle (see Export)
    uint64_t base_in, base_out;      // the exported allocations' base addresses in the exporter
    uint64_t size_in, size_out;      // and their sizes
    int64_t pid;                     // the exporter
};

struct ShmCtl {
    std::atomic<uint64_t> magic;
    uint32_t world;
    std::atomic<uint32_t> joined;
    std::atomic<uint32_t> count;
    std::atomic<uint32_t> gen;
    std::atomic<int32_t> abort;
    ShmSlot slot[kMaxRanks];
};

// One export per allocation.  `serial` numbers this process's exports: the handle bytes of a new allocation
// at a freed one's address and size repeat (observed on ROCm 7.2), so importers tell a new
// allocation from the freed one by the serial, not by the bytes.
struct Export {
    size_t size;
    uint64_t buffer_id;
    uint64_t serial;
    hipIpcMemHandle_t handle;
};

struct Mapping {
    void* base;
    uint64_t serial;
    size_t bytes;
    uint32_t users;      // collectives of this process between their import and their last phase point
    uint64_t import_id;  // the runtime's buffer id of this import (0: unknown)
};

uint64_t buffer_id_of(void* p) {
    uint64_t id = 0;
    if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, reinterpret_cast<hipDeviceptr_t>(p)) !=
        hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return id;
}

// Exports and peer mappings are per PROCESS, shared by every IPC communicator in it: the runtime hands out
// one import per handle per process (opening handle bytes that are already open returns that mapping), so
// a cache per communicator could not replace a stale mapping another communicator still holds.  Mappings
// are keyed by the exporting process and the allocation's address there, for every peer of every communicator.
struct ProcCache {
    std::mutex mu;
    uint64_t next_serial = 1;
    std::map<uintptr_t, Export> exported;  // allocation base -> its export
    std::map<std::string, Mapping> opened;  // (exporter pid, allocation base) -> mapping
    std::deque<std::string> open_order;     // oldest first
    size_t open_bytes = 0;
    uint32_t comms = 0;                     // live IPC communicators of this process
};

ProcCache& cache() {
    static ProcCache* c = new ProcCache;  // never destroyed: communicators may outlive static destructors
    return *c;
}

struct IpcXport {
    ShmCtl* ctl = nullptr;
    double timeout_s = 300.0;
};

IpcXport* xport(const dcclComm* c) { return static_cast<IpcXport*>(c->ipc); }

// DCCL_IPC_DEBUG=1: one line on stderr per export made and per peer mapping opened, reused or replaced
// (read once per process)
bool ipc_debug() {
    static const bool on = [] {
        const char* v = std::getenv("DCCL_IPC_DEBUG");
        return v != nullptr && *v == '1';
    }();
    return on;
}

// Sense-reversing barrier on the shared counters that also agrees on success: a rank arriving with
// ok == false raises the segment's abort flag, and every rank returns ncclRemoteError from a barrier that
// completes with the flag up.  The flag is sticky (the transport is unusable after a failed collective,
// like an aborted NCCL communicator).  Every waiter gives up (and tells the others) after timeout_s, so
// a dead peer turns into an error instead of a hang.
ncclResult_t shm_barrier(IpcXport* x, bool ok = true) {
    ShmCtl* s = x->ctl;
    if (!ok) s->abort.store(1, std::memory_order_relaxed);
    const uint32_t g = s->gen.load(std::memory_order_acquire);
    if (s->count.fetch_add(1, std::memory_order_acq_rel) + 1 == s->world) {
        s->count.store(0, std::memory_order_relaxed);
        s->gen.store(g + 1, std::memory_order_release);
        return s->abort.load(std::memory_order_relaxed) ? dccl::ncclRemoteError : dccl::ncclSuccess;
    }
    // Spin (with the pause hint) for up to kSpin before sleeping: peers arrive within microseconds of
    // each other in a collective, and a 20 us sleep costs 50-80 us once the kernel's timer slack is
    // added, which set the latency of small collectives (tools/ipc_latency.py).
    constexpr auto kSpin = std::chrono::milliseconds(2);
    const auto start = std::chrono::steady_clock::now();
    const auto deadline = start + std::chrono::duration<double>(x->timeout_s);
    for (uint64_t i = 0; s->gen.load(std::memory_order_acquire) == g; ++i) {
        if (s->abort.load(std::memory_order_relaxed)) return dccl::ncclRemoteError;
        if ((i & 1023) != 1023) {
            __builtin_ia32_pause();
            continue;
        }
        const auto now = std::chrono::steady_clock::now();
        if (now > deadline) {
            s->abort.store(1, std::memory_order_relaxed);
            return dccl::ncclSystemError;
        }
        if (now - start > kSpin) std::this_thread::sleep_for(std::chrono::microseconds(20));
        else std::this_thread::yield();  // a peer without a core of its own gets one
    }
    return s->abort.load(std::memory_order_relaxed) ? dccl::ncclRemoteError : dccl::ncclSuccess;
}

ncclResult_t export_ptr(const void* p, unsigned char* handle_out, uint64_t* off_out, uint64_t* serial_out,
                        uint64_t* base_out, uint64_t* size_out) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (const hipError_t e = hipMemGetAddressRange(&base, &size, const_cast<void*>(p)); e != hipSuccess) {
        (void)hipGetLastError();
        if (ipc_debug()) std::fprintf(stderr, "[dccl ipc %d] hipMemGetAddressRange(%p) -> %d\n", ::getpid(), p, int(e));
        return dccl::ncclInvalidArgument;  // not a device allocation of this process
    }
    uint64_t id = 0;
    const bool have_id = hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID,
                                                reinterpret_cast<hipDeviceptr_t>(base)) == hipSuccess;
    if (!have_id) {
        (void)hipGetLastError();
        if (ipc_debug()) std::fprintf(stderr, "[dccl ipc %d] no buffer id for %p: exported afresh\n", ::getpid(), base);
    }
    const uintptr_t b = reinterpret_cast<uintptr_t>(base);
    ProcCache& pc = cache();
    std::lock_guard<std::mutex> lock(pc.mu);
    auto it = pc.exported.find(b);
    // without the allocation's buffer id the cached export cannot be told from a freed allocation's at the
    // same address and size: export again (a new serial makes the peers re-map)
    if (!have_id || it == pc.exported.end() || it->second.size != size || it->second.buffer_id != id) {
        Export e{size, id, pc.next_serial++, {}};
        // Exporting an allocation at the address of a freed one that a peer still maps can fail for a moment
        // (hipErrorInvalidValue; seen about once in 600 re-allocations in tests/test_direct.py::
        // test_ipc_reallocated_buffers); retry with backoff for ~0.5 s, like the re-open in import_ptr.
        for (int attempt = 0, us = 100;; ++attempt, us = std::min(2 * us, 100000)) {
            const hipError_t he = hipIpcGetMemHandle(&e.handle, base);
            if (he == hipSuccess) break;
            (void)hipGetLastError();
            if (ipc_debug())
                std::fprintf(stderr, "[dccl ipc %d] hipIpcGetMemHandle(base=%p size=%zu buffer_id=%llu) -> %d "
                             "(attempt %d)\n", ::getpid(), base, size, static_cast<unsigned long long>(id), int(he),
                             attempt);
            if (attempt == 14) return dccl::ncclUnhandledCudaError;
            std::this_thread::sleep_for(std::chrono::microseconds(us));
        }
        // entries whose range this allocation now covers name freed allocations: drop them, so the map
        // holds one entry per address range in use rather than one per allocation ever exported
        for (auto o = pc.exported.lower_bound(b); o != pc.exported.begin();) {
            --o;
            if (o->first + o->second.size <= b) break;
            o = pc.exported.erase(o);
        }
        for (auto o = pc.exported.lower_bound(b); o != pc.exported.end() && o->first < b + size;)
            o = pc.exported.erase(o);
        it = pc.exported.emplace(b, e).first;
        if (ipc_debug())
            std::fprintf(stderr, "[dccl ipc %d] export base=%p size=%zu buffer_id=%llu serial=%llu\n", ::getpid(),
                         base, size, static_cast<unsigned long long>(id), static_cast<unsigned long long>(e.serial));
    }
    std::memcpy(handle_out, &it->second.handle, kHandleBytes);
    *off_out = reinterpret_cast<uintptr_t>(p) - b;
    *serial_out = it->second.serial;
    *base_out = b;
    *size_out = it->second.size;
    return dccl::ncclSuccess;
}

void close_mapping(ProcCache& pc, std::map<std::string, Mapping>::iterator it) {
    (void)hipIpcCloseMemHandle(it->second.base);
    pc.open_bytes -= it->second.bytes;
    const std::string key = it->first;
    pc.opened.erase(it);
    for (auto o = pc.open_order.begin(); o != pc.open_order.end(); ++o)
        if (*o == key) {
            pc.open_order.erase(o);
            break;
        }
}

// Close the oldest unused mappings so that this call's imports fit under kMaxOpenMappings and the
// mappings kept from earlier calls under kMaxOpenBytes.  A mapping in use by a collective of this process
// (another communicator, another thread) is never closed.  Caller holds pc.mu.
void trim_mappings(ProcCache& pc, size_t incoming) {
    for (size_t i = 0; i < pc.open_order.size() &&
                       (pc.opened.size() + incoming > kMaxOpenMappings || pc.open_bytes > kMaxOpenBytes);) {
        auto it = pc.opened.find(pc.open_order[i]);
        if (it != pc.opened.end() && it->second.users == 0) {
            if (ipc_debug())
                std::fprintf(stderr, "[dccl ipc %d] trim: closing serial %llu at %p (%zu open, %zu bytes)\n", ::getpid(),
                             static_cast<unsigned long long>(it->second.serial), it->second.base, pc.opened.size(),
                             pc.open_bytes);
            close_mapping(pc, it);
        } else {
            ++i;
        }
    }
}

// Map a peer's export (handle, serial) once and keep it; the caller holds a use of it (users) until its
// last phase point.  The same exporter address with another serial names a new allocation that replaced a
// freed one: the old mapping (which would still show the freed buffer's contents) is closed first, so the
// open below imports the new allocation.  No collective of this process can still be using the old mapping:
// the exporter freed that allocation, which it does only after every collective on it has completed on
// every rank.  Caller holds pc.mu.
ncclResult_t import_ptr(ProcCache& pc, uint32_t peer, int64_t pid, uint64_t base, uint64_t size,
                        const unsigned char* handle, uint64_t serial, uint64_t off, unsigned char** out,
                        std::vector<std::string>* held) {
    // the key is the exporter's process and allocation address, not the handle bytes: a new allocation at a
    // freed one's address is the same key with another serial whatever its handle bytes, so the freed
    // allocation's mapping is closed before the new one is opened (the runtime may otherwise hand back its
    // import of that address)
    std::string key(reinterpret_cast<const char*>(&pid), sizeof(pid));
    key.append(reinterpret_cast<const char*>(&base), sizeof(base));
    uint64_t stale_id = 0;
    auto it = pc.opened.find(key);
    if (it != pc.opened.end() && it->second.serial != serial) {
        if (ipc_debug())
            std::fprintf(stderr, "[dccl ipc %d] peer %u: handle repeats with serial %llu (mapped: %llu, users %u), "
                         "remapping\n", ::getpid(), peer, static_cast<unsigned long long>(serial),
                         static_cast<unsigned long long>(it->second.serial), it->second.users);
        if (it->second.users != 0) return dccl::ncclInternalError;  // see above: cannot happen
        stale_id = it->second.import_id;
        close_mapping(pc, it);
        it = pc.opened.end();
    }
    if (it == pc.opened.end()) {
        hipIpcMemHandle_t h;
        std::memcpy(&h, handle, kHandleBytes);
        void* mapped = nullptr;
        // Re-opening an address whose previous mapping was closed just above races with the runtime's
        // release of the old import: the open can fail for a moment (hipErrorInvalidDevicePointer, about
        // one call in six in tests/test_direct.py::test_ipc_reallocated_buffers).  It is retried with
        // backoff for ~0.5 s, and so is an open that hands back the closed import itself (the same runtime
        // buffer id; never seen in tools/ipc_churn_stress.py runs, checked because it would be silent).
        for (int attempt = 0, us = 100;; ++attempt, us = std::min(2 * us, 100000)) {
            hipError_t e = hipIpcOpenMemHandle(&mapped, h, hipIpcMemLazyEnablePeerAccess);
            if (e == hipSuccess && stale_id != 0 && buffer_id_of(mapped) == stale_id) {
                (void)hipIpcCloseMemHandle(mapped);
                e = hipErrorInvalidHandle;  // the old import again: not ours to use
            }
            if (e == hipSuccess) {  // an import of another size is another allocation: not ours either
                hipDeviceptr_t mb = nullptr;
                size_t got = 0;
                if (hipMemGetAddressRange(&mb, &got, mapped) == hipSuccess && got != size) {
                    if (ipc_debug())
                        std::fprintf(stderr, "[dccl ipc %d] peer %u: import of serial %llu is %zu bytes, not %llu\n",
                                     ::getpid(), peer, static_cast<unsigned long long>(serial), got,
                                     static_cast<unsigned long long>(size));
                    (void)hipIpcCloseMemHandle(mapped);
                    e = hipErrorInvalidHandle;
                }
            }
            if (e == hipSuccess) break;
            (void)hipGetLastError();
            if (ipc_debug())
                std::fprintf(stderr, "[dccl ipc %d] peer %u: hipIpcOpenMemHandle(serial %llu) -> %d (attempt %d)\n",
                             ::getpid(), peer, static_cast<unsigned long long>(serial), int(e), attempt);
            if (attempt == 14) return dccl::ncclUnhandledCudaError;
            std::this_thread::sleep_for(std::chrono::microseconds(us));
        }
        hipDeviceptr_t mb = nullptr;
        size_t bytes = 0;
        if (hipMemGetAddressRange(&mb, &bytes, mapped) != hipSuccess) {
            (void)hipGetLastError();
            bytes = 0;  // not counted against kMaxOpenBytes
        }
        pc.open_bytes += bytes;
        it = pc.opened.emplace(key, Mapping{mapped, serial, bytes, 0, buffer_id_of(mapped)}).first;
        pc.open_order.push_back(key);
        if (ipc_debug())
            std::fprintf(stderr, "[dccl ipc %d] peer %u: opened serial %llu at %p (%zu bytes, %zu mapped, import %llu, "
                         "replaced %llu)\n", ::getpid(), peer, static_cast<unsigned long long>(serial), mapped, bytes,
                         pc.open_bytes, static_cast<unsigned long long>(it->second.import_id),
                         static_cast<unsigned long long>(stale_id));
    }
    ++it->second.users;
    held->push_back(key);
    *out = static_cast<unsigned char*>(it->second.base) + off;
    return dccl::ncclSuccess;
}

// Peer addresses of one collective's two buffers, own rank included.  On the IPC transport it holds a use
// of every peer mapping it resolved, released when the collective returns (after its last phase point).
struct Peers {
    std::vector<const unsigned char*> in;
    std::vector<unsigned char*> out;
    std::vector<std::string> held;
    Peers() = default;
    Peers(const Peers&) = delete;
    Peers& operator=(const Peers&) = delete;
    ~Peers() {
        if (held.empty()) return;
        ProcCache& pc = cache();
        std::lock_guard<std::mutex> lock(pc.mu);
        for (const std::string& k : held) {
            auto it = pc.opened.find(k);
            if (it != pc.opened.end() && it->second.users > 0) --it->second.users;
        }
    }
};

// A phase point of a direct collective: this rank's stream has drained (its inputs / outputs are
// complete) and every rank got here.  It agrees on success: a rank whose step failed (rc) still comes
// here, and every rank returns an error from the same phase point if any rank failed, so no rank is
// left waiting at a later barrier and no rank goes on to read a peer's unfinished chunk.
ncclResult_t arrive(dcclComm* c, hipStream_t st, ncclResult_t rc = dccl::ncclSuccess) {
    if (hipStreamSynchronize(st) != hipSuccess) {  // drained even after a failed launch: peers' reads end
        (void)hipGetLastError();
        if (rc == dccl::ncclSuccess) rc = dccl::ncclUnhandledCudaError;
    }
    const bool ok = rc == dccl::ncclSuccess;
    const ncclResult_t all = c->ipc ? shm_barrier(xport(c), ok)
                                    : (c->group->barrier(ok) ? dccl::ncclSuccess : dccl::ncclRemoteError);
    return ok ? all : rc;
}

// Publish (in, out), meet every rank, then resolve every rank's (in, out) in this process.  *met is
// false when the meeting itself failed (every rank sees that and returns); when it is true, a non-success
// return is this rank's own failure to map a peer, which the caller carries into its next phase point.
ncclResult_t exchange(dcclComm* c, const void* in, void* out, hipStream_t st, Peers* P, bool* met) {
    const uint32_t W = c->world, r = c->rank;
    P->in.assign(W, nullptr);
    P->out.assign(W, nullptr);
    ncclResult_t rc = dccl::ncclSuccess;
    if (c->ipc) {
        ShmSlot& s = xport(c)->ctl->slot[r];
        s.pid = ::getpid();
        rc = export_ptr(in, s.h_in, &s.off_in, &s.serial_in, &s.base_in, &s.size_in);
        if (rc == dccl::ncclSuccess)
            rc = export_ptr(out, s.h_out, &s.off_out, &s.serial_out, &s.base_out, &s.size_out);
    } else {
        c->group->pub_in[r] = in;
        c->group->pub_out[r] = out;
    }
    rc = arrive(c, st, rc);
    *met = rc == dccl::ncclSuccess;
    if (!*met) return rc;
    ProcCache& pc = cache();
    std::unique_lock<std::mutex> lock(pc.mu, std::defer_lock);
    if (c->ipc) {
        lock.lock();
        trim_mappings(pc, 2 * size_t(W));
    }
    for (uint32_t p = 0; p < W; ++p) {
        if (p == r) {
            P->in[p] = static_cast<const unsigned char*>(in);
            P->out[p] = static_cast<unsigned char*>(out);
        } else if (c->ipc) {
            const ShmSlot& s = xport(c)->ctl->slot[p];
            unsigned char* pi = nullptr;
            unsigned char* po = nullptr;
            rc = import_ptr(pc, p, s.pid, s.base_in, s.size_in, s.h_in, s.serial_in, s.off_in, &pi, &P->held);
            if (rc == dccl::ncclSuccess)
                rc = import_ptr(pc, p, s.pid, s.base_out, s.size_out, s.h_out, s.serial_out, s.off_out, &po,
                                &P->held);
            if (rc != dccl::ncclSuccess) return rc;
            P->in[p] = pi;
            P->out[p] = po;
        } else {
            P->in[p] = static_cast<const unsigned char*>(c->group->pub_in[p]);
            P->out[p] = static_cast<unsigned char*>(c->group->pub_out[p]);
        }
    }
    return dccl::ncclSuccess;
}

// dst = the ring's combine chain for one chunk: contributions of ranks first, first+1, ...,
// first+W-2 (their `in` buffers at byte offset `off`), then `own` last.
ncclResult_t chain(const Peers& P, uint32_t W, uint32_t first, size_t off, const void* own, void* dst, size_t elems,
                   int dtype, int op, hipStream_t st, uint32_t rank) {
    if (fault_injected("direct_combine", rank)) return dccl::ncclUnhandledCudaError;
    const void* sends[kDirectMaxWorld];
    for (uint32_t j = 0; j + 1 < W; ++j) sends[j] = P.in[(first + j) % W] + off;
    return static_cast<ncclResult_t>(
        dccl_local_reduce_chain(sends, int(W - 1), own, dst, dtype, elems, op, static_cast<void*>(st)));
}

ncclResult_t copy_pairs(const std::vector<const void*>& src, const std::vector<void*>& dst, size_t bytes,
                        hipStream_t st) {
    return static_cast<ncclResult_t>(dccl_copy_multi(src.data(), dst.data(), int(src.size()), bytes, st));
}

}  // namespace

ncclResult_t ipc_join(dcclComm* c, uint32_t world, uint32_t rank) {
    if (world == 0 || world > kMaxRanks || rank >= world) return dccl::ncclInvalidArgument;
    if (hipGetDevice(&c->device) != hipSuccess) {
        (void)hipGetLastError();
        return dccl::ncclUnhandledCudaError;
    }
    // rendezvous file stamped by a live rank 0 (bootstrap.hpp): a name an earlier job left behind is never
    // taken, so no rank maps a stale segment
    const std::string path = rdv_path("dccl_ipc_name_");
    std::string name;
    int fd = -1;
    if (rank == 0) {
        std::random_device rd;
        name = "/dccl_ipc_" + std::to_string(::getpid()) + "_" + std::to_string(rd());
        fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, sizeof(ShmCtl)) != 0) {
            if (fd >= 0) {
                ::close(fd);
                shm_unlink(name.c_str());
            }
            return dccl::ncclSystemError;
        }
    } else {
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(rdv_timeout_s());
        while (fd < 0) {
            const double left = std::chrono::duration<double>(deadline - std::chrono::steady_clock::now()).count();
            if (left <= 0 || rdv_read(path, world, rank, left, &name) != dccl::ncclSuccess) return dccl::ncclSystemError;
            fd = shm_open(name.c_str(), O_RDWR, 0600);
            if (fd < 0) std::this_thread::sleep_for(std::chrono::milliseconds(10));
        }
    }
    void* m = mmap(nullptr, sizeof(ShmCtl), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) {
        if (rank == 0) shm_unlink(name.c_str());
        return dccl::ncclSystemError;
    }
    auto* ctl = static_cast<ShmCtl*>(m);
    if (rank == 0) {
        std::memset(m, 0, sizeof(ShmCtl));  // fresh segment; atomics are plain words here
        ctl->world = world;
        ctl->magic.store(kMagic, std::memory_order_release);
        if (rdv_publish(path, world, name) != dccl::ncclSuccess) {
            munmap(m, sizeof(ShmCtl));
            shm_unlink(name.c_str());
            return dccl::ncclSystemError;
        }
    } else {
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(120);
        while (ctl->magic.load(std::memory_order_acquire) != kMagic) {
            if (std::chrono::steady_clock::now() > deadline) {
                munmap(m, sizeof(ShmCtl));
                return dccl::ncclSystemError;
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
        if (ctl->world != world) {
            munmap(m, sizeof(ShmCtl));
            return dccl::ncclInvalidUsage;
        }
    }
    auto* x = new IpcXport;
    x->ctl = ctl;
    if (const char* t = std::getenv("DCCL_IPC_TIMEOUT_S")) x->timeout_s = std::strtod(t, nullptr);
    ctl->joined.fetch_add(1);
    {
        std::lock_guard<std::mutex> lock(cache().mu);
        ++cache().comms;
    }
    c->ipc = x;
    c->rank = rank;
    c->world = world;
    const ncclResult_t rc = shm_barrier(x);  // everyone mapped the segment
    if (rc == dccl::ncclSuccess && rank == 0) {   // nothing left to find by name
        shm_unlink(name.c_str());
        rdv_remove(path);
    }
    return rc;
}

ncclResult_t ipc_leave(dcclComm* c) {
    IpcXport* x = xport(c);
    if (x == nullptr) return dccl::ncclInvalidArgument;
    const ncclResult_t rc = shm_barrier(x);  // no peer still reads our buffers
    {
        // the last IPC communicator of the process releases the peer mappings (and with them the peers'
        // freed allocations they kept alive)
        ProcCache& pc = cache();
        std::lock_guard<std::mutex> lock(pc.mu);
        if (pc.comms > 0 && --pc.comms == 0) {
            for (auto it = pc.opened.begin(); it != pc.opened.end();) {
                auto next = std::next(it);
                if (it->second.users == 0) close_mapping(pc, it);
                it = next;
            }
        }
    }
    munmap(x->ctl, sizeof(ShmCtl));
    delete x;
    c->ipc = nullptr;
    return rc;
}

// In-process groups take the direct collectives for device buffers unless DCCL_ALLREDUCE_ALGORITHM names
// another algorithm: "direct", "auto" and unset select them.  They are faster than the ring at every
// size measured (4 ranks, 1024 floats 199 -> 66 us; 8 ranks 992 -> 108 us) and give
// the ring's results bit for bit.  Host buffers, the RCCL transport and groups above 8 ranks keep the ring.
bool direct_selected(const dcclComm* c) {
    if (c->ipc != nullptr) return true;
    if (c->p2p != nullptr || c->world > kDirectMaxWorld) return false;
    const char* a = std::getenv("DCCL_ALLREDUCE_ALGORITHM");
    if (a == nullptr || *a == 0) return true;
    const std::string s(a);
    return s == "auto" || s == "direct";
}

// ncclAllReduce: the ring all-reduce (all_reduce_ring.cpp:8-79) leaves chunk r+1 reduced on rank r;
// here rank r reduces that chunk from every rank's input in the ring's order, then pulls every other
// chunk from the rank that reduced it.
ncclResult_t direct_all_reduce(dcclComm* c, const void* send, void* recv, size_t count, int dtype, int op,
                               hipStream_t st) {
    const uint32_t W = c->world, r = c->rank;
    if (W > kDirectMaxWorld) return dccl::ncclInvalidUsage;
    const size_t esz = size_of_dtype(dtype), slot_elems = count / W, slot = slot_elems * esz;
    Peers P;
    bool met = false;
    ncclResult_t rc = exchange(c, send, recv, st, &P, &met);
    if (!met) return rc;
    const uint32_t mine = (r + 1) % W;
    if (rc == dccl::ncclSuccess)
        rc = chain(P, W, mine, mine * slot, P.in[r] + mine * slot, P.out[r] + mine * slot, slot_elems, dtype, op, st, r);
    if ((rc = arrive(c, st, rc)) != dccl::ncclSuccess) return rc;  // every chunk reduced by its owner
    std::vector<const void*> src;
    std::vector<void*> dst;
    for (uint32_t k = 0; k < W; ++k) {
        if (k == mine) continue;
        src.push_back(P.out[(k + W - 1) % W] + k * slot);  // chunk k lives on rank k-1
        dst.push_back(P.out[r] + k * slot);
    }
    return arrive(c, st, copy_pairs(src, dst, slot, st));  // peers are done reading our buffers
}

bool host_direct_selected(const dcclComm* c, size_t slot_bytes) {
    (void)slot_bytes;  // any size: dccl_local_reduce_chain_host stages in pieces
    if (c->ipc != nullptr || c->p2p != nullptr || c->group == nullptr || c->world > kDirectMaxWorld) return false;
    const char* a = std::getenv("DCCL_ALLREDUCE_ALGORITHM");
    if (a == nullptr || *a == 0) return true;
    const std::string s(a);
    return s == "auto" || s == "direct";
}

// The same choreography as direct_all_reduce on host memory: rank r reduces chunk r+1 from every rank's
// input in the ring's order with one staged chain kernel (one GPU round trip instead of the ring's W-1),
// then copies every other chunk from the rank that reduced it.  Every barrier is reached even after a
// failed combine, and the barrier after the combine agrees on success: if any rank failed, nobody copies
// a chunk (it could be unreduced) and every rank returns an error.
ncclResult_t direct_all_reduce_host(dcclComm* c, const void* send, void* recv, size_t count, int dtype, int op) {
    const uint32_t W = c->world, r = c->rank;
    const size_t esz = size_of_dtype(dtype), slot_elems = count / W, slot = slot_elems * esz;
    Group& g = *c->group;
    g.pub_in[r] = send;
    g.pub_out[r] = recv;
    g.barrier();  // every rank's buffers are published and its inputs are final
    const uint32_t mine = (r + 1) % W;
    const void* sends[kDirectMaxWorld];
    for (uint32_t j = 0; j + 1 < W; ++j)
        sends[j] = static_cast<const unsigned char*>(g.pub_in[(mine + j) % W]) + mine * slot;
    const ncclResult_t rc = fault_injected("direct_combine", r)
                                ? dccl::ncclUnhandledCudaError
                                : static_cast<ncclResult_t>(dccl_local_reduce_chain_host(
                                      sends, int(W - 1), static_cast<const unsigned char*>(send) + mine * slot,
                                      static_cast<unsigned char*>(recv) + mine * slot, dtype, slot_elems, op));
    const bool all = g.barrier(rc == dccl::ncclSuccess);  // every chunk reduced by its owner
    if (all)
        for (uint32_t k = 0; k < W; ++k)
            if (k != mine)  // chunk k lives on rank k-1
                std::memcpy(static_cast<unsigned char*>(recv) + k * slot,
                            static_cast<const unsigned char*>(g.pub_out[(k + W - 1) % W]) + k * slot, slot);
    g.barrier();  // peers are done reading our buffers
    return rc != dccl::ncclSuccess ? rc : (all ? dccl::ncclSuccess : dccl::ncclRemoteError);
}

// ncclReduceScatter on host memory: slot r reduced from every rank's input in the order of the ring with
// ncclReduceScatter's maps (as direct_reduce_scatter), one staged chain combine.
ncclResult_t direct_reduce_scatter_host(dcclComm* c, const void* send, void* recv, size_t recvcount, int dtype,
                                        int op) {
    const uint32_t W = c->world, r = c->rank;
    const size_t slot = recvcount * size_of_dtype(dtype);
    Group& g = *c->group;
    g.pub_in[r] = send;
    g.pub_out[r] = recv;
    g.barrier();
    const void* sends[kDirectMaxWorld];
    for (uint32_t j = 0; j + 1 < W; ++j)
        sends[j] = static_cast<const unsigned char*>(g.pub_in[(r + 1 + j) % W]) + r * slot;
    const ncclResult_t rc = fault_injected("direct_combine", r)
                                ? dccl::ncclUnhandledCudaError
                                : static_cast<ncclResult_t>(dccl_local_reduce_chain_host(
                                      sends, int(W - 1), static_cast<const unsigned char*>(send) + r * slot, recv,
                                      dtype, recvcount, op));
    const bool all = g.barrier(rc == dccl::ncclSuccess);  // peers are done reading our input
    return rc != dccl::ncclSuccess ? rc : (all ? dccl::ncclSuccess : dccl::ncclRemoteError);
}

// ncclReduceScatter: the ring with rank maps (o+W-1)%W / (n+1)%W (dccl.cpp:551-698) leaves slot o on
// rank o, combined in the order o+1, o+2, ..., o-1, o.
ncclResult_t direct_reduce_scatter(dcclComm* c, const void* send, void* recv, size_t recvcount, int dtype, int op,
                                   hipStream_t st) {
    const uint32_t W = c->world, r = c->rank;
    if (W > kDirectMaxWorld) return dccl::ncclInvalidUsage;
    const size_t slot = recvcount * size_of_dtype(dtype);
    Peers P;
    bool met = false;
    ncclResult_t rc = exchange(c, send, recv, st, &P, &met);
    if (!met) return rc;
    if (rc == dccl::ncclSuccess) rc = chain(P, W, (r + 1) % W, r * slot, P.in[r] + r * slot, recv, recvcount, dtype, op, st, r);
    return arrive(c, st, rc);
}

// ncclReduce: the reference runs the reduce-scatter ring with the same maps, then gathers the slots
// at the root (dccl.cpp:745-846); here the root reduces every slot itself.
ncclResult_t direct_reduce(dcclComm* c, const void* send, void* recv, size_t count, int dtype, int op, uint32_t root,
                           hipStream_t st) {
    const uint32_t W = c->world, r = c->rank;
    if (W > kDirectMaxWorld) return dccl::ncclInvalidUsage;
    const size_t slot_elems = count / W, slot = slot_elems * size_of_dtype(dtype);
    Peers P;
    bool met = false;
    ncclResult_t rc = exchange(c, send, r == root ? recv : const_cast<void*>(send), st, &P, &met);
    if (!met) return rc;
    if (r == root)
        for (uint32_t o = 0; o < W && rc == dccl::ncclSuccess; ++o)
            rc = chain(P, W, (o + 1) % W, o * slot, P.in[o] + o * slot, P.out[r] + o * slot, slot_elems, dtype, op,
                       st, r);
    return arrive(c, st, rc);
}

ncclResult_t direct_all_gather(dcclComm* c, const void* send, void* recv, size_t sendcount, int dtype,
                               hipStream_t st) {
    const uint32_t W = c->world, r = c->rank;
    if (W > kDirectMaxWorld) return dccl::ncclInvalidUsage;
    const size_t slot = sendcount * size_of_dtype(dtype);
    Peers P;
    bool met = false;
    ncclResult_t rc = exchange(c, send, recv, st, &P, &met);
    if (!met) return rc;
    if (rc == dccl::ncclSuccess) {
        std::vector<const void*> src;
        std::vector<void*> dst;
        for (uint32_t p = 0; p < W; ++p) {
            if (p == r && P.in[r] == P.out[r] + r * slot) continue;  // already in place
            src.push_back(P.in[p]);
            dst.push_back(P.out[r] + p * slot);
        }
        rc = copy_pairs(src, dst, slot, st);
    }
    return arrive(c, st, rc);
}

ncclResult_t direct_broadcast(dcclComm* c, const void* send, void* recv, size_t count, int dtype, uint32_t root,
                              hipStream_t st) {
    const uint32_t r = c->rank;
    const size_t bytes = count * size_of_dtype(dtype);
    Peers P;
    bool met = false;
    ncclResult_t rc = exchange(c, r == root ? send : recv, recv, st, &P, &met);
    if (!met) return rc;
    if (rc == dccl::ncclSuccess && P.in[root] != P.out[r]) {
        std::vector<const void*> src{P.in[root]};
        std::vector<void*> dst{P.out[r]};
        rc = copy_pairs(src, dst, bytes, st);
    }
    return arrive(c, st, rc);
}

}  // namespace dccl_amd
