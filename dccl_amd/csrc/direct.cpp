// dccl_amd/csrc/direct.cpp — see direct.hpp.
#include "direct.hpp"

#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
#include "ipc_cache.hpp"

namespace dccl_amd {
namespace {

using dccl::dcclComm;

constexpr uint64_t kMagic = 0x3243504943434344ull;  // "DCCIPC2"
constexpr uint32_t kMaxRanks = 64;
constexpr size_t kHandleBytes = ipc::kHandleBytes;
static_assert(sizeof(hipIpcMemHandle_t) == kHandleBytes, "HIP IPC handle size");
// Peer mappings kept for later calls (one cache per process, ipc_cache.hpp): the oldest unused one is
// closed beyond this many, or beyond this many bytes of peer memory (a mapping keeps the peer's pages alive).
constexpr size_t kMaxOpenMappings = 256;
constexpr size_t kMaxOpenBytes = size_t(64) << 30;
// Exports this rank ended and its peers have not necessarily seen yet (see ShmSlot::retired).
constexpr uint32_t kRetireRing = 256;
// The communicator's scratch (every input is copied there for the peers to read): at least the
// reference's initial scratchpad (SCRATCHPAD_INI_SIZE, /root/reference/src/core/dccl.cpp:57), in 2 MiB
// pages, grown by at least half when it grows.
constexpr size_t kScratchMin = size_t(64) << 20;
constexpr size_t kScratchPage = size_t(2) << 20;
// The first bytes of every scratch hold a random 128-bit token that the exporter publishes with it; a peer
// reads it through a new mapping before trusting the mapping (import_desc).  Data starts after the header.
constexpr size_t kScratchHeader = 256;

// One published buffer: the export holding it (serial 0: nothing published) and the offset in it.
struct Desc {
    unsigned char handle[kHandleBytes];
    uint64_t serial, off, size;  // size: of the exported allocation
    uint64_t token[2];           // the scratch's token at its first bytes (never 0, 0)
};

struct ShmSlot {
    Desc in, out;
    int64_t pid;     // this rank's process and its start time (bootstrap.hpp), for the barrier's liveness check
    uint64_t start;
    // Exports this rank's process ended (replaced scratch, finalized communicator): serials in a
    // ring, retired_n written last.  Every peer closes their mappings before it opens anything new.
    std::atomic<uint64_t> retired_n;
    uint64_t retired[kRetireRing];
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

// An allocation of this process that peers may map: a communicator's scratch buffer (peers never read user
// memory).  `serial` numbers this process's exports and is never reused, whatever the runtime's handle bytes do.
struct Export {
    size_t size;
    uint64_t buffer_id;
    uint64_t serial;
    ipc::Handle handle;
    bool fresh;  // its handle bytes never named another allocation of this process (see make_export)
};

// A device range registered with dcclRegisterCacheMemory: tracked only (round 5: peers read every input through
// the verified scratch, so a registration exports nothing).
struct Range {
    size_t len;
    uint32_t refs;  // registrations of this start address (e.g. one per communicator)
};

struct IpcXport {
    ShmCtl* ctl = nullptr;
    uint32_t rank = 0, world = 0;
    double timeout_s = 0;  // barrier wait limit, 0: none (set by ipc_join; a dead peer is caught by the liveness check)
    bool liveness = true;   // peers' pids are visible here (checked at join)
    // scratch: every input is copied here (one allocation, exported once)
    void* scratch = nullptr;        // allocation base: header (token), then scratch_bytes of data
    size_t scratch_bytes = 0;
    uint64_t token[2] = {0, 0};
    std::vector<void*> old_scratch;  // replaced buffers, freed at this rank's next collective
    std::vector<uint64_t> seen;      // retirements of each peer already applied
};

uint64_t buffer_id_of(const void* p) {
    uint64_t id = 0;
    if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID,
                               reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(p))) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return id;
}

struct HipOps final : ipc::Ops {
    bool open(const ipc::Handle& h, void** mapped) override {
        hipIpcMemHandle_t hh;
        std::memcpy(&hh, h.b, kHandleBytes);
        if (hipIpcOpenMemHandle(mapped, hh, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        return true;
    }
    void close(void* mapped) override {
        if (hipIpcCloseMemHandle(mapped) != hipSuccess) (void)hipGetLastError();
    }
    size_t size_of(void* mapped) override {
        hipDeviceptr_t b = nullptr;
        size_t s = 0;
        if (hipMemGetAddressRange(&b, &s, mapped) != hipSuccess) {
            (void)hipGetLastError();
            return 0;
        }
        return s;
    }
};

// Exports, registrations and peer mappings are per PROCESS, shared by its IPC communicators: the runtime
// hands out one import per handle per process, so one communicator's stale mapping would shadow another's.
struct ProcCache {
    std::mutex mu;
    uint64_t next_serial = 1;
    std::map<uintptr_t, Export> exports;  // allocation base -> export
    std::map<uintptr_t, Range> ranges;    // registered device range start -> range (tracked only)
    HipOps ops;
    ipc::ImportCache imports{&ops, kMaxOpenMappings, kMaxOpenBytes};
    std::vector<IpcXport*> xports;  // live IPC communicators of this process
    // read_token's 16 device bytes and stream, per device (a mapping belongs to the device it was opened on)
    std::map<int, std::pair<void*, hipStream_t>> token_io;
    // handle bytes of every export this process made -> the buffer id of the allocation they named
    std::map<std::string, uint64_t> handle_owner;
    // exporter-side counters (dccl_ipc_stats)
    uint64_t exports_made = 0, retirements = 0, scratch_copies = 0, scratch_bytes = 0, scratch_grows = 0,
             recycled_handles = 0;
};

ProcCache& cache() {
    static ProcCache* c = [] {
        auto* p = new ProcCache;  // never destroyed: communicators may outlive static destructors
        return p;
    }();
    return *c;
}

IpcXport* xport(const dcclComm* c) { return static_cast<IpcXport*>(c->ipc); }

// DCCL_IPC_DEBUG=1: one line on stderr per export made or retired (read once per process)
bool ipc_debug() {
    static const bool on = [] {
        const char* v = std::getenv("DCCL_IPC_DEBUG");
        return v != nullptr && *v == '1';
    }();
    return on;
}

// DCCL_IPC_LIVENESS=0 turns the liveness check off for every communicator of the process.
bool liveness_requested() {
    static const bool on = [] {
        const char* v = std::getenv("DCCL_IPC_LIVENESS");
        return v == nullptr || *v != '0';
    }();
    return on;
}

// False once peer p's process is gone (or its pid names another process now).
bool peer_alive(const ShmSlot& s) {
    if (s.pid <= 0) return true;  // not joined yet
    if (::kill(static_cast<pid_t>(s.pid), 0) != 0 && errno == ESRCH) return false;
    return proc_start_time(static_cast<long>(s.pid)) == s.start;  // 0 for a zombie (exited, not reaped)
}

// Apply every retirement the peers of every IPC communicator of this process wrote since the last call.
void apply_retirements(ProcCache& pc) {
    for (IpcXport* x : pc.xports) {
        for (uint32_t p = 0; p < x->world; ++p) {
            if (p == x->rank) continue;
            const ShmSlot& s = x->ctl->slot[p];
            const uint64_t n = s.retired_n.load(std::memory_order_acquire);
            uint64_t& seen = x->seen[p];
            if (n == seen) continue;
            if (n - seen > kRetireRing) {
                pc.imports.retire_pid(s.pid);
            } else {
                for (uint64_t i = seen; i < n; ++i) pc.imports.retire(s.pid, s.retired[i % kRetireRing]);
                // the writer may have lapped the ring while it was read
                if (s.retired_n.load(std::memory_order_acquire) - seen > kRetireRing) pc.imports.retire_pid(s.pid);
            }
            seen = n;
        }
    }
}

// Sense-reversing barrier on the shared counters that also agrees on success: a rank arriving with
// ok == false raises the segment's abort flag, and every rank returns ncclRemoteError from a barrier that
// completes with the flag up.  The flag is sticky (the transport is unusable after a failed collective,
// like an aborted NCCL communicator).  A waiter checks every ~100 ms that its peers' processes still
// exist, so a peer that died (a runtime abort, a kill) ends every other rank's wait with ncclRemoteError
// at once.  A live peer may take up to 30 minutes between collectives (a checkpoint, an evaluation);
// DCCL_IPC_TIMEOUT_S sets another limit (0: none); with the liveness check off the limit is 300 s.
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
    // added, which set the latency of small collectives.
    constexpr auto kSpin = std::chrono::milliseconds(2);
    constexpr auto kLiveness = std::chrono::milliseconds(100);
    const auto start = std::chrono::steady_clock::now();
    const bool limited = x->timeout_s > 0;
    const auto deadline = start + std::chrono::duration<double>(limited ? x->timeout_s : 0.0);
    auto next_check = start + kLiveness;
    for (uint64_t i = 0; s->gen.load(std::memory_order_acquire) == g; ++i) {
        if (s->abort.load(std::memory_order_relaxed)) return dccl::ncclRemoteError;
        if ((i & 1023) != 1023) {
            __builtin_ia32_pause();
            continue;
        }
        const auto now = std::chrono::steady_clock::now();
        if (limited && now > deadline) {
            s->abort.store(1, std::memory_order_relaxed);
            return dccl::ncclSystemError;
        }
        if (x->liveness && now > next_check) {
            next_check = now + kLiveness;
            for (uint32_t p = 0; p < s->world; ++p)
                if (p != x->rank && !peer_alive(s->slot[p])) {
                    if (ipc_debug()) std::fprintf(stderr, "[dccl ipc %d] rank %u's process is gone\n", ::getpid(), p);
                    s->abort.store(1, std::memory_order_relaxed);
                    return dccl::ncclRemoteError;
                }
        }
        if (now - start > kSpin) std::this_thread::sleep_for(std::chrono::microseconds(20));
        else std::this_thread::yield();  // a peer without a core of its own gets one
    }
    return s->abort.load(std::memory_order_relaxed) ? dccl::ncclRemoteError : dccl::ncclSuccess;
}

// --- exporter side (caller holds pc.mu) ---------------------------------------------------------------

// Tell every peer of every IPC communicator of this process that export `serial` ended.
void write_retirement(ProcCache& pc, uint64_t serial) {
    ++pc.retirements;
    for (IpcXport* x : pc.xports) {
        ShmSlot& s = x->ctl->slot[x->rank];
        const uint64_t n = s.retired_n.load(std::memory_order_relaxed);
        s.retired[n % kRetireRing] = serial;
        s.retired_n.store(n + 1, std::memory_order_release);
    }
    if (ipc_debug()) std::fprintf(stderr, "[dccl ipc %d] retired serial %llu\n", ::getpid(), (unsigned long long)serial);
}

void drop_export(ProcCache& pc, std::map<uintptr_t, Export>::iterator it) {
    write_retirement(pc, it->second.serial);
    pc.exports.erase(it);
}

// Export the allocation [base, base + size) with buffer id `id`; exports whose range it overlaps name
// freed allocations and are retired.
ncclResult_t make_export(ProcCache& pc, uintptr_t base, size_t size, uint64_t id) {
    for (auto o = pc.exports.lower_bound(base); o != pc.exports.begin();) {
        --o;
        if (o->first + o->second.size <= base) break;
        drop_export(pc, o);
        o = pc.exports.lower_bound(base);
    }
    for (auto o = pc.exports.lower_bound(base); o != pc.exports.end() && o->first < base + size;
         o = pc.exports.lower_bound(base))
        drop_export(pc, o);
    Export e{size, id, pc.next_serial++, {}, true};
    hipIpcMemHandle_t h;
    // exporting an allocation at the address of a freed one that a peer still maps can fail for a moment
    for (int attempt = 0, us = 100;; ++attempt, us = std::min(2 * us, 100000)) {
        if (hipIpcGetMemHandle(&h, reinterpret_cast<void*>(base)) == hipSuccess) break;
        (void)hipGetLastError();
        if (attempt == 14) return dccl::ncclUnhandledCudaError;
        std::this_thread::sleep_for(std::chrono::microseconds(us));
    }
    std::memcpy(e.handle.b, &h, kHandleBytes);
    // Handle bytes that already named another (freed) allocation of this process are never published: a peer
    // that mapped them once and opens them again can be handed the earlier import's pages by the runtime,
    // even after it closed that mapping (registered-buffer churn read stale data in 6 of 6
    // runs at W = 2 although every mapping was closed before the new open).  Such an export stays unused
    // (`fresh` false): the scratch is allocated again.
    // Without a buffer id, or past a bound on the table, nothing counts as fresh.
    const std::string key(reinterpret_cast<const char*>(e.handle.b), kHandleBytes);
    auto owner = pc.handle_owner.find(key);
    if (owner != pc.handle_owner.end()) {
        e.fresh = id != 0 && owner->second == id;
        owner->second = id;
    } else if (pc.handle_owner.size() < (size_t(1) << 20)) {
        pc.handle_owner.emplace(key, id);
        e.fresh = id != 0;
    } else {
        e.fresh = false;
    }
    if (!e.fresh) ++pc.recycled_handles;
    pc.exports.emplace(base, e);
    ++pc.exports_made;
    if (ipc_debug())
        std::fprintf(stderr, "[dccl ipc %d] export base=%#zx size=%zu buffer_id=%llu serial=%llu%s\n", ::getpid(),
                     size_t(base), size, (unsigned long long)id, (unsigned long long)e.serial,
                     e.fresh ? "" : " (recycled handle: not published)");
    return dccl::ncclSuccess;
}

void describe(const Export& e, uintptr_t base, const void* p, const uint64_t* token, Desc* d) {
    std::memcpy(d->handle, e.handle.b, kHandleBytes);
    d->serial = e.serial;
    d->off = reinterpret_cast<uintptr_t>(p) - base;
    d->size = e.size;
    d->token[0] = token[0];
    d->token[1] = token[1];
}

// Make the communicator's scratch hold at least `bytes`.  A replaced buffer is retired now and freed at
// this rank's next collective, after every peer passed this collective's exchange (and closed it).
ncclResult_t ensure_ipc_scratch(ProcCache& pc, IpcXport* x, size_t bytes) {
    if (bytes <= x->scratch_bytes) return dccl::ncclSuccess;
    size_t want = std::max({bytes + kScratchHeader, x->scratch_bytes + x->scratch_bytes / 2, kScratchMin});
    want = (want + kScratchPage - 1) / kScratchPage * kScratchPage;
    // an allocation whose handle bytes are recycled (make_export) is kept until a fresh one is found, so the
    // next allocation cannot be handed the same bytes, then freed
    std::vector<void*> recycled;
    void* p = nullptr;
    ncclResult_t rc = dccl::ncclSuccess;
    for (int attempt = 0; attempt < 8; ++attempt) {
        if (hipMalloc(&p, want) != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
            rc = dccl::ncclUnhandledCudaError;
            break;
        }
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        if (hipMemGetAddressRange(&base, &size, p) != hipSuccess || base != p) {  // the export is keyed by its base
            (void)hipGetLastError();
            recycled.push_back(p);
            p = nullptr;
            rc = dccl::ncclUnhandledCudaError;
            break;
        }
        rc = make_export(pc, reinterpret_cast<uintptr_t>(base), size, buffer_id_of(base));
        if (rc != dccl::ncclSuccess) {
            recycled.push_back(p);
            p = nullptr;
            break;
        }
        auto e = pc.exports.find(reinterpret_cast<uintptr_t>(base));
        if (e->second.fresh) break;
        pc.exports.erase(e);  // never published: nothing to retire
        recycled.push_back(p);
        p = nullptr;
        rc = dccl::ncclInternalError;
    }
    for (void* q : recycled) (void)hipFree(q);
    if (p == nullptr) return rc == dccl::ncclSuccess ? dccl::ncclInternalError : rc;
    uint64_t token[2] = {0, 0};
    {
        std::random_device rd;
        for (uint64_t& t : token) t = (uint64_t(rd()) << 32) ^ rd() ^ (uint64_t(pc.next_serial) << 48);
        if (token[0] == 0 && token[1] == 0) token[1] = 1;
    }
    if (hipMemcpy(p, token, sizeof(token), hipMemcpyHostToDevice) != hipSuccess) {  // complete on return
        (void)hipGetLastError();
        auto e = pc.exports.find(reinterpret_cast<uintptr_t>(p));
        if (e != pc.exports.end()) pc.exports.erase(e);  // never published
        (void)hipFree(p);
        return dccl::ncclUnhandledCudaError;
    }
    if (x->scratch != nullptr) {
        auto old = pc.exports.find(reinterpret_cast<uintptr_t>(x->scratch));
        if (old != pc.exports.end()) drop_export(pc, old);
        x->old_scratch.push_back(x->scratch);
    }
    x->scratch = p;
    x->scratch_bytes = want - kScratchHeader;
    x->token[0] = token[0];
    x->token[1] = token[1];
    ++pc.scratch_grows;
    return dccl::ncclSuccess;
}

// --- importer side (caller holds pc.mu) ---------------------------------------------------------------

// Read a new mapping's token through a compute kernel (dccl_copy_multi into 16 device bytes, then to the
// host), i.e. through the address translation the combine kernels use, not a DMA engine's.  The round-4
// zero-copy failures were a recycled importer address reading other pages on first use.
bool read_token(ProcCache& pc, const void* mapped, uint64_t got[2]) {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    auto io = pc.token_io.find(dev);
    if (io == pc.token_io.end()) {
        void* buf = nullptr;
        hipStream_t st = nullptr;
        if (hipMalloc(&buf, 16) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipFree(buf);
            return false;
        }
        io = pc.token_io.emplace(dev, std::make_pair(buf, st)).first;
    }
    const void* src = mapped;
    void* dst = io->second.first;
    hipStream_t st = io->second.second;
    if (dccl_copy_multi(&src, &dst, 1, 16, st) != DCCL_SUCCESS ||
        hipMemcpyAsync(got, dst, 16, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return true;
}

// Peer addresses of one collective's two buffers, own rank included.  On the IPC transport it holds a use
// of every peer mapping it resolved, released when the collective returns (after its last phase point).
struct Peers {
    std::vector<const unsigned char*> in;
    std::vector<unsigned char*> out;
    std::vector<std::pair<int64_t, uint64_t>> held;
    Peers() = default;
    Peers(const Peers&) = delete;
    Peers& operator=(const Peers&) = delete;
    ~Peers() { release(); }
    // This rank no longer reads through the mappings (its stream has drained past the last kernel that did).
    void release() {
        if (held.empty()) return;
        ProcCache& pc = cache();
        std::lock_guard<std::mutex> lock(pc.mu);
        for (const auto& k : held) pc.imports.release(k.first, k.second);
        held.clear();
    }
};

ncclResult_t import_desc(ProcCache& pc, uint32_t peer, int64_t pid, const Desc& d, unsigned char** out, Peers* P) {
    if (d.serial == 0) {
        *out = nullptr;
        return dccl::ncclSuccess;
    }
    ipc::Handle h;
    std::memcpy(h.b, d.handle, kHandleBytes);
    void* base = nullptr;
    ipc::Result r = ipc::kOk;
    // A new mapping of a scratch is trusted only once its first bytes read back the token the exporter
    // published: the mapping then provably shows the exporter's allocation.  One close and re-open on a
    // mismatch, then an error (never data read through a wrong mapping).
    for (int attempt = 0; attempt < 2; ++attempt) {
        bool opened = false;
        r = pc.imports.acquire(pid, d.serial, h, d.size, &base, 15, &opened);
        if (r != ipc::kOk || !opened || (d.token[0] == 0 && d.token[1] == 0)) break;
        uint64_t got[2] = {0, 0};
        (void)read_token(pc, base, got);  // a failed read leaves {0, 0}: never a valid token
        if (got[0] == d.token[0] && got[1] == d.token[1]) break;
        ++pc.imports.stats.verify_failures;
        if (ipc_debug())
            std::fprintf(stderr, "[dccl ipc %d] peer %u serial %llu: token mismatch at %p (attempt %d)\n", ::getpid(),
                         peer, (unsigned long long)d.serial, base, attempt);
        pc.imports.release(pid, d.serial);
        pc.imports.retire(pid, d.serial);  // closes it: the next acquire opens afresh
        r = ipc::kAliasOpened;
    }
    if (r != ipc::kOk) {
        if (ipc_debug())
            std::fprintf(stderr, "[dccl ipc %d] peer %u serial %llu: import failed (%d)\n", ::getpid(), peer,
                         (unsigned long long)d.serial, int(r));
        return r == ipc::kOpenFailed ? dccl::ncclUnhandledCudaError : dccl::ncclInternalError;
    }
    P->held.emplace_back(pid, d.serial);
    *out = static_cast<unsigned char*>(base) + d.off;
    if (ipc_debug())
        std::fprintf(stderr, "[dccl ipc %d] peer %u (pid %lld) serial %llu -> %p + %llu\n", ::getpid(), peer,
                     (long long)pid, (unsigned long long)d.serial, base, (unsigned long long)d.off);
    return dccl::ncclSuccess;
}

// A phase point of a direct collective: this rank's stream has drained (its inputs / outputs are
// complete) and every rank got here.  It agrees on success: a rank whose step failed (rc) still comes
// here, and every rank returns an error from the same phase point if any rank failed, so no rank is
// left waiting at a later barrier and no rank goes on to read a peer's unfinished chunk.
// `done` (the collective's last phase point): its peer mappings are released once the stream has drained,
// before the barrier, so no use is held while this rank waits for the others (another thread's
// communicator can then retire and close them without waiting for this collective to return).
ncclResult_t arrive(dcclComm* c, hipStream_t st, ncclResult_t rc = dccl::ncclSuccess, Peers* done = nullptr) {
    if (hipStreamSynchronize(st) != hipSuccess) {  // drained even after a failed launch: peers' reads end
        (void)hipGetLastError();
        if (rc == dccl::ncclSuccess) rc = dccl::ncclUnhandledCudaError;
    }
    if (done != nullptr) done->release();
    const bool ok = rc == dccl::ncclSuccess;
    const ncclResult_t all = c->ipc ? shm_barrier(xport(c), ok)
                                    : (c->group->barrier(ok) ? dccl::ncclSuccess : dccl::ncclRemoteError);
    return ok ? all : rc;
}

// What one rank publishes for a collective: `in` (peers read it; nullptr: nothing) of in_bytes, and
// `out` (peers read the reduced chunks from it; nullptr: nothing) of out_bytes.  On the IPC transport both
// are replaced by the communicator's scratch: `in` is copied there on `st`, and `out` becomes the scratch
// itself (the caller copies the result out).
struct Publish {
    const void* in = nullptr;
    size_t in_bytes = 0;
    void* out = nullptr;
    size_t out_bytes = 0;
    bool out_scratch = false;
};

// Copy `in` into the scratch and describe it (and `out`, the scratch itself) in this rank's slot (IPC).  Peers
// only ever read the library-owned scratch, whose every new mapping they verify by its token: the round-4
// opt-in that let them read registered user buffers in place returned another allocation's data in about one
// of 1,000 first uses under registration churn, with no way to verify a user allocation, and is gone.
ncclResult_t plan_ipc(dcclComm* c, Publish* pub, hipStream_t st) {
    IpcXport* x = xport(c);
    ProcCache& pc = cache();
    std::lock_guard<std::mutex> lock(pc.mu);
    for (void* p : x->old_scratch) (void)hipFree(p);  // every peer closed them in the previous collective
    x->old_scratch.clear();
    pub->out_scratch = pub->out != nullptr;
    // `out` in the scratch shares it with `in` (the all_reduce combines in place there)
    const size_t need = std::max(pub->in ? pub->in_bytes : 0, pub->out ? pub->out_bytes : 0);
    if (need > 0) {
        const ncclResult_t rc = ensure_ipc_scratch(pc, x, need);
        if (rc != dccl::ncclSuccess) return rc;
    }
    ShmSlot& s = x->ctl->slot[x->rank];
    s.in.serial = s.out.serial = 0;
    const uintptr_t sb = reinterpret_cast<uintptr_t>(x->scratch);
    unsigned char* data = static_cast<unsigned char*>(x->scratch) + kScratchHeader;
    if (pub->in) {
        if (hipMemcpyAsync(data, pub->in, pub->in_bytes, hipMemcpyDeviceToDevice, st) != hipSuccess) {
            (void)hipGetLastError();
            return dccl::ncclUnhandledCudaError;
        }
        ++pc.scratch_copies;
        pc.scratch_bytes += pub->in_bytes;
        pub->in = data;
    }
    if (pub->out) pub->out = data;
    const auto e = pc.exports.find(sb);
    if (pub->in) describe(e->second, e->first, pub->in, x->token, &s.in);
    if (pub->out) describe(e->second, e->first, pub->out, x->token, &s.out);
    return dccl::ncclSuccess;
}

// Publish, meet every rank, then resolve every rank's (in, out) in this process.  *met is false when the
// meeting itself failed (every rank sees that and returns); when it is true, a non-success return is this
// rank's own failure to map a peer, which the caller carries into its next phase point.
ncclResult_t exchange(dcclComm* c, Publish* pub, hipStream_t st, Peers* P, bool* met) {
    const uint32_t W = c->world, r = c->rank;
    P->in.assign(W, nullptr);
    P->out.assign(W, nullptr);
    ncclResult_t rc = dccl::ncclSuccess;
    if (c->ipc) {
        rc = plan_ipc(c, pub, st);
    } else {
        c->group->pub_in[r] = pub->in;
        c->group->pub_out[r] = pub->out;
    }
    rc = arrive(c, st, rc);
    *met = rc == dccl::ncclSuccess;
    if (!*met) return rc;
    P->in[r] = static_cast<const unsigned char*>(pub->in);
    P->out[r] = static_cast<unsigned char*>(pub->out);
    if (!c->ipc) {
        for (uint32_t p = 0; p < W; ++p)
            if (p != r) {
                P->in[p] = static_cast<const unsigned char*>(c->group->pub_in[p]);
                P->out[p] = static_cast<unsigned char*>(c->group->pub_out[p]);
            }
        return dccl::ncclSuccess;
    }
    ProcCache& pc = cache();
    std::lock_guard<std::mutex> lock(pc.mu);
    apply_retirements(pc);  // before any open: a retired export's handle bytes may come back
    pc.imports.trim(2 * size_t(W));
    const ShmCtl* ctl = xport(c)->ctl;
    for (uint32_t p = 0; p < W; ++p) {
        if (p == r) continue;
        const ShmSlot& s = ctl->slot[p];
        unsigned char* pi = nullptr;
        if ((rc = import_desc(pc, p, s.pid, s.in, &pi, P)) != dccl::ncclSuccess) return rc;
        if ((rc = import_desc(pc, p, s.pid, s.out, &P->out[p], P)) != dccl::ncclSuccess) return rc;
        P->in[p] = pi;
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
    if (src.empty()) return dccl::ncclSuccess;
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
    x->rank = rank;
    x->world = world;
    x->seen.assign(world, 0);
    x->liveness = liveness_requested();
    // A live peer stuck for half an hour (a hung kernel, a blocked synchronise) ends the wait;
    // DCCL_IPC_TIMEOUT_S sets another limit, 0 none at all (ranks that may pause longer between collectives).
    x->timeout_s = 1800;
    const char* t = std::getenv("DCCL_IPC_TIMEOUT_S");
    const bool explicit_limit = t != nullptr && *t != 0;
    if (explicit_limit) {
        const double v = std::strtod(t, nullptr);
        x->timeout_s = v > 0 ? v : 0;
    }
    if (!x->liveness && (!explicit_limit || x->timeout_s <= 0)) x->timeout_s = 300;  // a dead peer ends the wait
    ShmSlot& me = ctl->slot[rank];
    me.start = proc_start_time(static_cast<long>(::getpid()));
    // tests only (DCCL_FAULT_INJECT=hidden_pid:<rank>): publish a pid no peer can see, as a rank in another pid
    // namespace would
    me.pid = fault_injected("hidden_pid", rank) ? int64_t(0x7ffffff0) : int64_t(::getpid());
    ctl->joined.fetch_add(1);
    c->ipc = x;
    c->rank = rank;
    c->world = world;
    // Everyone mapped the segment.  This wait runs with the liveness check off and bounded by the rendezvous
    // timeout: a rank may wait here for a late joiner, and a peer whose process it cannot see would
    // look dead to a check made before the visibility probe below.
    const bool live = x->liveness;
    const double limit = x->timeout_s;
    x->liveness = false;
    x->timeout_s = rdv_timeout_s();
    const ncclResult_t rc = shm_barrier(x);
    x->liveness = live;
    x->timeout_s = limit;
    // Ranks that share /dev/shm but not a pid namespace (containers with --ipc=host), or a /proc mounted with
    // hidepid, cannot see each other's processes: a live peer would look dead.  Then this communicator goes
    // without the liveness check (and with the 300 s default limit), said once.
    if (rc == dccl::ncclSuccess && x->liveness) {
        for (uint32_t p = 0; p < world; ++p)
            if (p != rank && !peer_alive(ctl->slot[p])) {
                x->liveness = false;
                if (!explicit_limit || x->timeout_s <= 0) x->timeout_s = 300;
                std::fprintf(stderr, "[dccl ipc %d] rank %u's process (pid %lld) is not visible from here: liveness "
                                     "check off for this communicator\n", ::getpid(), p, (long long)ctl->slot[p].pid);
                break;
            }
    }
    {
        // retirements written from here on reach this segment's peers (none can refer to an earlier export:
        // nothing was published here before)
        ProcCache& pc = cache();
        std::lock_guard<std::mutex> lock(pc.mu);
        for (uint32_t p = 0; p < world; ++p) x->seen[p] = ctl->slot[p].retired_n.load(std::memory_order_acquire);
        pc.xports.push_back(x);
    }
    if (rc == dccl::ncclSuccess && rank == 0) {  // nothing left to find by name
        shm_unlink(name.c_str());
        rdv_remove(path);
    }
    return rc;
}

ncclResult_t ipc_leave(dcclComm* c) {
    IpcXport* x = xport(c);
    if (x == nullptr) return dccl::ncclInvalidArgument;
    ProcCache& pc = cache();
    {
        // the scratch ends with the communicator: retire it for every peer (of this and of every other
        // communicator of this process) before the last meeting
        std::lock_guard<std::mutex> lock(pc.mu);
        if (x->scratch != nullptr) {
            auto e = pc.exports.find(reinterpret_cast<uintptr_t>(x->scratch));
            if (e != pc.exports.end()) drop_export(pc, e);
        }
    }
    ncclResult_t rc = shm_barrier(x);  // no peer still reads our buffers; every retirement is written
    {
        std::lock_guard<std::mutex> lock(pc.mu);
        apply_retirements(pc);  // close the peers' scratch mappings
        pc.xports.erase(std::remove(pc.xports.begin(), pc.xports.end(), x), pc.xports.end());
        // the last IPC communicator of the process releases every peer mapping (and with them the peers'
        // freed allocations they kept alive)
        if (pc.xports.empty()) pc.imports.close_unused();
    }
    const ncclResult_t rc2 = shm_barrier(x);  // every peer closed our scratch
    if (rc == dccl::ncclSuccess) rc = rc2;
    for (void* p : x->old_scratch) (void)hipFree(p);
    if (x->scratch) (void)hipFree(x->scratch);
    munmap(x->ctl, sizeof(ShmCtl));
    delete x;
    c->ipc = nullptr;
    return rc;
}

// dcclRegisterCacheMemory of device memory on an IPC communicator: validated (a device allocation of this
// process, the range inside it) and counted, nothing exported.  The reference registers RDMA memory for its
// transport (/root/reference/src/core/dccl.cpp:503-549); peers here read the scratch, which needs none.
ncclResult_t ipc_register(void* buffer, size_t size) {
    hipDeviceptr_t base = nullptr;
    size_t asize = 0;
    if (hipMemGetAddressRange(&base, &asize, buffer) != hipSuccess) {
        (void)hipGetLastError();
        return dccl::ncclInvalidArgument;  // not a device allocation of this process
    }
    const uintptr_t b = reinterpret_cast<uintptr_t>(base), a = reinterpret_cast<uintptr_t>(buffer);
    if (a + size > b + asize) return dccl::ncclInvalidArgument;  // past its allocation
    ProcCache& pc = cache();
    std::lock_guard<std::mutex> lock(pc.mu);
    Range& r = pc.ranges[a];
    r.len = std::max(r.len, size);
    ++r.refs;
    return dccl::ncclSuccess;
}

// dcclDeregisterCacheMemory: as often as the start was registered; an unknown start is an error.
ncclResult_t ipc_deregister(void* buffer) {
    ProcCache& pc = cache();
    std::lock_guard<std::mutex> lock(pc.mu);
    auto r = pc.ranges.find(reinterpret_cast<uintptr_t>(buffer));
    if (r == pc.ranges.end()) return dccl::ncclInvalidArgument;
    if (--r->second.refs == 0) pc.ranges.erase(r);
    return dccl::ncclSuccess;
}

int ipc_stats(uint64_t* out, int n) {
    ProcCache& pc = cache();
    std::lock_guard<std::mutex> lock(pc.mu);
    const ipc::ImportStats& s = pc.imports.stats;
    // slots 2, 6 and 19 (registered-buffer hits, stale registrations, registered fallbacks) counted the
    // registered in-place path removed in round 5; they stay in the ABI, always 0
    const uint64_t v[] = {pc.exports_made, pc.retirements, 0, pc.scratch_copies, pc.scratch_bytes,
                          pc.scratch_grows, 0, s.opened, s.reused, s.retired, s.retired_pid,
                          s.trimmed, s.alias_evicted, s.alias_errors, s.open_retries, s.size_mismatch,
                          uint64_t(pc.imports.size()), uint64_t(pc.imports.bytes()), pc.recycled_handles,
                          0, s.verify_failures};
    const int m = std::min<int>(n, int(sizeof(v) / sizeof(v[0])));
    for (int i = 0; i < m; ++i) out[i] = v[i];
    return int(sizeof(v) / sizeof(v[0]));
}

// In-process groups take the direct collectives for device buffers unless DCCL_ALLREDUCE_ALGORITHM names
// another algorithm: "direct", "auto" and unset select them.  They are faster than the ring at every
// size measured and give the ring's results bit for bit.  Host buffers, the RCCL
// transport and groups above 8 ranks keep the ring.
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
// chunk from the rank that reduced it.  On the IPC transport `send` is read from the scratch copy, and
// `recv` is replaced by the scratch for the reduced chunk (reduced in
// place there: no other rank reads that chunk of anyone's input), which this rank then copies out.
ncclResult_t direct_all_reduce(dcclComm* c, const void* send, void* recv, size_t count, int dtype, int op,
                               hipStream_t st) {
    const uint32_t W = c->world, r = c->rank;
    if (W > kDirectMaxWorld) return dccl::ncclInvalidUsage;
    const size_t esz = size_of_dtype(dtype), slot_elems = count / W, slot = slot_elems * esz, total = count * esz;
    Publish pub;
    pub.in = send;
    pub.in_bytes = total;
    pub.out = recv;
    pub.out_bytes = total;
    Peers P;
    bool met = false;
    ncclResult_t rc = exchange(c, &pub, st, &P, &met);
    if (!met) return rc;
    const uint32_t mine = (r + 1) % W;
    if (rc == dccl::ncclSuccess)
        rc = chain(P, W, mine, mine * slot, P.in[r] + mine * slot, P.out[r] + mine * slot, slot_elems, dtype, op, st, r);
    if ((rc = arrive(c, st, rc)) != dccl::ncclSuccess) return rc;  // every chunk reduced by its owner
    std::vector<const void*> src;
    std::vector<void*> dst;
    for (uint32_t k = 0; k < W; ++k) {
        if (k == mine && !pub.out_scratch) continue;  // reduced in place
        src.push_back(P.out[(k + W - 1) % W] + k * slot);  // chunk k lives on rank k-1
        dst.push_back(static_cast<unsigned char*>(recv) + k * slot);
    }
    return arrive(c, st, copy_pairs(src, dst, slot, st), &P);  // peers are done reading our buffers
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
    Publish pub;
    pub.in = send;
    pub.in_bytes = slot * W;
    Peers P;
    bool met = false;
    ncclResult_t rc = exchange(c, &pub, st, &P, &met);
    if (!met) return rc;
    if (rc == dccl::ncclSuccess) rc = chain(P, W, (r + 1) % W, r * slot, P.in[r] + r * slot, recv, recvcount, dtype, op, st, r);
    return arrive(c, st, rc, &P);
}

// ncclReduce: the reference runs the reduce-scatter ring with the same maps, then gathers the slots
// at the root (dccl.cpp:745-846); here the root reduces every slot itself.
ncclResult_t direct_reduce(dcclComm* c, const void* send, void* recv, size_t count, int dtype, int op, uint32_t root,
                           hipStream_t st) {
    const uint32_t W = c->world, r = c->rank;
    if (W > kDirectMaxWorld) return dccl::ncclInvalidUsage;
    const size_t slot_elems = count / W, slot = slot_elems * size_of_dtype(dtype);
    Publish pub;
    pub.in = send;
    pub.in_bytes = slot * W;
    Peers P;
    bool met = false;
    ncclResult_t rc = exchange(c, &pub, st, &P, &met);
    if (!met) return rc;
    if (r == root)
        for (uint32_t o = 0; o < W && rc == dccl::ncclSuccess; ++o)
            rc = chain(P, W, (o + 1) % W, o * slot, P.in[o] + o * slot, static_cast<unsigned char*>(recv) + o * slot,
                       slot_elems, dtype, op, st, r);
    return arrive(c, st, rc, &P);
}

ncclResult_t direct_all_gather(dcclComm* c, const void* send, void* recv, size_t sendcount, int dtype,
                               hipStream_t st) {
    const uint32_t W = c->world, r = c->rank;
    if (W > kDirectMaxWorld) return dccl::ncclInvalidUsage;
    const size_t slot = sendcount * size_of_dtype(dtype);
    unsigned char* const out = static_cast<unsigned char*>(recv);
    Publish pub;
    pub.in = send;
    pub.in_bytes = slot;
    Peers P;
    bool met = false;
    ncclResult_t rc = exchange(c, &pub, st, &P, &met);
    if (!met) return rc;
    if (rc == dccl::ncclSuccess) {
        std::vector<const void*> src;
        std::vector<void*> dst;
        for (uint32_t p = 0; p < W; ++p) {
            const void* from = p == r ? send : static_cast<const void*>(P.in[p]);  // own slice: the user's copy
            if (p == r && from == out + r * slot) continue;  // already in place
            src.push_back(from);
            dst.push_back(out + p * slot);
        }
        rc = copy_pairs(src, dst, slot, st);
    }
    return arrive(c, st, rc, &P);
}

ncclResult_t direct_broadcast(dcclComm* c, const void* send, void* recv, size_t count, int dtype, uint32_t root,
                              hipStream_t st) {
    const uint32_t r = c->rank;
    const size_t bytes = count * size_of_dtype(dtype);
    Publish pub;
    if (r == root) {
        pub.in = send;
        pub.in_bytes = bytes;
    }
    Peers P;
    bool met = false;
    ncclResult_t rc = exchange(c, &pub, st, &P, &met);
    if (!met) return rc;
    const void* from = r == root ? send : static_cast<const void*>(P.in[root]);
    if (rc == dccl::ncclSuccess && from != recv) {
        std::vector<const void*> src{from};
        std::vector<void*> dst{recv};
        rc = copy_pairs(src, dst, bytes, st);
    }
    return arrive(c, st, rc, &P);
}

}  // namespace dccl_amd
