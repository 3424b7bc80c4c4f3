// dccl_amd/csrc/ipc_cache.hpp — the importer side of the IPC transport: which peer allocations this
// process has mapped, and when a mapping may no longer be used.
//
// The reference never infers buffer identity from runtime state: RDMA-visible memory is registered and
// deregistered explicitly (dcclRegisterCacheMemory / dcclDeregisterCacheMemory,
// /root/reference/src/core/dccl.cpp:503-549) and the library's own scratchpads have a known lifetime
// (:57-84, 170-237).  The IPC transport follows that: every buffer a peer may read is an EXPORT with a
// serial that its process never reuses (a registered user allocation, or the communicator's scratch),
// and an export ends only by an explicit retirement that the exporter writes into the shared segment
// (direct.cpp).  Mappings here are keyed by (exporter pid, serial), so two exports can never share a key.
//
// What the runtime does underneath is still guarded, because the handle BYTES of a new allocation may
// repeat those of a freed one (dmabuf handles on ROCm 7.2), and opening handle bytes that
// this process already has open hands back that earlier import (the freed allocation's pages):
//   * before an open, any mapping of the same exporter with the same handle bytes names an export that
//     has ended (two live allocations never share a handle): it is closed first if unused, and the open
//     fails with kAliasInUse if a collective of this process still uses it;
//   * after an open, a mapped base already held under another key is an alias the bytes did not reveal:
//     kAliasOpened, and nothing is closed (whether the runtime counted that open is unknown).
// Every mapping is closed exactly once, by the entry that opened it.
//
// Header-only and free of HIP types: the runtime calls go through `Ops`, so tests/test_ipc_cache.py can
// drive this logic with a fake runtime on the CPU (tests/native/ipc_cache_test.cpp).  Not thread-safe:
// the caller holds its process-wide mutex.
#pragma once

#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <deque>
#include <iterator>
#include <map>
#include <thread>
#include <utility>

namespace dccl_amd {
namespace ipc {

constexpr size_t kHandleBytes = 64;  // HIP_IPC_HANDLE_SIZE

struct Handle {
    unsigned char b[kHandleBytes];
    bool operator==(const Handle& o) const { return std::memcmp(b, o.b, kHandleBytes) == 0; }
};

// The runtime calls the cache makes: hipIpcOpenMemHandle / hipIpcCloseMemHandle / hipMemGetAddressRange
// in the product (direct.cpp), a fake in the tests.
struct Ops {
    virtual ~Ops() = default;
    virtual bool open(const Handle& h, void** mapped) = 0;
    virtual void close(void* mapped) = 0;
    virtual size_t size_of(void* mapped) = 0;  // bytes of the mapped allocation, 0 if unknown
    virtual void backoff(int attempt) {         // between failed opens
        std::this_thread::sleep_for(std::chrono::microseconds(std::min(100 << attempt, 100000)));
    }
};

// Counters of one process (the importer side; direct.cpp adds the exporter side).
struct ImportStats {
    uint64_t opened = 0;         // mappings opened
    uint64_t reused = 0;         // acquisitions served by an open mapping
    uint64_t retired = 0;        // mappings closed because their export was retired
    uint64_t retired_pid = 0;    // retirement-log overflows (every unused mapping of that exporter closed)
    uint64_t trimmed = 0;        // mappings closed to bound the cache
    uint64_t alias_evicted = 0;  // unused mappings with the incoming handle's bytes, closed before the open
    uint64_t alias_errors = 0;   // opens refused: kAliasInUse or kAliasOpened
    uint64_t open_retries = 0;   // failed open attempts (retried)
    uint64_t size_mismatch = 0;  // opens whose allocation size differed from the published one (retried)
    uint64_t verify_failures = 0;  // new mappings whose content token did not match the exporter's (direct.cpp)
};

enum Result { kOk = 0, kOpenFailed = 1, kAliasInUse = 2, kAliasOpened = 3 };

class ImportCache {
public:
    struct Key {
        int64_t pid;
        uint64_t serial;
        bool operator<(const Key& o) const { return pid != o.pid ? pid < o.pid : serial < o.serial; }
        bool operator==(const Key& o) const { return pid == o.pid && serial == o.serial; }
    };
    struct Entry {
        void* base = nullptr;
        size_t bytes = 0;
        Handle handle{};
        uint32_t users = 0;    // collectives of this process that resolved it and have not returned
        bool retired = false;  // its export ended while in use: closed at the last release
        bool suspect = false;  // in use when its exporter's retirement log overflowed: maybe ended, maybe not
    };

    ImportCache(Ops* ops, size_t max_mappings, size_t max_bytes)
        : ops_(ops), max_mappings_(max_mappings), max_bytes_(max_bytes) {}

    // Map export (pid, serial) with handle `h` of an allocation of `size` bytes and take a use of it.
    // *opened (optional): true when the caller must verify the mapping before trusting it: this call opened
    // it, or it was suspect (see retire_pid).  A failed verification is followed by release + retire.
    Result acquire(int64_t pid, uint64_t serial, const Handle& h, uint64_t size, void** base, int max_attempts = 15,
                   bool* opened = nullptr) {
        const Key k{pid, serial};
        if (opened) *opened = false;
        auto it = map_.find(k);
        if (it != map_.end() && !it->second.retired) {
            ++it->second.users;
            ++stats.reused;
            *base = it->second.base;
            if (it->second.suspect && opened) *opened = true;  // re-verified by the caller, then trusted again
            it->second.suspect = false;
            return kOk;
        }
        if (it != map_.end()) {  // a retired export published again: the exporter broke its serials
            ++stats.alias_errors;
            return kAliasInUse;
        }
        // the same handle bytes under another serial of this exporter: that export has ended
        for (auto o = map_.begin(); o != map_.end();) {
            if (o->first.pid == pid && o->second.handle == h) {
                if (o->second.users != 0) {
                    ++stats.alias_errors;
                    return kAliasInUse;
                }
                ++stats.alias_evicted;
                o = close_entry(o);
            } else {
                ++o;
            }
        }
        void* mapped = nullptr;
        for (int attempt = 0;; ++attempt) {
            bool ok = ops_->open(h, &mapped);
            if (ok) {
                const size_t got = ops_->size_of(mapped);
                if (got != 0 && got != size) {  // an import of another allocation: not ours
                    ++stats.size_mismatch;
                    ops_->close(mapped);
                    ok = false;
                }
            }
            if (ok) break;
            ++stats.open_retries;
            if (attempt + 1 >= max_attempts) return kOpenFailed;
            ops_->backoff(attempt);
        }
        for (auto& kv : map_)
            if (kv.second.base == mapped) {  // the runtime handed back an import another key holds
                ++stats.alias_errors;
                return kAliasOpened;
            }
        Entry e;
        e.base = mapped;
        e.bytes = ops_->size_of(mapped);
        e.handle = h;
        e.users = 1;
        map_.emplace(k, e);
        order_.push_back(k);
        bytes_ += e.bytes;
        ++stats.opened;
        *base = mapped;
        if (opened) *opened = true;
        return kOk;
    }

    // Drop one use taken by acquire(); a retired mapping is closed with its last use, and so is a suspect one
    // (if its export really ended, nothing would acquire it again and it would pin the peer's freed
    // pages until trim; a live export is simply reopened and verified by its next acquire).
    void release(int64_t pid, uint64_t serial) {
        auto it = map_.find(Key{pid, serial});
        if (it == map_.end() || it->second.users == 0) return;
        if (--it->second.users == 0 && (it->second.retired || it->second.suspect)) close_entry(it);
    }

    // The exporter ended export (pid, serial): close its mapping now, or with its last use.
    void retire(int64_t pid, uint64_t serial) {
        auto it = map_.find(Key{pid, serial});
        if (it == map_.end() || it->second.retired) return;
        ++stats.retired;
        if (it->second.users == 0) close_entry(it);
        else it->second.retired = true;
    }

    // The exporter's retirement log overflowed: every mapping of it may be stale.  Unused ones are closed; one
    // in use (possibly a live export, such as the peer's current scratch that another communicator's collective
    // is reading) becomes SUSPECT rather than retired: its next acquire hands it out for re-verification
    // (retiring it made a concurrent acquire fail with kAliasInUse although nothing was stale).
    void retire_pid(int64_t pid) {
        ++stats.retired_pid;
        for (auto it = map_.begin(); it != map_.end();) {
            auto next = std::next(it);
            if (it->first.pid == pid && !it->second.retired) {
                if (it->second.users == 0) close_entry(it);
                else it->second.suspect = true;
            }
            it = next;
        }
    }

    // Close the oldest unused mappings until `incoming` more fit under the count bound and the mappings
    // kept hold at most max_bytes of peer memory (a mapping keeps the peer's pages alive).
    void trim(size_t incoming) {
        for (size_t i = 0; i < order_.size() && (map_.size() + incoming > max_mappings_ || bytes_ > max_bytes_);) {
            auto it = map_.find(order_[i]);
            if (it != map_.end() && it->second.users == 0) {
                ++stats.trimmed;
                close_entry(it);
            } else {
                ++i;
            }
        }
    }

    void close_unused() {
        for (auto it = map_.begin(); it != map_.end();) {
            auto next = std::next(it);
            if (it->second.users == 0) close_entry(it);
            it = next;
        }
    }

    size_t size() const { return map_.size(); }
    size_t bytes() const { return bytes_; }
    const Entry* find(int64_t pid, uint64_t serial) const {
        auto it = map_.find(Key{pid, serial});
        return it == map_.end() ? nullptr : &it->second;
    }

    ImportStats stats;

private:
    std::map<Key, Entry>::iterator close_entry(std::map<Key, Entry>::iterator it) {
        ops_->close(it->second.base);
        bytes_ -= it->second.bytes;
        for (auto o = order_.begin(); o != order_.end(); ++o)
            if (*o == it->first) {
                order_.erase(o);
                break;
            }
        return map_.erase(it);
    }

    Ops* ops_;
    size_t max_mappings_, max_bytes_;
    std::map<Key, Entry> map_;
    std::deque<Key> order_;  // oldest first
    size_t bytes_ = 0;
};

}  // namespace ipc
}  // namespace dccl_amd
