// tests/native/ipc_cache_test.cpp — the IPC importer cache (dccl_amd/csrc/ipc_cache.hpp) against a fake
// runtime that behaves like the one that broke round 3's transport: opening handle bytes that this process
// already has open hands back that import (no reference count), and closing a base that is not open is an
// error ("Memobj map does not have ptr").  Built and run by tests/test_ipc_cache.py (g++, ASan + UBSan).
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

#include "ipc_cache.hpp"

using namespace dccl_amd::ipc;

namespace {

int failures = 0;
#define CHECK(cond)                                                              \
    do {                                                                         \
        if (!(cond)) {                                                           \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                          \
        }                                                                        \
    } while (0)

struct FakeRuntime final : Ops {
    size_t key_bytes = kHandleBytes;  // how much of the handle the runtime uses to find an existing import
    std::map<std::string, void*> imports;  // handle key -> mapped base
    std::map<void*, size_t> sizes;         // open bases -> allocation size
    std::map<std::string, size_t> alloc_size;  // what the exporter's allocation behind a handle key holds
    uintptr_t next = 0x100000;
    int opens = 0, closes = 0, bad_closes = 0, fail_next_opens = 0;

    std::string key(const Handle& h) const { return std::string(reinterpret_cast<const char*>(h.b), key_bytes); }
    bool open(const Handle& h, void** mapped) override {
        ++opens;
        if (fail_next_opens > 0) {
            --fail_next_opens;
            return false;
        }
        auto it = imports.find(key(h));
        if (it != imports.end()) {  // the existing import, not counted
            *mapped = it->second;
            return true;
        }
        void* b = reinterpret_cast<void*>(next);
        next += 0x100000;
        imports[key(h)] = b;
        auto s = alloc_size.find(key(h));
        sizes[b] = s == alloc_size.end() ? 4096 : s->second;
        *mapped = b;
        return true;
    }
    void close(void* mapped) override {
        ++closes;
        if (!sizes.count(mapped)) {
            ++bad_closes;
            return;
        }
        sizes.erase(mapped);
        for (auto it = imports.begin(); it != imports.end(); ++it)
            if (it->second == mapped) {
                imports.erase(it);
                break;
            }
    }
    size_t size_of(void* mapped) override {
        auto it = sizes.find(mapped);
        return it == sizes.end() ? 0 : it->second;
    }
    void backoff(int) override {}
};

Handle handle(int v, int tail = 0) {
    Handle h{};
    h.b[0] = static_cast<unsigned char>(v);
    h.b[kHandleBytes - 1] = static_cast<unsigned char>(tail);
    return h;
}

void test_reuse_and_release() {
    FakeRuntime rt;
    ImportCache c(&rt, 16, 1 << 30);
    void *a = nullptr, *b = nullptr;
    bool opened = false;
    CHECK(c.acquire(100, 1, handle(1), 4096, &a, 15, &opened) == kOk && opened);
    CHECK(c.acquire(100, 1, handle(1), 4096, &b, 15, &opened) == kOk && !opened);
    CHECK(a == b && rt.opens == 1);
    CHECK(c.find(100, 1)->users == 2);
    c.release(100, 1);
    c.release(100, 1);
    CHECK(c.find(100, 1)->users == 0);
    CHECK(c.stats.opened == 1 && c.stats.reused == 1);
}

// Round 3's failure: a freed allocation's handle bytes come back for a new export (another serial, and
// another address in the exporter).  The old mapping must be closed BEFORE the open, else the runtime
// hands back the freed buffer's import and every peer reads stale pages.
void test_repeated_handle_bytes_evicts_first() {
    FakeRuntime rt;
    ImportCache c(&rt, 16, 1 << 30);
    void *a = nullptr, *b = nullptr;
    CHECK(c.acquire(100, 1, handle(7), 4096, &a) == kOk);
    c.release(100, 1);
    CHECK(c.acquire(100, 2, handle(7), 4096, &b) == kOk);
    CHECK(b != a);                      // a fresh import, not the freed buffer's
    CHECK(c.find(100, 1) == nullptr);   // the old entry is gone
    CHECK(c.stats.alias_evicted == 1);
    CHECK(rt.closes == 1 && rt.bad_closes == 0);
    c.release(100, 2);
    c.close_unused();
    CHECK(rt.bad_closes == 0 && rt.imports.empty());
    // another exporter's identical bytes are not an alias
    void *x = nullptr, *y = nullptr;
    CHECK(c.acquire(100, 3, handle(9), 4096, &x) == kOk);
    CHECK(c.acquire(200, 3, handle(9, 1), 4096, &y) == kOk);
    CHECK(c.stats.alias_evicted == 1);
}

void test_repeated_handle_bytes_in_use_fails() {
    FakeRuntime rt;
    ImportCache c(&rt, 16, 1 << 30);
    void *a = nullptr, *b = nullptr;
    CHECK(c.acquire(100, 1, handle(7), 4096, &a) == kOk);  // still in use by a collective
    CHECK(c.acquire(100, 2, handle(7), 4096, &b) == kAliasInUse);
    CHECK(rt.closes == 0);              // nothing closed under the user
    CHECK(c.find(100, 1)->users == 1 && c.find(100, 2) == nullptr);
    CHECK(c.stats.alias_errors == 1);
}

// A runtime that finds an existing import by fewer bytes than the whole handle: the bytes differ, yet the
// open returns a base another entry holds.  Refused, and nothing closed (no double close later).
void test_open_returns_cached_base() {
    FakeRuntime rt;
    rt.key_bytes = 8;
    ImportCache c(&rt, 16, 1 << 30);
    void *a = nullptr, *b = nullptr;
    CHECK(c.acquire(100, 1, handle(5, 1), 4096, &a) == kOk);
    c.release(100, 1);
    CHECK(c.acquire(100, 2, handle(5, 2), 4096, &b) == kAliasOpened);
    CHECK(c.find(100, 2) == nullptr && c.find(100, 1) != nullptr);
    CHECK(rt.closes == 0);
    CHECK(c.stats.alias_errors == 1);
    // after the exporter's retirement of serial 1 arrives, serial 2 maps cleanly
    c.retire(100, 1);
    CHECK(rt.closes == 1 && rt.bad_closes == 0);
    CHECK(c.acquire(100, 2, handle(5, 2), 4096, &b) == kOk);
    CHECK(b != a || rt.imports.size() == 1);
    c.release(100, 2);
    c.close_unused();
    CHECK(rt.bad_closes == 0 && rt.imports.empty());
}

void test_retire_while_in_use_closes_at_release() {
    FakeRuntime rt;
    ImportCache c(&rt, 16, 1 << 30);
    void* a = nullptr;
    CHECK(c.acquire(100, 1, handle(1), 4096, &a) == kOk);
    c.retire(100, 1);
    CHECK(rt.closes == 0 && c.find(100, 1)->retired);
    void* b = nullptr;
    CHECK(c.acquire(100, 1, handle(1), 4096, &b) == kAliasInUse);  // a retired serial never comes back
    c.release(100, 1);
    CHECK(rt.closes == 1 && c.find(100, 1) == nullptr && rt.bad_closes == 0);
}

void test_retire_pid() {
    FakeRuntime rt;
    ImportCache c(&rt, 16, 1 << 30);
    void* a = nullptr;
    for (int s = 1; s <= 3; ++s) CHECK(c.acquire(100, s, handle(s), 4096, &a) == kOk);
    CHECK(c.acquire(200, 1, handle(1, 9), 4096, &a) == kOk);
    c.release(100, 1);
    c.release(100, 2);
    c.retire_pid(100);
    CHECK(c.find(100, 1) == nullptr && c.find(100, 2) == nullptr);
    // in use: suspect, not retired (it may be a live export another collective is reading)
    CHECK(c.find(100, 3) != nullptr && !c.find(100, 3)->retired && c.find(100, 3)->suspect);
    CHECK(c.find(200, 1) != nullptr && !c.find(200, 1)->retired && !c.find(200, 1)->suspect);
    c.release(100, 3);  // a suspect mapping closes with its last use
    CHECK(c.find(100, 3) == nullptr && rt.bad_closes == 0);
    bool opened = false;  // a live export is reopened and handed out for verification
    CHECK(c.acquire(100, 3, handle(3), 4096, &a, 15, &opened) == kOk && opened && c.find(100, 3)->users == 1);
    c.release(100, 3);
    CHECK(c.find(100, 3) != nullptr && rt.bad_closes == 0);  // verified and trusted: kept
}

// a retirement-log overflow while a mapping is in use.  A concurrent acquire of the same live
// export gets it for re-verification instead of kAliasInUse; when verification passes it is trusted again; when
// it fails (the export had ended) the caller's release + retire close it with its last use.
void test_overflow_while_in_use() {
    FakeRuntime rt;
    ImportCache c(&rt, 16, 1 << 30);
    void *a = nullptr, *b = nullptr;
    bool opened = false;
    CHECK(c.acquire(100, 5, handle(5), 4096, &a, 15, &opened) == kOk && opened);  // collective 1 holds it
    c.retire_pid(100);
    CHECK(c.acquire(100, 5, handle(5), 4096, &b, 15, &opened) == kOk && opened);  // collective 2: verify it
    CHECK(a == b && rt.opens == 1 && c.stats.alias_errors == 0 && c.find(100, 5)->users == 2);
    CHECK(!c.find(100, 5)->suspect);
    CHECK(c.acquire(100, 5, handle(5), 4096, &b, 15, &opened) == kOk && !opened);  // verified: trusted again
    c.release(100, 5);
    c.release(100, 5);
    c.release(100, 5);
    CHECK(c.find(100, 5) != nullptr && c.find(100, 5)->users == 0);
    // the same with a failed verification: collective 2 releases and retires; closed at collective 1's release
    CHECK(c.acquire(100, 6, handle(6), 4096, &a, 15, &opened) == kOk && opened);
    c.retire_pid(100);  // closes the unused (100, 5), marks (100, 6) suspect
    CHECK(c.find(100, 5) == nullptr && c.find(100, 6)->suspect);
    CHECK(c.acquire(100, 6, handle(6), 4096, &b, 15, &opened) == kOk && opened);
    c.release(100, 6);
    c.retire(100, 6);
    CHECK(c.find(100, 6) != nullptr && c.find(100, 6)->retired);  // collective 1 still reads it
    c.release(100, 6);
    CHECK(c.find(100, 6) == nullptr && rt.bad_closes == 0 && c.stats.alias_errors == 0);
}

void test_trim() {
    FakeRuntime rt;
    ImportCache c(&rt, 4, 3 * 4096);
    void* a = nullptr;
    for (int s = 1; s <= 4; ++s) {
        CHECK(c.acquire(100, s, handle(s), 4096, &a) == kOk);
        if (s != 2) c.release(100, s);
    }
    c.trim(2);  // 4 + 2 > 4 and 4 pages > 3: close the oldest unused, never the one in use (2)
    CHECK(c.size() == 2 && c.find(100, 2) != nullptr && c.find(100, 1) == nullptr && c.find(100, 3) == nullptr);
    CHECK(c.stats.trimmed == 2 && rt.bad_closes == 0);
}

void test_size_mismatch_and_open_failure() {
    FakeRuntime rt;
    ImportCache c(&rt, 16, 1 << 30);
    void* a = nullptr;
    rt.alloc_size[std::string(reinterpret_cast<const char*>(handle(3).b), kHandleBytes)] = 8192;
    CHECK(c.acquire(100, 1, handle(3), 4096, &a, 3) == kOpenFailed);  // always the wrong allocation
    CHECK(c.stats.size_mismatch == 3 && rt.bad_closes == 0 && rt.imports.empty());
    rt.fail_next_opens = 2;
    CHECK(c.acquire(100, 2, handle(4), 4096, &a, 3) == kOk);  // two transient failures, then the open
    CHECK(c.stats.open_retries == 5);
    rt.fail_next_opens = 5;
    CHECK(c.acquire(100, 3, handle(6), 4096, &a, 3) == kOpenFailed);
}

// Many free / re-allocate rounds, the exporter retiring each round's export before publishing the next
// (what direct.cpp does for a deregistered or replaced buffer): every acquisition maps the live buffer.
void test_churn() {
    FakeRuntime rt;
    ImportCache c(&rt, 256, size_t(1) << 40);
    std::vector<void*> bases;
    uint64_t serial = 1;
    for (int round = 0; round < 500; ++round) {
        const Handle h = handle(round % 3);  // handle bytes repeat every 3 rounds
        void* b = nullptr;
        CHECK(c.acquire(100, serial, h, 4096, &b) == kOk);
        CHECK(rt.imports.size() == c.size());
        c.release(100, serial);
        if (round % 2) c.retire(100, serial);  // half the retirements arrive; the bytes catch the rest
        ++serial;
    }
    CHECK(rt.bad_closes == 0 && c.stats.alias_errors == 0);
    c.close_unused();
    CHECK(rt.imports.empty() && rt.bad_closes == 0);
}

}  // namespace

int main() {
    test_reuse_and_release();
    test_repeated_handle_bytes_evicts_first();
    test_repeated_handle_bytes_in_use_fails();
    test_open_returns_cached_base();
    test_retire_while_in_use_closes_at_release();
    test_retire_pid();
    test_overflow_while_in_use();
    test_trim();
    test_size_mismatch_and_open_failure();
    test_churn();
    if (failures) {
        std::fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    std::printf("ipc_cache: ok\n");
    return 0;
}
