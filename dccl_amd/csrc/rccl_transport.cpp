// dccl_amd/csrc/rccl_transport.cpp — see rccl_transport.hpp.
#include "rccl_transport.hpp"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

namespace dccl_amd {
namespace {

struct RcclApi {
    decltype(&::ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&::ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&::ncclCommDestroy) comm_destroy = nullptr;
    decltype(&::ncclSend) send = nullptr;
    decltype(&::ncclRecv) recv = nullptr;
    decltype(&::ncclGroupStart) group_start = nullptr;
    decltype(&::ncclGroupEnd) group_end = nullptr;
    bool ok = false;
};

const RcclApi& api() {
    static RcclApi a;
    static std::once_flag once;
    std::call_once(once, [] {
        // prefer a copy already in the process (torch ships one), then the system ROCm one
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return;
        auto bind = [h](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            return fn != nullptr;
        };
        a.ok = bind(a.get_unique_id, "ncclGetUniqueId") && bind(a.comm_init_rank, "ncclCommInitRank") &&
               bind(a.comm_destroy, "ncclCommDestroy") && bind(a.send, "ncclSend") && bind(a.recv, "ncclRecv") &&
               bind(a.group_start, "ncclGroupStart") && bind(a.group_end, "ncclGroupEnd");
    });
    return a;
}

constexpr int kInternal = 3;  // ncclInternalError
constexpr int kSystem = 2;    // ncclSystemError

inline int rc(ncclResult_t r) { return static_cast<int>(r); }  // same numbering as dccl::ncclResult_t

}  // namespace

int rccl_available() { return api().ok ? 1 : 0; }

int rccl_get_unique_id(void* out128) {
    if (!api().ok) return kSystem;
    ncclUniqueId id;
    const int r = rc(api().get_unique_id(&id));
    if (r == 0) std::memcpy(out128, id.internal, kRcclUniqueIdBytes);
    return r;
}

int rccl_comm_init(void** rcomm, uint32_t world, uint32_t rank, const void* id128) {
    if (!api().ok) return kSystem;
    ncclUniqueId id;
    std::memcpy(id.internal, id128, kRcclUniqueIdBytes);
    ncclComm_t c = nullptr;
    const int r = rc(api().comm_init_rank(&c, static_cast<int>(world), id, static_cast<int>(rank)));
    *rcomm = c;
    return r;
}

int rccl_comm_destroy(void* rcomm) {
    if (!api().ok || rcomm == nullptr) return kInternal;
    return rc(api().comm_destroy(static_cast<ncclComm_t>(rcomm)));
}

int rccl_exchange(void* rcomm, const void* sendbuf, size_t send_bytes, uint32_t to, void* recvbuf,
                  size_t recv_bytes, uint32_t from, hipStream_t stream) {
    const RcclApi& a = api();
    if (!a.ok) return kSystem;
    auto c = static_cast<ncclComm_t>(rcomm);
    int r = rc(a.group_start());
    if (r != 0) return r;
    if (sendbuf != nullptr && send_bytes) r = rc(a.send(sendbuf, send_bytes, ncclUint8, int(to), c, stream));
    if (r == 0 && recvbuf != nullptr && recv_bytes) r = rc(a.recv(recvbuf, recv_bytes, ncclUint8, int(from), c, stream));
    const int re = rc(a.group_end());  // always close the group
    return r != 0 ? r : re;
}

int rccl_fan(void* rcomm, bool send, void* const* bufs, size_t bytes, uint32_t world, uint32_t self,
             hipStream_t stream) {
    const RcclApi& a = api();
    if (!a.ok) return kSystem;
    auto c = static_cast<ncclComm_t>(rcomm);
    int r = rc(a.group_start());
    if (r != 0) return r;
    for (uint32_t p = 0; p < world && r == 0 && bytes; ++p) {
        if (p == self) continue;
        r = send ? rc(a.send(bufs[p], bytes, ncclUint8, int(p), c, stream))
                 : rc(a.recv(bufs[p], bytes, ncclUint8, int(p), c, stream));
    }
    const int re = rc(a.group_end());  // always close the group
    return r != 0 ? r : re;
}

int rccl_exchange_all(void* rcomm, const void* const* sendbufs, void* const* recvbufs, size_t bytes, uint32_t world,
                      uint32_t self, hipStream_t stream) {
    const RcclApi& a = api();
    if (!a.ok) return kSystem;
    auto c = static_cast<ncclComm_t>(rcomm);
    int r = rc(a.group_start());
    if (r != 0) return r;
    for (uint32_t p = 0; p < world && r == 0 && bytes; ++p) {
        if (p == self) continue;
        if (sendbufs[p] != nullptr) r = rc(a.send(sendbufs[p], bytes, ncclUint8, int(p), c, stream));
        if (r == 0 && recvbufs[p] != nullptr) r = rc(a.recv(recvbufs[p], bytes, ncclUint8, int(p), c, stream));
    }
    const int re = rc(a.group_end());  // always close the group
    return r != 0 ? r : re;
}

}  // namespace dccl_amd
