// tests/native/ring_p2p_harness.cpp — TEST INFRASTRUCTURE: the ring algorithms' point-to-point branch
// (dccl_amd/csrc/algorithms.cpp, the path RCCL or a plugged-in transport takes) driven on the CPU.
//
// Linked with algorithms.cpp itself and nothing else of the product: the transport is a fake exchange that
// moves bytes between W thread-ranks through per-(source, destination) mailboxes and records every call;
// the combine the algorithms call after each receive is the oracle restatement (oracle/host_reduce.c), so
// the choreography (peer, slot, bytes of every step) and the final buffers can be checked against the
// reference's formulas (tests/ringsim.py, tests/rabsim.py) without a GPU.  On the GPU box the same branch
// runs with the real combine through dccl_comm_init_p2p (tests/test_p2p_transport.py).
//
//   ring_p2p_harness <algo> <world> <count> <dtype> <op> <outdir>
//     algo: rs (reduce_scatter_ring, identity maps) | rs_api (ncclReduceScatter's maps) |
//           ag (all_gather_ring) | ar (all_reduce_ring) | rab (all_reduce_rabenseifner) |
//           grs / grs_api / gar (reduce_scatter_grouped shift 1 / 0, all_reduce_grouped: grouped.cpp, with the
//           grouped RCCL exchange faked on the same mailboxes and the chain combine done by the oracle)
//   grs / grs_api leave the owned slot's result in place ((r + 1) % W, resp. r), as the ring does.
//   rank r's buffer starts as oracle_synth_fill(seed 0xDCC1, buffer_id r); <outdir>/rank<r>.bin gets the
//   final buffer; stdout gets one JSON line: {"rc": [...], "log": [[[to, from, send_off, recv_off,
//   send_bytes, recv_bytes], ...] per rank]} with offsets relative to the rank's buffer (-1: the
//   scratchpad, -2: no buffer).
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "algorithms.hpp"

extern "C" {
int oracle_expected_reduce(const void* send, void* recv, size_t count, int dtype, int op);
int oracle_synth_fill(void* dst, int dtype, size_t count, int op, uint64_t seed, uint64_t buffer_id, size_t first);
}

namespace dccl_amd {
// The product's transport verbs and scratch/combine, replaced for this harness (the p2p branch never calls
// the in-process verbs).
ncclResult_t xport_send(dccl::dcclComm*, uint32_t, const void*, size_t, bool, hipStream_t) {
    return dccl::ncclInternalError;
}
ncclResult_t xport_recv(dccl::dcclComm*, uint32_t, void*, size_t, bool, hipStream_t) { return dccl::ncclInternalError; }
ncclResult_t xport_wait_send(dccl::dcclComm*, uint32_t, bool, hipStream_t) { return dccl::ncclInternalError; }
ncclResult_t xport_recv_combine(dccl::dcclComm*, uint32_t, void*, size_t, int, int, bool, hipStream_t) {
    return dccl::ncclInternalError;
}
ncclResult_t ensure_scratch(dccl::dcclComm* c, size_t bytes, bool device) {
    void*& pad = device ? c->dev_scratch : c->host_scratch;  // "device" memory is host memory here
    size_t& have = device ? c->dev_scratch_bytes : c->host_scratch_bytes;
    if (have >= bytes) return dccl::ncclSuccess;
    std::free(pad);
    pad = std::aligned_alloc(64, (bytes + 63) / 64 * 64);
    have = bytes;
    return pad ? dccl::ncclSuccess : dccl::ncclSystemError;
}
ncclResult_t combine(const void* send, void* recv, int dtype, size_t count, int op, bool device, hipStream_t) {
    if (device) return dccl::ncclInternalError;
    return static_cast<ncclResult_t>(oracle_expected_reduce(send, recv, count, dtype, op));
}
int rccl_exchange_all(void* rcomm, const void* const* sendbufs, void* const* recvbufs, size_t bytes, uint32_t world,
                      uint32_t self, hipStream_t stream);  // below: the fake exchange's grouped form
}  // namespace dccl_amd

// dccl_local_reduce_chain on host memory: dst = op(own, op(s{k-1}, ... op(s1, s0))), every application
// op(recv = the next part, send = the partial so far), as reduce_scatter_ring.cpp:84-94 applies it.
extern "C" int dccl_local_reduce_chain(const void* const* sends, int nsend, const void* own, void* dst, int dtype,
                                       size_t count, int op, void*) {
    const size_t bytes = count * dccl_amd::size_of_dtype(dtype);
    std::vector<unsigned char> acc(static_cast<const unsigned char*>(sends[0]),
                                   static_cast<const unsigned char*>(sends[0]) + bytes);
    for (int k = 1; k <= nsend; ++k) {
        const auto* part = static_cast<const unsigned char*>(k < nsend ? sends[k] : own);
        std::vector<unsigned char> next(part, part + bytes);
        const int rc = oracle_expected_reduce(acc.data(), next.data(), count, dtype, op);
        if (rc != 0) return rc;
        acc.swap(next);
    }
    std::memcpy(dst, acc.data(), bytes);
    return 0;
}

namespace {

struct Net {
    std::mutex mu;
    std::condition_variable cv;
    std::map<std::pair<uint32_t, uint32_t>, std::deque<std::vector<unsigned char>>> q;
};

struct Endpoint {
    Net* net;
    dccl::dcclComm* comm;
    uint32_t rank;
    const unsigned char* base;
    size_t bytes;
    std::vector<std::vector<long long>> log;
};

long long offset_of(const Endpoint* e, const void* p) {
    if (p == nullptr) return -2;
    const auto* b = static_cast<const unsigned char*>(p);
    if (b >= e->base && b < e->base + e->bytes) return b - e->base;
    return p == e->comm->host_scratch ? -1 : -3;
}

int fake_exchange(void* ctx, const void* sendbuf, size_t send_bytes, uint32_t to, void* recvbuf, size_t recv_bytes,
                  uint32_t from, void*) {
    auto* e = static_cast<Endpoint*>(ctx);
    e->log.push_back({sendbuf ? (long long)to : -1, recvbuf ? (long long)from : -1, offset_of(e, sendbuf),
                      offset_of(e, recvbuf), (long long)send_bytes, (long long)recv_bytes});
    Net& n = *e->net;
    if (sendbuf != nullptr) {
        std::vector<unsigned char> m(static_cast<const unsigned char*>(sendbuf),
                                     static_cast<const unsigned char*>(sendbuf) + send_bytes);
        std::lock_guard<std::mutex> lk(n.mu);
        n.q[{e->rank, to}].push_back(std::move(m));
        n.cv.notify_all();
    }
    if (recvbuf != nullptr) {
        std::unique_lock<std::mutex> lk(n.mu);
        auto& box = n.q[{from, e->rank}];
        if (!n.cv.wait_for(lk, std::chrono::seconds(30), [&] { return !box.empty(); })) return dccl::ncclSystemError;
        std::vector<unsigned char> m = std::move(box.front());
        box.pop_front();
        if (m.size() != recv_bytes) return dccl::ncclInvalidUsage;
        std::memcpy(recvbuf, m.data(), recv_bytes);
    }
    return dccl::ncclSuccess;
}

}  // namespace

// The grouped exchange on the same mailboxes: every send first, then every receive (one log entry per peer).
int dccl_amd::rccl_exchange_all(void* rcomm, const void* const* sendbufs, void* const* recvbufs, size_t bytes,
                                uint32_t world, uint32_t self, hipStream_t) {
    auto* e = static_cast<Endpoint*>(rcomm);
    for (uint32_t p = 0; p < world; ++p)
        if (p != self) {
            const int rc = fake_exchange(e, sendbufs[p], sendbufs[p] ? bytes : 0, p, nullptr, 0, 0, nullptr);
            if (rc != 0) return rc;
        }
    for (uint32_t p = 0; p < world; ++p)
        if (p != self) {
            const int rc = fake_exchange(e, nullptr, 0, 0, recvbufs[p], recvbufs[p] ? bytes : 0, p, nullptr);
            if (rc != 0) return rc;
        }
    return 0;
}

int main(int argc, char** argv) {
    if (argc != 7) {
        std::fprintf(stderr, "usage: %s algo world count dtype op outdir\n", argv[0]);
        return 2;
    }
    const std::string algo = argv[1];
    const uint32_t W = static_cast<uint32_t>(std::atoi(argv[2]));
    const size_t count = std::strtoull(argv[3], nullptr, 10);
    const int dtype = std::atoi(argv[4]), op = std::atoi(argv[5]);
    const std::string outdir = argv[6];
    const size_t esz = dccl_amd::size_of_dtype(dtype);
    if (W == 0 || esz == 0) return 2;
    Net net;
    std::vector<std::vector<unsigned char>> bufs(W, std::vector<unsigned char>(count * esz + 64));
    std::vector<dccl::dcclComm> comms(W);
    std::vector<Endpoint> eps(W);
    std::vector<int> rcs(W, -1);
    for (uint32_t r = 0; r < W; ++r) {
        oracle_synth_fill(bufs[r].data(), dtype, count, op, 0xDCC1, r, 0);
        comms[r].rank = r;
        comms[r].world = W;
        comms[r].p2p = &fake_exchange;
        comms[r].p2p_ctx = &eps[r];
        comms[r].p2p_host = true;
        comms[r].rccl = &eps[r];  // read by grouped.cpp only, as the fake rccl_exchange_all's context
        eps[r] = Endpoint{&net, &comms[r], r, bufs[r].data(), count * esz, {}};
    }
    const dccl_amd::RankMap id = [](uint32_t x) { return x; };
    std::vector<std::thread> ts;
    for (uint32_t r = 0; r < W; ++r) {
        ts.emplace_back([&, r] {
            dccl::dcclComm* c = &comms[r];
            void* b = bufs[r].data();
            dccl::ncclResult_t rc = dccl::ncclInvalidArgument;
            if (algo == "rs") {
                rc = dccl_amd::reduce_scatter_ring(c, b, nullptr, count, dtype, op, false, nullptr, id, id);
            } else if (algo == "rs_api") {
                rc = dccl_amd::reduce_scatter_ring(c, b, nullptr, count, dtype, op, false, nullptr,
                                                   [W](uint32_t o) { return (o + W - 1) % W; },
                                                   [W](uint32_t n) { return (n + 1) % W; });
            } else if (algo == "ag") {
                rc = dccl_amd::all_gather_ring(c, b, count / W, dtype, false, nullptr, id, id);
            } else if (algo == "ar") {
                rc = dccl_amd::all_reduce_ring(c, b, nullptr, count, dtype, op, false, nullptr);
            } else if (algo == "rab") {
                rc = dccl_amd::all_reduce_rabenseifner(c, b, nullptr, count, dtype, op, false, nullptr);
            } else if (algo == "grs" || algo == "grs_api") {  // the owned slot's result in place, like the ring
                const uint32_t shift = algo == "grs" ? 1 : 0;
                unsigned char* mine = static_cast<unsigned char*>(b) + ((r + shift) % W) * (count / W) * esz;
                rc = dccl_amd::reduce_scatter_grouped(c, b, mine, count, dtype, op, nullptr, shift);
            } else if (algo == "gar") {
                rc = dccl_amd::all_reduce_grouped(c, b, b, count, dtype, op, nullptr);
            }
            rcs[r] = static_cast<int>(rc);
        });
    }
    for (auto& t : ts) t.join();
    for (uint32_t r = 0; r < W; ++r) {
        const std::string path = outdir + "/rank" + std::to_string(r) + ".bin";
        FILE* f = std::fopen(path.c_str(), "wb");
        if (f == nullptr) return 3;
        std::fwrite(bufs[r].data(), 1, count * esz, f);
        std::fclose(f);
        std::free(comms[r].host_scratch);
        comms[r].host_scratch = nullptr;
        std::free(comms[r].dev_scratch);
        comms[r].dev_scratch = nullptr;
    }
    std::printf("{\"rc\": [");
    for (uint32_t r = 0; r < W; ++r) std::printf("%s%d", r ? ", " : "", rcs[r]);
    std::printf("], \"log\": [");
    for (uint32_t r = 0; r < W; ++r) {
        std::printf("%s[", r ? ", " : "");
        for (size_t i = 0; i < eps[r].log.size(); ++i) {
            const auto& v = eps[r].log[i];
            std::printf("%s[%lld, %lld, %lld, %lld, %lld, %lld]", i ? ", " : "", v[0], v[1], v[2], v[3], v[4], v[5]);
        }
        std::printf("]");
    }
    std::printf("]}\n");
    return 0;
}
