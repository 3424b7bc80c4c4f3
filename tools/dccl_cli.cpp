// tools/dccl_cli.cpp — the MI355X build's counterpart of the reference's dccl_cli
// (/root/reference/src/application/cli.cpp:190-557): a functional + timing driver of the
// namespace-dccl API.  Ranks are threads of this process (one communicator each, joined with
// dcclCommInitRank); -n sets the world size (the reference takes it from layout.json).  With -p the
// process is ONE rank, as the reference's dccl_cli is (one process per rank, README.md:74-101): rank and
// world come from DCCL_RANK / DCCL_WORLD_SIZE (or RANK / WORLD_SIZE) and the communicator from the
// reference's own ncclCommInit(&comm) (cli.cpp:360), over the transport DCCL_TRANSPORT names (rccl or ipc;
// device buffers, -g).
//
// Buffers and inputs follow the reference CLI: host buffers are 64-B aligned with
// sendbuf = memset(rank), recvbuf = memset(rank + 128) (cli.cpp:371-381); device buffers are
// memset(rank) (cli.cpp:386-396).  Every API runs in place on sendbuf exactly as
// RUN_WITH_COUNTER does (cli.cpp:421-453).  Op names are parsed correctly (the reference's
// parse_reduce_operation drops `== 0` after the first strcmp, cli.cpp:167-182, so `prod`
// becomes Max and `max`/`min`/`avg` become Prod: documented deviation).
//
// Output: one JSON line per rank: first element's bits, whether the buffer is uniform, an
// FNV-1a hash of the whole buffer and the mean latency per call.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <getopt.h>
#include <string>
#include <thread>
#include <vector>

#include "dccl/dccl.hpp"
#include "dccl/dccl_reduce.h"

using namespace dccl;

namespace {

struct Opts {
    std::string api;
    int gpu = -1;          // -1: host buffers
    bool multi_gpu = false;
    long warmup = 0, repeat = 1000, count = 1024;
    int world = 1;
    bool process = false;  // -p: this process is one rank (ncclCommInit)
    int rank = 0;          // -p: from the environment
    ncclDataType_t dtype = ncclUint32;
    ncclRedOp_t op = ncclSum;
};

bool parse_dtype(const char* s, ncclDataType_t* d) {
    const char* names[] = {"int8", "uint8", "int32", "uint32", "int64", "uint64", "float16", "float32",
                           "float64", "bfloat16"};
    for (int i = 0; i < 10; ++i)
        if (std::strcmp(s, names[i]) == 0) { *d = static_cast<ncclDataType_t>(i); return true; }
    return false;
}

bool parse_op(const char* s, ncclRedOp_t* o) {
    const char* names[] = {"sum", "prod", "max", "min", "avg"};
    for (int i = 0; i < 5; ++i)
        if (std::strcmp(s, names[i]) == 0) { *o = static_cast<ncclRedOp_t>(i); return true; }
    return false;
}

uint64_t fnv1a(const unsigned char* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

struct Result {
    int rc = 0;
    double us_per_call = 0;
    std::vector<unsigned char> bytes;
};

void run_rank(const Opts& o, int rank, Result* out) {
    const size_t esz = dccl_size_of_type(o.dtype);
    const size_t nbytes = size_t(o.count) * esz;
    if (o.gpu >= 0) {
        int ndev = 1;
        (void)hipGetDeviceCount(&ndev);
        if (hipSetDevice(o.multi_gpu ? (o.gpu + rank) % ndev : o.gpu) != hipSuccess) { out->rc = 1; return; }
    }
    ncclComm_t comm = nullptr;
    if ((out->rc = o.process ? ncclCommInit(&comm) : dcclCommInitRank(&comm, o.world, rank)) != ncclSuccess) return;
    void *send = nullptr, *recv = nullptr;
    hipStream_t stream = nullptr;
    if (o.gpu < 0) {
        if (posix_memalign(&send, 64, nbytes + 64) || posix_memalign(&recv, 64, nbytes + 64)) { out->rc = 2; return; }
        std::memset(send, rank, nbytes);
        std::memset(recv, rank + 128, nbytes);
        (void)dcclRegisterCacheMemory(comm, send, (nbytes + 63) / 64 * 64);
    } else {
        if (hipMalloc(&send, nbytes + 128) != hipSuccess || hipMalloc(&recv, nbytes + 128) != hipSuccess ||
            hipStreamCreate(&stream) != hipSuccess || hipMemset(send, rank, nbytes) != hipSuccess ||
            hipMemset(recv, rank, nbytes) != hipSuccess) { out->rc = 1; return; }
    }
    auto* sb = static_cast<unsigned char*>(send);
    const size_t slot_off = size_t(rank) * nbytes / o.world;
    auto once = [&]() -> ncclResult_t {
        if (o.api == "all_reduce") return ncclAllReduce(send, send, o.count, o.dtype, o.op, comm, stream);
        if (o.api == "reduce_scatter")
            return ncclReduceScatter(send, sb + slot_off, o.count / o.world, o.dtype, o.op, comm, stream);
        if (o.api == "all_gather") return ncclAllGather(sb + slot_off, send, o.count / o.world, o.dtype, comm, stream);
        if (o.api == "reduce") return ncclReduce(send, send, o.count, o.dtype, o.op, 0, comm, stream);
        if (o.api == "broadcast") return ncclBroadcast(send, recv, o.count, o.dtype, 0, comm, stream);
        if (o.api == "send") return rank < 2 ? ncclSend(send, o.count, o.dtype, 1 - rank, comm, stream) : ncclSuccess;
        if (o.api == "recv") return rank < 2 ? ncclRecv(send, o.count, o.dtype, 1 - rank, comm, stream) : ncclSuccess;
        return ncclInvalidArgument;
    };
    for (long i = 0; i < o.warmup && out->rc == 0; ++i) out->rc = once();
    if (stream) (void)hipStreamSynchronize(stream);
    const auto t0 = std::chrono::steady_clock::now();
    for (long i = 0; i < o.repeat && out->rc == 0; ++i) out->rc = once();
    if (stream) (void)hipStreamSynchronize(stream);
    const auto t1 = std::chrono::steady_clock::now();
    out->us_per_call = o.repeat ? std::chrono::duration<double, std::micro>(t1 - t0).count() / o.repeat : 0;
    out->bytes.resize(nbytes);
    const void* result = (o.api == "broadcast") ? recv : send;
    if (o.gpu < 0) std::memcpy(out->bytes.data(), result, nbytes);
    else if (hipMemcpy(out->bytes.data(), result, nbytes, hipMemcpyDeviceToHost) != hipSuccess) out->rc = 1;
    if (o.gpu < 0) {
        (void)dcclDeregisterCacheMemory(comm, send);
        std::free(send);
        std::free(recv);
    } else {
        (void)hipFree(send);
        (void)hipFree(recv);
        (void)hipStreamDestroy(stream);
    }
    const ncclResult_t frc = ncclCommFinalize(comm);
    if (out->rc == 0) out->rc = frc;
}

}  // namespace

int main(int argc, char** argv) {
    Opts o;
    static struct option lo[] = {{"api", required_argument, 0, 'a'},    {"gpu", required_argument, 0, 'g'},
                                 {"warmup", required_argument, 0, 'w'}, {"repeat", required_argument, 0, 'r'},
                                 {"type", required_argument, 0, 't'},   {"op", required_argument, 0, 'o'},
                                 {"count", required_argument, 0, 'c'},  {"world", required_argument, 0, 'n'},
                                 {"multi-gpu", no_argument, 0, 'm'},    {"help", no_argument, 0, 'h'},
                                 {"process", no_argument, 0, 'p'},
                                 {0, 0, 0, 0}};
    int c;
    while ((c = getopt_long(argc, argv, "a:g:w:r:t:o:c:n:mph", lo, nullptr)) != -1) {
        switch (c) {
        case 'a': o.api = optarg; break;
        case 'g': o.gpu = std::atoi(optarg); break;
        case 'w': o.warmup = std::atol(optarg); break;
        case 'r': o.repeat = std::atol(optarg); break;
        case 'c': o.count = std::atol(optarg); break;
        case 'n': o.world = std::atoi(optarg); break;
        case 'm': o.multi_gpu = true; break;
        case 'p': o.process = true; break;
        case 't': if (!parse_dtype(optarg, &o.dtype)) { std::fprintf(stderr, "unknown type %s\n", optarg); return 1; } break;
        case 'o': if (!parse_op(optarg, &o.op)) { std::fprintf(stderr, "unknown op %s\n", optarg); return 1; } break;
        default:
            std::printf("usage: %s -a {all_reduce,reduce_scatter,all_gather,reduce,broadcast,send,recv} "
                        "[-t type] [-o op] [-c count] [-w warmup] [-r repeat] [-g gpu|-1] [-n world] [-m] [-p]\n", argv[0]);
            return c == 'h' ? 0 : 1;
        }
    }
    if (o.process) {
        auto env = [](const char* a, const char* b) {
            const char* v = std::getenv(a);
            if (v == nullptr) v = std::getenv(b);
            return v == nullptr ? -1 : std::atoi(v);
        };
        o.rank = env("DCCL_RANK", "RANK");
        o.world = env("DCCL_WORLD_SIZE", "WORLD_SIZE");
        if (o.rank < 0 || o.world < 1 || o.rank >= o.world) {
            std::fprintf(stderr, "-p: set DCCL_RANK / DCCL_WORLD_SIZE (or RANK / WORLD_SIZE)\n");
            return 1;
        }
    }
    if (o.api.empty() || o.world < 1 || o.count < 0) { std::fprintf(stderr, "missing/invalid -a/-n/-c\n"); return 1; }
    const int first_rank = o.process ? o.rank : 0, ranks = o.process ? 1 : o.world;
    std::vector<Result> res(ranks);
    std::vector<std::thread> th;
    for (int i = 0; i < ranks; ++i) th.emplace_back(run_rank, std::cref(o), first_rank + i, &res[i]);
    for (auto& t : th) t.join();
    int rc = 0;
    const size_t esz = dccl_size_of_type(o.dtype);
    for (int i = 0; i < ranks; ++i) {
        const int r = first_rank + i;
        const Result& x = res[i];
        uint64_t first = 0;
        bool uniform = true;
        if (!x.bytes.empty()) {
            std::memcpy(&first, x.bytes.data(), esz < 8 ? esz : 8);
            for (size_t i = esz; i < x.bytes.size() && uniform; i += esz)
                uniform = std::memcmp(x.bytes.data(), x.bytes.data() + i, esz) == 0;
        }
        std::printf("{\"rank\": %d, \"rc\": %d, \"first\": \"0x%0*llx\", \"uniform\": %s, \"fnv1a\": \"0x%016llx\", "
                    "\"us_per_call\": %.3f}\n",
                    r, x.rc, int(esz * 2), static_cast<unsigned long long>(first), uniform ? "true" : "false",
                    static_cast<unsigned long long>(fnv1a(x.bytes.data(), x.bytes.size())), x.us_per_call);
        if (x.rc) rc = 2;
    }
    return rc;
}
