// oracle/ref_harness.cpp — TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).
//
// Wraps the reference's own `do_host_reduce<DT>` (read at build time from
// /root/reference/src/core/internal_common.hpp:496-586 by oracle/build_ref.sh into a
// scratch directory outside the repository) behind a C entry point so the tests can
// pin oracle/host_reduce.c against the real thing.  Compiled with the reference's
// Release flags (-O3 -mprefer-vector-width=512, /root/reference/CMakeLists.txt:25)
// against the reference's public header /root/reference/include/dccl/dccl.hpp.
#include <dccl/dccl.hpp>
#include <cstdint>
#include <typeinfo>

// The body logs through spdlog macros; the oracle build has no logger.
#define dccl_warn(...) ((void)0)
#define dccl_trace(...) ((void)0)

namespace dccl {
#include "host_reduce_body.inc"
}  // namespace dccl

// Mirrors ON_DCCL_DATATYPE of a non-CUDA build (internal_common.hpp:383-413): dtypes
// without a host specialisation (fp16, bf16, unknown) are skipped and the caller's
// `ret` is left unchanged.  -1 signals "skipped" so the tests can see it.
extern "C" int ref_host_reduce(const void* send, void* recv, size_t count, int dtype, int op) {
    using namespace dccl;
    const ncclRedOp_t o = static_cast<ncclRedOp_t>(op);
    switch (dtype) {
    case ncclInt8: return do_host_reduce<int8_t>(send, recv, count, o);
    case ncclUint8: return do_host_reduce<uint8_t>(send, recv, count, o);
    case ncclInt32: return do_host_reduce<int32_t>(send, recv, count, o);
    case ncclUint32: return do_host_reduce<uint32_t>(send, recv, count, o);
    case ncclInt64: return do_host_reduce<int64_t>(send, recv, count, o);
    case ncclUint64: return do_host_reduce<uint64_t>(send, recv, count, o);
    case ncclFloat32: return do_host_reduce<float>(send, recv, count, o);
    case ncclFloat64: return do_host_reduce<double>(send, recv, count, o);
    default: return -1;
    }
}
