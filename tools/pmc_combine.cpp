// tools/pmc_combine.cpp — the bench's combine as a bare process, for rocprofv3 --pmc passes that bench.py
// runs while it measures (roofline.traffic): no Python, no torch, so a counter pass takes seconds.
//
//   pmc_combine <bytes_per_operand> <launches> [dtype] [op]
//
// Operands are laid out like bench.py's pooled layout: one hipMalloc, recv first, send 4 KiB past its end,
// filled with the counter-based generator (include/dccl/dccl_synth.h).  The combine (dccl_local_reduce)
// then runs <launches> times back to back on one stream.  Exit status 0 only if every call succeeded.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "dccl/dccl_reduce.h"
#include "dccl/dccl_synth.h"

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s bytes_per_operand launches [dtype] [op]\n", argv[0]);
        return 2;
    }
    const size_t nbytes = std::strtoull(argv[1], nullptr, 10);
    const int launches = std::atoi(argv[2]);
    const int dtype = argc > 3 ? std::atoi(argv[3]) : 7;
    const int op = argc > 4 ? std::atoi(argv[4]) : 0;
    const size_t esz = dccl_size_of_type(dtype);
    if (esz == 0 || nbytes % esz || launches <= 0) return 2;
    const size_t n = nbytes / esz, gap = 4096;
    unsigned char* pool = nullptr;
    if (hipMalloc(&pool, 2 * nbytes + gap) != hipSuccess) return 3;
    unsigned char* recv = pool;
    unsigned char* send = pool + nbytes + gap;
    hipStream_t st = nullptr;
    if (hipStreamCreate(&st) != hipSuccess) return 3;
    int rc = dccl_synth_fill(send, dtype, n, op, 0xDCC1, 0, st);
    if (rc == 0) rc = dccl_synth_fill(recv, dtype, n, op, 0xDCC1, 1, st);
    for (int i = 0; i < launches && rc == 0; ++i) rc = dccl_local_reduce(send, recv, dtype, n, op, st);
    if (hipStreamSynchronize(st) != hipSuccess) rc = rc ? rc : 1;
    (void)hipStreamDestroy(st);
    (void)hipFree(pool);
    if (rc != 0) std::fprintf(stderr, "pmc_combine: %s\n", dccl_result_string(rc));
    return rc == 0 ? 0 : 1;
}
