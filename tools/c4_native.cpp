// tools/c4_native.cpp — BASELINE C4's small and mid sizes as a C++ caller issues them: back-to-back eager
// dccl_local_reduce calls from a native loop (DCCL's ring step loop is C++), timed with HIP events on the
// launch stream.  bench.py runs it beside its Python-issued (ctypes) and HIP-graph-replayed C4 columns.
//
//   c4_native [max_log2_bytes = 26]
//
// fp32 Sum, 2^12 ... 2^max bytes per operand, powers of 2.  Operands rotate over `sets` pairs spread across a
// 4 GiB-per-operand pool (recv in the first half, send 4 KiB past it, bench.py's pooled layout) whenever one
// pair's working set is below 512 MiB, so the 256 MiB Infinity Cache does not keep them (the bench's rule).
// One JSON line per size on stdout.  Exit status 0 only if every call succeeded.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "dccl/dccl_reduce.h"

int main(int argc, char** argv) {
    const int max_log2 = argc > 1 ? std::atoi(argv[1]) : 26;
    if (max_log2 < 12 || max_log2 > 32) return 2;
    const size_t top = size_t(4) << 30, gap = 4096;
    unsigned char* pool = nullptr;
    if (hipMalloc(&pool, 2 * top + gap) != hipSuccess) return 3;
    if (hipMemset(pool, 0, 2 * top + gap) != hipSuccess) return 3;
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (hipStreamCreate(&st) != hipSuccess || hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
        return 3;
    int rc = 0;
    for (int lg = 12; lg <= max_log2 && rc == 0; ++lg) {
        const size_t nb = size_t(1) << lg, n = nb / 4;
        size_t sets = 1;
        if (2 * nb < (size_t(512) << 20)) {
            sets = ((size_t(512) << 20) + 2 * nb - 1) / (2 * nb);
            if (sets < 2) sets = 2;
            if (sets > top / nb) sets = top / nb;
        }
        const size_t stride = sets > 1 ? top / sets / 4096 * 4096 : 0;
        auto launch = [&](size_t j) {
            unsigned char* r = pool + (j % sets) * stride;
            return dccl_local_reduce(r + top + gap, r, 7, n, 0, st);
        };
        for (size_t j = 0; j < 8 && rc == 0; ++j) rc = launch(j);
        if (rc != 0 || hipStreamSynchronize(st) != hipSuccess) { rc = rc ? rc : 1; break; }
        // ~20 ms of launches at the size's expected duration (at least 2 us, else 3 nb at 6.5 TB/s)
        double t_est = 3.0 * double(nb) / 6.5e12;
        if (t_est < 2e-6) t_est = 2e-6;
        size_t launches = size_t(20e-3 / t_est);
        if (launches > 20000) launches = 20000;
        if (launches < 20) launches = 20;
        (void)hipEventRecord(e0, st);
        for (size_t j = 0; j < launches && rc == 0; ++j) rc = launch(j);
        (void)hipEventRecord(e1, st);
        if (rc != 0 || hipEventSynchronize(e1) != hipSuccess) { rc = rc ? rc : 1; break; }
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double us = 1e3 * double(ms) / double(launches);
        std::printf("{\"bytes_per_operand\": %zu, \"sets\": %zu, \"launches\": %zu, \"native_eager_us_per_launch\": %.3f, "
                    "\"native_eager_frac\": %.4f}\n",
                    nb, sets, launches, us, 3.0 * double(nb) / (us * 1e-6) / 1e9 / 8000.0);
        std::fflush(stdout);
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(st);
    (void)hipFree(pool);
    if (rc != 0) std::fprintf(stderr, "c4_native: %s\n", dccl_result_string(rc));
    return rc == 0 ? 0 : 1;
}
