// tools/host_waves_ab.cpp — A/B of the zero-copy host combine's wave cap (DCCL_HOST_ZEROCOPY_WAVES; the shipped
// 512 is host_staged.cpp's zero_copy_waves): dccl_local_reduce_host per call vs size, registered and hipHostMalloc
// operands (profiles/r6_zero_copy_waves.json).
//   hipcc -std=c++17 -O2 -I include tools/host_waves_ab.cpp -o /tmp/ab -L dccl_amd/lib -ldccl_amd -Wl,-rpath,$PWD/dccl_amd/lib
//   for c in 0 256 512 1024; do DCCL_...WAVES=$c /tmp/ab; done     (one JSON line per case)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "dccl/dccl_reduce.h"
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "%s failed line %d\n", #x, __LINE__); exit(1);} } while (0)
int main(int argc, char** argv) {
    const size_t top = size_t(1) << 30;
    const size_t sizes[] = {65536, 1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20, size_t(1) << 30};
    unsigned char *rs = (unsigned char*)aligned_alloc(4096, top), *rr = (unsigned char*)aligned_alloc(4096, top);
    memset(rs, 0, top); memset(rr, 0, top);
    CK(hipHostRegister(rs, top, hipHostRegisterDefault)); CK(hipHostRegister(rr, top, hipHostRegisterDefault));
    unsigned char *ps, *pr;
    CK(hipHostMalloc((void**)&ps, top, hipHostMallocDefault)); CK(hipHostMalloc((void**)&pr, top, hipHostMallocDefault));
    memset(ps, 0, top); memset(pr, 0, top);
    const char* cap = getenv("DCCL_HOST_ZEROCOPY_WAVES");
    for (int kind = 0; kind < 2; ++kind) {
        unsigned char* s = kind ? ps : rs; unsigned char* r = kind ? pr : rr;
        for (size_t S : sizes) {
            const size_t n = S / 4, nsets = top / S;
            int reps = S <= (1 << 20) ? 1000 : (S <= (64 << 20) ? 40 : 5);
            if (dccl_local_reduce_host(s, r, 7, n, 0)) return 2;
            double best = 1e9;
            for (int trial = 0; trial < 3; ++trial) {
                double t0 = now();
                for (int i = 0; i < reps; ++i) { size_t k = (i % nsets) * S; if (dccl_local_reduce_host(s + k, r + k, 7, n, 0)) return 2; }
                const double t = (now() - t0) / reps;
                if (t < best) best = t;
            }
            printf("{\"cap\": \"%s\", \"kind\": \"%s\", \"bytes\": %zu, \"full_us\": %.2f, \"payload_gib_s\": %.2f}\n", cap ? cap : "0",
                   kind ? "pinned" : "registered", S, best * 1e6, S / best / (1 << 30));
            fflush(stdout);
        }
    }
    return 0;
}
