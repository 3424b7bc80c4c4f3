// tools/chain_waves_ab.cpp — A/B of the host chain combine's wave cap (DCCL_HOST_CHAIN_WAVES; the shipped 256 is
// host_staged.cpp's chain_waves): dccl_local_reduce_chain_host per call, registered and pageable operands
// (profiles/r6_chain_host_waves.json).
//   hipcc -std=c++17 -O2 -I include tools/chain_waves_ab.cpp -o /tmp/ab -L dccl_amd/lib -ldccl_amd -Wl,-rpath,$PWD/dccl_amd/lib
//   for c in 0 256 512 1024; do DCCL_...WAVES=$c /tmp/ab; done     (one JSON line per case)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "dccl/dccl_reduce.h"
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "%s failed line %d\n", #x, __LINE__); exit(1);} } while (0)
int main() {
    const size_t S_MAX = size_t(64) << 20;
    const int K_MAX = 7;
    unsigned char* reg[K_MAX + 1]; unsigned char* pag[K_MAX + 1];
    for (int i = 0; i <= K_MAX; ++i) {
        reg[i] = (unsigned char*)aligned_alloc(4096, S_MAX); memset(reg[i], 0, S_MAX);
        CK(hipHostRegister(reg[i], S_MAX, hipHostRegisterDefault));
        pag[i] = (unsigned char*)aligned_alloc(4096, S_MAX); memset(pag[i], 0, S_MAX);
    }
    const char* cap = getenv("DCCL_HOST_CHAIN_WAVES");
    const size_t sizes[] = {1 << 20, 16 << 20, 64 << 20};
    const int ks[] = {1, 3, 7};
    for (int kind = 0; kind < 2; ++kind)
        for (int k : ks)
            for (size_t S : sizes) {
                unsigned char** b = kind ? pag : reg;
                const void* sends[8];
                for (int j = 0; j < k; ++j) sends[j] = b[j + 1];
                const size_t n = S / 4;
                int reps = S <= (1 << 20) ? 300 : 20;
                if (dccl_local_reduce_chain_host(sends, k, b[0], b[0], 7, n, 0)) return 2;
                double best = 1e9;
                for (int trial = 0; trial < 3; ++trial) {
                    double t0 = now();
                    for (int i = 0; i < reps; ++i) if (dccl_local_reduce_chain_host(sends, k, b[0], b[0], 7, n, 0)) return 2;
                    double t = (now() - t0) / reps; if (t < best) best = t;
                }
                printf("{\"cap\": \"%s\", \"kind\": \"%s\", \"k\": %d, \"bytes\": %zu, \"us\": %.1f, \"gib_s_k_plus_2\": %.2f}\n", cap ? cap : "0",
                       kind ? "pageable" : "registered", k, S, best * 1e6, (k + 2) * S / best / (1 << 30));
                fflush(stdout);
            }
    return 0;
}
