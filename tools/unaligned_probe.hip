// tools/unaligned_probe.hip — does gfx950 take 16-B global loads / stores at any byte address, and how fast?
// (tuning only)  fp32 Sum over 1 GiB operands with recv and send displaced by (roff, soff) bytes: every
// lane moves 16 B of whole elements with ONE global_load_dwordx4 / global_store_dwordx4 at the displaced
// address (align-1 pointer types; gfx950 code objects are built with unaligned access mode).  Adjacent
// lanes' 16-B pieces are disjoint, so no byte is written by two lanes.  Checks every element against a
// host loop on a sample, times with HIP events, prints one JSON line per (roff, soff).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));

template <bool NT>
__global__ __launch_bounds__(64) void add_unaligned(const unsigned char* s, unsigned char* r, size_t nvec) {
    const size_t i = size_t(blockIdx.x) * 64 + threadIdx.x;
    if (i < nvec) {
        const u32x4 a = *reinterpret_cast<const u32x4_u*>(r + 16 * i);
        const u32x4 b = *reinterpret_cast<const u32x4_u*>(s + 16 * i);
        const f32x4 c = __builtin_bit_cast(f32x4, a) + __builtin_bit_cast(f32x4, b);
        *reinterpret_cast<u32x4_u*>(r + 16 * i) = __builtin_bit_cast(u32x4, c);
    }
}

#define CHECK(x) do { if ((x) != hipSuccess) { std::printf("{\"error\": \"%s\"}\n", #x); return 1; } } while (0)

int main(int argc, char** argv) {
    const size_t nbytes = size_t(1) << 30, nvec = nbytes / 16 - 2;
    unsigned char *s = nullptr, *r = nullptr;
    CHECK(hipMalloc(&s, nbytes + 256));
    CHECK(hipMalloc(&r, nbytes + 256));
    std::vector<float> hs(1 << 20), hr(1 << 20), out(1 << 20);
    for (size_t i = 0; i < hs.size(); ++i) { hs[i] = float(i % 1000) * 0.5f; hr[i] = float(i % 777) - 3.0f; }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int offs[][2] = {{0, 0}, {1, 0}, {2, 0}, {3, 0}, {5, 9}, {0, 1}, {0, 4}, {4, 4}, {8, 12}};
    for (auto& o : offs) {
        const int roff = o[0], soff = o[1];
        // correctness on the first 4 MiB: host data in, device result back
        CHECK(hipMemcpy(s + soff, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(r + roff, hr.data(), hr.size() * 4, hipMemcpyHostToDevice));
        add_unaligned<false><<<(hs.size() / 4 + 63) / 64, 64>>>(s + soff, r + roff, hs.size() / 4);
        CHECK(hipMemcpy(out.data(), r + roff, out.size() * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < out.size(); ++i) bad += out[i] != hr[i] + hs[i];
        // speed on 1 GiB
        const unsigned grid = unsigned((nvec + 63) / 64);
        add_unaligned<false><<<grid, 64>>>(s + soff, r + roff, nvec);
        CHECK(hipEventRecord(e0));
        const int reps = 20;
        for (int k = 0; k < reps; ++k) add_unaligned<false><<<grid, 64>>>(s + soff, r + roff, nvec);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        std::printf("{\"roff\": %d, \"soff\": %d, \"bad_elements\": %zu, \"ms\": %.4f, \"frac\": %.4f}\n", roff, soff, bad,
                    ms, 3.0 * nvec * 16 / (ms * 1e-3) / 8e12);
    }
    return 0;
}
