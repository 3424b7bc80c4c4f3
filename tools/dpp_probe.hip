// tools/dpp_probe.hip — which lane does each DPP wave-level shift read on gfx950 (wave_shl:1 0x130,
// wave_rol:1 0x134, wave_shr:1 0x138, wave_ror:1 0x13C), and what does a lane with no source get?
// Lane i starts with 100 + i; old = -1.  Prints one line per control.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void probe(int* out) {
    const int x = 100 + int(threadIdx.x);
    out[0 * 64 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x130, 0xF, 0xF, false);
    out[1 * 64 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x134, 0xF, 0xF, false);
    out[2 * 64 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x138, 0xF, 0xF, false);
    out[3 * 64 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x13C, 0xF, 0xF, false);
}

int main() {
    int* d = nullptr;
    int h[256];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    probe<<<1, 64>>>(d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char* names[4] = {"wave_shl1", "wave_rol1", "wave_shr1", "wave_ror1"};
    for (int c = 0; c < 4; ++c) {
        std::printf("%s:", names[c]);
        for (int i = 0; i < 64; ++i) std::printf(" %d", h[c * 64 + i]);
        std::printf("\n");
    }
    (void)hipFree(d);
    return 0;
}
