// tools/launch_cost.hip — host issue cost per kernel launch on MI355X (tuning only): back-to-back launches of
// (a) dccl_local_reduce on 4 KiB operands, (b) an empty kernel through hipLaunchKernel, (c) the same kernel
// through hipModuleLaunchKernel with its hipFunction_t looked up once (hipGetFuncBySymbol), (d) the same
// kernel with triple-chevron syntax.  Host time per call (steady clock around the issue loop) and GPU time
// per launch (HIP events), one JSON line each.
//   hipcc --offload-arch=gfx950 -O2 -I include -I dccl_amd/csrc tools/launch_cost.hip -L dccl_amd/lib -ldccl_amd -o launch_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#include "dccl/dccl_reduce.h"
#include "reduce_kernels.hpp"

__global__ void empty_kernel(float* p) {
    if (p != nullptr && threadIdx.x == 1024) p[0] = 0.f;  // never true: keeps the argument
}

template <typename F>
static void time_it(const char* name, F&& f, hipStream_t st, int n) {
    for (int i = 0; i < 200; ++i) f();
    (void)hipStreamSynchronize(st);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, st);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) f();
    const auto t1 = std::chrono::steady_clock::now();
    (void)hipEventRecord(e1, st);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    // the same in batches of 256 launches, each followed by a sync: the host issue time of a batch that
    // cannot fill the device queue (no back-pressure), apart from the GPU's own time per launch
    double host_batch = 0.0;
    const int batches = n / 256;
    for (int b = 0; b < batches; ++b) {
        const auto b0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 256; ++i) f();
        host_batch += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - b0).count();
        (void)hipStreamSynchronize(st);
    }
    std::printf("{\"what\": \"%s\", \"host_us_per_call\": %.3f, \"gpu_us_per_launch\": %.3f, "
                "\"host_us_per_call_batched\": %.3f}\n", name,
                std::chrono::duration<double, std::micro>(t1 - t0).count() / n, 1e3 * ms / n,
                host_batch / (256.0 * batches));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main() {
    hipStream_t st;
    if (hipStreamCreate(&st) != hipSuccess) return 3;
    float* buf = nullptr;
    if (hipMalloc(&buf, 1 << 20) != hipSuccess) return 3;
    (void)hipMemset(buf, 0, 1 << 20);
    const int n = 20000;
    time_it("dccl_local_reduce 4 KiB", [&] { (void)dccl_local_reduce(buf + 4096, buf, 7, 1024, 0, st); }, st, n);
    void* args[] = {&buf};
    time_it("hipLaunchKernel empty 1x64",
            [&] { (void)hipLaunchKernel(reinterpret_cast<const void*>(&empty_kernel), dim3(1), dim3(64), args, 0, st); },
            st, n);
    hipFunction_t fn = nullptr;
    if (hipGetFuncBySymbol(&fn, reinterpret_cast<const void*>(&empty_kernel)) == hipSuccess) {
        time_it("hipModuleLaunchKernel empty 1x64",
                [&] { (void)hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, st, args, nullptr); }, st, n);
    }
    time_it("triple chevron empty 1x64", [&] { empty_kernel<<<1, 64, 0, st>>>(buf); }, st, n);
    {  // the library's kernel, instantiated here (TAG 2), launched directly with the library's arguments
        using C = dccl_amd::VecCfg<64, 1, 7, false, 2>;
        const unsigned char* sp = reinterpret_cast<const unsigned char*>(buf + 4096);
        unsigned char* rp = reinterpret_cast<unsigned char*>(buf);
        size_t head = 0, nvec = 256, tail = 0;
        void* kargs[] = {&sp, &rp, &head, &nvec, &tail};
        time_it("hipLaunchKernel reduce_vec_kernel 4x64 (4 KiB)", [&] {
            (void)hipLaunchKernel(reinterpret_cast<const void*>(&dccl_amd::reduce_vec_kernel<float, 0, C>), dim3(4),
                                  dim3(64), kargs, 0, st);
        }, st, n);
        time_it("dccl_local_reduce 4 KiB (again)", [&] { (void)dccl_local_reduce(buf + 4096, buf, 7, 1024, 0, st); },
                st, n);
    }
    time_it("hipLaunchKernel empty 4x64",
            [&] { (void)hipLaunchKernel(reinterpret_cast<const void*>(&empty_kernel), dim3(4), dim3(64), args, 0, st); },
            st, n);
    (void)hipFree(buf);
    (void)hipStreamDestroy(st);
    return 0;
}
