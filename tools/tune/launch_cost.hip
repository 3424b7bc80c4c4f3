// tools/tune/launch_cost.hip — tuning only: host cost of issuing one small combine launch by three HIP entry
// points, for the eager small-size launches of DCCL's step loop (C1's 1 KiB chunks, C4 below ~1 MiB):
//   mode 0: hipLaunchKernel(host stub, ...)                      (the product's launch())
//   mode 1: hipModuleLaunchKernel(hipFunction_t cached from hipGetFuncBySymbol, ...)
//   mode 2: hipExtLaunchKernel(host stub, ..., no events)
// lc_run issues `n` back-to-back launches of a one-block fp32 Sum combine of `count` elements on `stream` and
// returns the host seconds per launch spent issuing them (*drain_s: until the stream drained).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>

#include "reduce_kernels.hpp"

using namespace dccl_amd;

namespace {
using Cfg = VecCfg<64, 1, kNtSend | kNtRecv | kNtStore, false>;
const void* kernel_ptr() { return reinterpret_cast<const void*>(&reduce_vec_kernel<float, kSum, Cfg>); }
}  // namespace

extern "C" double lc_run(int mode, int n, const void* send, void* recv, size_t count, void* stream, double* drain_s) {
    hipStream_t st = static_cast<hipStream_t>(stream);
    const unsigned char* s = static_cast<const unsigned char*>(send);
    unsigned char* r = static_cast<unsigned char*>(recv);
    Split sp = split_for_vectors<float>(reinterpret_cast<uintptr_t>(r), count, 128);
    size_t grid = ceil_div(sp.nvec, size_t(64));
    if (grid == 0) grid = 1;
    void* args[] = {&s, &r, &sp.head, &sp.nvec, &sp.tail};
    hipFunction_t f = nullptr;
    if (mode == 1 && hipGetFuncBySymbol(&f, kernel_ptr()) != hipSuccess) return -1.0;
    (void)hipStreamSynchronize(st);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) {
        hipError_t e = hipSuccess;
        if (mode == 0)
            e = hipLaunchKernel(kernel_ptr(), dim3(unsigned(grid)), dim3(64), args, 0, st);
        else if (mode == 1)
            e = hipModuleLaunchKernel(f, unsigned(grid), 1, 1, 64, 1, 1, 0, st, args, nullptr);
        else
            e = hipExtLaunchKernel(kernel_ptr(), dim3(unsigned(grid)), dim3(64), args, 0, st, nullptr, nullptr, 0);
        if (e != hipSuccess) return -2.0;
    }
    const auto t1 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(st);
    const auto t2 = std::chrono::steady_clock::now();
    if (drain_s) *drain_s = std::chrono::duration<double>(t2 - t0).count() / n;
    return std::chrono::duration<double>(t1 - t0).count() / n;
}
