// tools/sync_latency.hip — cross-stream hand-off latency on one MI355X (tuning tool, not product).
//
// The in-process ring moves a chunk from rank r's stream to rank r+1's stream every step; each
// hand-off is a cross-stream dependency.  This ping-pong measures one hand-off (a tiny kernel on
// stream A, then a tiny kernel on stream B that depends on it, and back) for four mechanisms:
//   event   hipEventRecord on A + hipStreamWaitEvent on B (what comm.cpp uses)
//   value   hipStreamWriteValue32 on A + hipStreamWaitValue32 on B (signal memory)
//   poll    the host spins on hipEventQuery(A's event), then launches on B
//   sync    the host hipEventSynchronize(A's event), then launches on B
// Output: one JSON line per mechanism with microseconds per hand-off.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void tick(unsigned* p, unsigned v) {
    if (threadIdx.x == 0) p[0] = v;
}

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));        \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
    hipStream_t s[2];
    for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    unsigned* scratch = nullptr;
    CK(hipMalloc(&scratch, 256));
    hipEvent_t ev[2];
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int can_wait = 0;
    CK(hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, 0));
    unsigned *sig = nullptr, *hostflag = nullptr, *devflag = nullptr;
    if (can_wait && hipExtMallocWithFlags(reinterpret_cast<void**>(&sig), 8, hipMallocSignalMemory) != hipSuccess) {
        (void)hipGetLastError();
        sig = nullptr;
    }
    CK(hipHostMalloc(reinterpret_cast<void**>(&hostflag), 64, hipHostMallocCoherent));
    CK(hipMalloc(reinterpret_cast<void**>(&devflag), 64));

    for (const char* mode : {"event", "value-signal", "value-host", "value-device", "poll", "sync"}) {
        unsigned* flag = !std::strcmp(mode, "value-signal") ? sig
                         : !std::strcmp(mode, "value-host") ? hostflag
                         : !std::strcmp(mode, "value-device") ? devflag : nullptr;
        if (!std::strncmp(mode, "value", 5) && (!can_wait || flag == nullptr)) {
            std::printf("{\"mode\": \"%s\", \"supported\": false}\n", mode);
            continue;
        }
        if (flag == sig && flag) *flag = 0;
        else if (flag == hostflag) *flag = 0;
        else if (flag) CK(hipMemset(flag, 0, 4));
        CK(hipDeviceSynchronize());
        const int warm = 50;
        std::chrono::steady_clock::time_point t0;
        for (int i = 0; i < warm + iters; ++i) {
            if (i == warm) {
                CK(hipDeviceSynchronize());
                t0 = std::chrono::steady_clock::now();
            }
            const int a = i & 1, b = a ^ 1;
            // kernel on stream a (stream b's previous kernel must have finished: the hand-off of i-1)
            hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, s[a], scratch + a, unsigned(i));
            if (!std::strcmp(mode, "event")) {
                CK(hipEventRecord(ev[a], s[a]));
                CK(hipStreamWaitEvent(s[b], ev[a], 0));
            } else if (!std::strncmp(mode, "value", 5)) {
                CK(hipStreamWriteValue32(s[a], flag, unsigned(i + 1), 0));
                CK(hipStreamWaitValue32(s[b], flag, unsigned(i + 1), hipStreamWaitValueGte, 0xFFFFFFFFu));
            } else {
                CK(hipEventRecord(ev[a], s[a]));
                if (!std::strcmp(mode, "poll")) {
                    while (hipEventQuery(ev[a]) == hipErrorNotReady) {
                    }
                } else {
                    CK(hipEventSynchronize(ev[a]));
                }
            }
        }
        CK(hipDeviceSynchronize());
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        std::printf("{\"mode\": \"%s\", \"us_per_handoff\": %.3f, \"iters\": %d}\n", mode, us / iters, iters);
        std::fflush(stdout);
    }
    // reference point: the same kernels back to back on one stream (no hand-off)
    CK(hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, s[0], scratch, unsigned(i));
    CK(hipDeviceSynchronize());
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    std::printf("{\"mode\": \"same-stream\", \"us_per_kernel\": %.3f, \"iters\": %d}\n", us / iters, iters);
    return 0;
}
