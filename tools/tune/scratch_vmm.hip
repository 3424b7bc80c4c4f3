// tools/tune/scratch_vmm.hip — tuning only: device scratch allocated through the HIP virtual
// memory API in granules whose physical creation order differs from their virtual order, to see whether the
// scratchpad's physical placement moves DCCL's ring-step combine (send = library scratch, recv = a chunk of a
// separate user buffer) between the DRAM's fast and slow service modes.
//
//   int vmm_alloc(size_t bytes, size_t granule, int order, void** out)
//     order 0: granule i created i-th, mapped at slot i (sequential)
//     order 1: created i-th, mapped at slot n-1-i (reversed)
//     order 2: created i-th, mapped at slot 2i (i < n/2) or 2(i - n/2) + 1 (two interleaved halves)
//     order 3: one physical allocation of the whole size (granule ignored)
//   int vmm_free(void* p)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <mutex>
#include <vector>

namespace {
struct Mapping {
    size_t bytes;
    std::vector<hipMemGenericAllocationHandle_t> handles;
};
std::mutex mu;
std::map<void*, Mapping> live;

hipMemAllocationProp prop_for(int dev) {
    hipMemAllocationProp p{};
    p.type = hipMemAllocationTypePinned;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = dev;
    return p;
}
}  // namespace

extern "C" int vmm_granularity(size_t* g) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1;
    hipMemAllocationProp p = prop_for(dev);
    return hipMemGetAllocationGranularity(g, &p, hipMemAllocationGranularityMinimum) == hipSuccess ? 0 : 2;
}

extern "C" int vmm_alloc(size_t bytes, size_t granule, int order, void** out) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1;
    hipMemAllocationProp p = prop_for(dev);
    size_t g = 0;
    if (hipMemGetAllocationGranularity(&g, &p, hipMemAllocationGranularityMinimum) != hipSuccess) return 2;
    if (order == 3) granule = bytes;
    granule = (granule + g - 1) / g * g;
    bytes = (bytes + granule - 1) / granule * granule;
    const size_t n = bytes / granule;
    void* base = nullptr;
    if (hipMemAddressReserve(&base, bytes, size_t(2) << 20, nullptr, 0) != hipSuccess) return 3;
    Mapping m{bytes, {}};
    for (size_t i = 0; i < n; ++i) {
        hipMemGenericAllocationHandle_t h{};
        if (hipMemCreate(&h, granule, &p, 0) != hipSuccess) return 4;
        size_t slot = i;
        if (order == 1) slot = n - 1 - i;
        if (order == 2) slot = i < n / 2 ? 2 * i : 2 * (i - n / 2) + 1;
        if (order == 2 && n % 2 && i == n - 1) slot = n - 1;
        if (hipMemMap(static_cast<char*>(base) + slot * granule, granule, 0, h, 0) != hipSuccess) return 5;
        m.handles.push_back(h);
    }
    hipMemAccessDesc a{};
    a.location.type = hipMemLocationTypeDevice;
    a.location.id = dev;
    a.flags = hipMemAccessFlagsProtReadWrite;
    if (hipMemSetAccess(base, bytes, &a, 1) != hipSuccess) return 6;
    std::lock_guard<std::mutex> lock(mu);
    live[base] = std::move(m);
    *out = base;
    return 0;
}

extern "C" int vmm_free(void* base) {
    std::lock_guard<std::mutex> lock(mu);
    auto it = live.find(base);
    if (it == live.end()) return 1;
    (void)hipDeviceSynchronize();
    (void)hipMemUnmap(base, it->second.bytes);
    for (auto h : it->second.handles) (void)hipMemRelease(h);
    (void)hipMemAddressFree(base, it->second.bytes);
    live.erase(it);
    return 0;
}

// hipExtMallocWithFlags with a flag (hipDeviceMallocContiguous = 4: physically contiguous), for the placement
// probe (tools/alloc_probe.py); free with hipFree.
extern "C" int ext_alloc(size_t bytes, unsigned flags, void** out) {
    return hipExtMallocWithFlags(out, bytes, flags) == hipSuccess ? 0 : 1;
}
extern "C" int ext_free(void* p) { return hipFree(p) == hipSuccess ? 0 : 1; }
