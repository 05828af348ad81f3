// free_probe — which HIP runtime calls wait for unrelated device work (ROCm 7.2,
// MI355X)?  A bounded spin kernel (300 ms of wall clock, one block) runs on stream A;
// meanwhile this thread times, one at a time, the calls an index free / growth makes
// on its own stream B: pool alloc + hipFreeAsync, hipMalloc + hipFree, hipHostMalloc +
// hipHostFree, stream and event create / destroy, hipStreamSynchronize(B).  A call
// that takes ~the kernel's remaining time waited for the device.
// build: make -C tools free_probe     usage: free_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdint>
#include <functional>
#include <thread>

__global__ void spin_kernel(uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

using clk = std::chrono::steady_clock;

static double ms_of(const std::function<void()>& f) {
    const auto t0 = clk::now();
    f();
    return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
}

int main() {
    hipStream_t sa = nullptr, sb = nullptr;
    if (hipStreamCreateWithFlags(&sa, hipStreamNonBlocking) != hipSuccess) return 1;
    if (hipStreamCreateWithFlags(&sb, hipStreamNonBlocking) != hipSuccess) return 1;
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = 0;
    hipMemPool_t pool = nullptr;
    if (hipMemPoolCreate(&pool, &props) != hipSuccess) return 1;
    uint64_t keep = UINT64_MAX;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    // warm everything once with the device idle
    void* p = nullptr;
    (void)hipMallocFromPoolAsync(&p, 64 << 20, pool, sb);
    (void)hipFreeAsync(p, sb);
    (void)hipStreamSynchronize(sb);
    // wall_clock64 runs at 100 MHz: 300 ms
    const uint64_t ticks = 30000000ull;
    struct Case {
        const char* name;
        std::function<void()> f;
    };
    void* q = nullptr;
    void* h = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t ev = nullptr;
    Case cases[] = {
        {"pool_alloc_64MiB", [&] { (void)hipMallocFromPoolAsync(&q, 64 << 20, pool, sb); }},
        {"hipFreeAsync", [&] { (void)hipFreeAsync(q, sb); }},
        {"pool_alloc_1GiB", [&] { (void)hipMallocFromPoolAsync(&q, (size_t)1 << 30, pool, sb); }},
        {"hipFreeAsync_1GiB", [&] { (void)hipFreeAsync(q, sb); }},
        {"hipStreamSynchronize_own", [&] { (void)hipStreamSynchronize(sb); }},
        {"hipMalloc_64MiB", [&] { (void)hipMalloc(&q, 64 << 20); }},
        {"hipFree", [&] { (void)hipFree(q); }},
        {"hipHostMalloc_16MiB", [&] { (void)hipHostMalloc(&h, 16 << 20, hipHostMallocDefault); }},
        {"hipHostFree", [&] { (void)hipHostFree(h); }},
        {"hipStreamCreate", [&] { (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking); }},
        {"hipStreamDestroy_idle", [&] { (void)hipStreamDestroy(st); }},
        {"hipEventCreate", [&] { (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming); }},
        {"hipEventRecord_own", [&] { (void)hipEventRecord(ev, sb); }},
        {"hipEventDestroy", [&] { (void)hipEventDestroy(ev); }},
    };
    std::printf("{");
    bool first = true;
    for (const Case& c : cases) {
        hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, sa, ticks);
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
        const double ms = ms_of(c.f);
        const double rest = ms_of([&] { (void)hipStreamSynchronize(sa); });
        std::printf("%s\"%s\": [%.3f, %.1f]", first ? "" : ", ", c.name, ms, rest);
        first = false;
        std::fflush(stdout);
    }
    std::printf("}\n");
    (void)hipDeviceSynchronize();
    return 0;
}
