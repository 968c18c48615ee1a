// Which streams share a hardware queue: a 1-block kernel that waits ~300 us is launched on stream 0
// and on stream j together; the pair takes ~300 us when the streams sit on different hardware
// queues and ~600 us when one queue serialises them. Streams 1..11 are plain (creation order),
// then a high-priority stream and two CU-masked streams (hipExtStreamCreateWithCUMask).
// Build: hipcc --offload-arch=gfx950 -O2 -o queue_probe tools/queue_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void k_wait(long long ticks) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) {
    }
}

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                     \
            return 1;                                                               \
        }                                                                           \
    } while (0)

static double pair_us(hipStream_t a, hipStream_t b, long long ticks) {
    (void)hipDeviceSynchronize();
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, a, ticks);
    hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, b, ticks);
    (void)hipStreamSynchronize(a);
    (void)hipStreamSynchronize(b);
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
    int dev = 0, rate = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, dev));   // kHz
    const long long ticks = (long long)rate * 300 / 1000;                      // ~300 us
    std::vector<hipStream_t> s(12);
    for (auto &x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t sp;
    CK(hipStreamCreateWithPriority(&sp, hipStreamNonBlocking, hi));
    const uint32_t all[8] = {~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u};
    hipStream_t sc1, sc2;
    CK(hipExtStreamCreateWithCUMask(&sc1, 8, all));
    CK(hipExtStreamCreateWithCUMask(&sc2, 8, all));
    (void)pair_us(s[0], s[1], ticks);   // warm-up
    std::printf("wall clock %d kHz, priority range %d..%d\n", rate, lo, hi);
    std::printf("alone: %.0f us\n", pair_us(s[0], s[0], ticks) / 2);
    for (int j = 1; j < 12; ++j) std::printf("s0 + s%-2d: %.0f us\n", j, pair_us(s[0], s[j], ticks));
    for (int j = 2; j < 6; ++j) std::printf("s1 + s%-2d: %.0f us\n", j, pair_us(s[1], s[j], ticks));
    std::printf("s0 + high priority: %.0f us\n", pair_us(s[0], sp, ticks));
    std::printf("s0 + cu-masked 1: %.0f us\n", pair_us(s[0], sc1, ticks));
    std::printf("cu-masked 1 + 2: %.0f us\n", pair_us(sc1, sc2, ticks));
    for (int j = 1; j < 6; ++j) std::printf("cu-masked 1 + s%d: %.0f us\n", j, pair_us(sc1, s[j], ticks));
    return 0;
}
