// Host cost of a kernel launch and the GPU's time per back-to-back tiny kernel on gfx950: N
// launches of an empty kernel (grid 1 and grid 1024) on one stream, host time of the enqueue loop
// and device time (events) of the whole run; the same N launches captured once in a hipGraph and
// replayed. Build: hipcc --offload-arch=gfx950 -O2 -o launch_bench tools/launch_bench.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_empty(int *p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = 1;
}

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                     \
            return 1;                                                               \
        }                                                                           \
    } while (0)

int main() {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int N = 2000;
    for (int grid : {1, 1024}) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipStreamSynchronize(st));
            const auto t0 = std::chrono::steady_clock::now();
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, st, nullptr);
            CK(hipEventRecord(e1, st));
            const auto t1 = std::chrono::steady_clock::now();
            CK(hipStreamSynchronize(st));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::printf("grid %4d: host enqueue %.2f us/launch, device %.2f us/kernel\n", grid,
                        std::chrono::duration<double, std::micro>(t1 - t0).count() / N, 1e3 * ms / N);
        }
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, st, nullptr);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        const auto t0 = std::chrono::steady_clock::now();
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < N / 100; ++i) CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        const auto t1 = std::chrono::steady_clock::now();
        CK(hipStreamSynchronize(st));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("grid %4d graph of 100: host %.2f us/kernel, device %.2f us/kernel\n", grid,
                    std::chrono::duration<double, std::micro>(t1 - t0).count() / N, 1e3 * ms / N);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}
