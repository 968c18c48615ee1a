// Issue rate of the run-tagged DP cell's instruction MIX on gfx950 (tools/, not product code): the
// k_align<24, true, 6> cell is 6 full-rate VOP2 ops and 3 maxes (v_max_i32 x2, v_max3_i32), which
// tools/valu_microbench.hip measures at ~0.40 and ~0.235 wave-instructions per SIMD-cycle alone.
// Here the mix runs as 8 independent chains per lane (no memory, no dependency limit), at 2-8
// waves per SIMD, so its rate is the ceiling any kernel with that mix can reach; the untagged cell
// (7 + 3) is measured too. Build: hipcc --offload-arch=gfx950 -O2 -o cellmix_bench tools/cellmix_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048
#define R8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)
#define ADD(i) "v_add_u32 %" #i ", %" #i ", %8\n"
#define SUB(i) "v_sub_u32 %" #i ", %" #i ", %8\n"
#define OR(i) "v_or_b32 %" #i ", %" #i ", %8\n"
#define AND(i) "v_and_b32 %" #i ", %" #i ", %9\n"
#define XOR(i) "v_xor_b32 %" #i ", %" #i ", %8\n"
#define MAX(i) "v_max_i32 %" #i ", %" #i ", %8\n"
#define MAX3(i) "v_max3_i32 %" #i ", %" #i ", %8, %9\n"
#define REGS : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c)

// 6 full-rate + 3 half-rate per chain and iteration (72 wave-instructions)
__global__ __launch_bounds__(256) void k_mix_tagged(int *out, int seed) {
    int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    int b = seed, c = ~seed;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(R8(ADD) R8(MAX) R8(OR) R8(ADD) R8(MAX) R8(SUB) R8(MAX3) R8(XOR) R8(AND) REGS);
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// 7 full-rate + 3 half-rate (80 wave-instructions)
__global__ __launch_bounds__(256) void k_mix_untagged(int *out, int seed) {
    int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    int b = seed, c = ~seed;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(R8(ADD) R8(MAX) R8(OR) R8(ADD) R8(MAX) R8(SUB) R8(MAX3) R8(XOR) R8(AND) R8(OR) REGS);
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

static void run(void (*k)(int *, int), const char *name, int per_iter, int *d, int blocks_per_cu) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * blocks_per_cu;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 3);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 3);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double instrs = 3.0 * blocks * 4 * ITERS * per_iter;   // wave-instructions
    const double per_simd = instrs / 1024.0;                      // 256 CU x 4 SIMD
    printf("%-16s waves/SIMD=%d  %.3f ms  %.3f wave-instr/cycle/SIMD at 2.4 GHz\n", name, blocks_per_cu, ms,
           per_simd / (ms * 1e-3 * 2.4e9));
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    int *d;
    hipMalloc(&d, 256 * 8 * 256 * sizeof(int));
    for (int b : {2, 4, 6, 8}) run(k_mix_tagged, "tagged 6+3", 72, d, b);
    for (int b : {2, 4, 6, 8}) run(k_mix_untagged, "untagged 7+3", 80, d, b);
    hipFree(d);
    return 0;
}
