// VALU issue-rate microbenchmark for gfx950 (tools/, not product code).
// Each kernel runs a fully unrolled stream of INDEPENDENT instructions of one kind (8
// accumulators, inline asm so the compiler cannot fold them) and reports wave-instructions per
// cycle per SIMD, to calibrate the VALU roofline peak used by bench.py for integer DP work.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define ITERS 4096

#define BODY8(INS)                                                                              \
    asm volatile(INS " %0, %0, %8\n" INS " %1, %1, %8\n" INS " %2, %2, %8\n" INS " %3, %3, %8\n" \
                 INS " %4, %4, %8\n" INS " %5, %5, %8\n" INS " %6, %6, %8\n" INS " %7, %7, %8\n" \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                 : "v"(b));

#define KERNEL(NAME, INS)                                                                       \
    __global__ __launch_bounds__(256) void NAME(int *out, int seed) {                           \
        int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,  \
            a6 = a0 + 6, a7 = a0 + 7, b = seed;                                                 \
        for (int i = 0; i < ITERS; ++i) {                                                       \
            BODY8(INS) BODY8(INS) BODY8(INS) BODY8(INS)                                         \
        }                                                                                       \
        out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;            \
    }

KERNEL(k_add_u32, "v_add_u32")
KERNEL(k_max_i32, "v_max_i32")
KERNEL(k_or_b32, "v_or_b32")
KERNEL(k_add_f32, "v_add_f32")
KERNEL(k_pk_add_u16, "v_pk_add_u16")
KERNEL(k_pk_max_i16, "v_pk_max_i16")
KERNEL(k_max_f32, "v_max_f32")
KERNEL(k_max_u32, "v_max_u32")
KERNEL(k_sub_u32, "v_sub_u32")
KERNEL(k_xor_b32, "v_xor_b32")
KERNEL(k_and_b32, "v_and_b32")
KERNEL(k_min_u32, "v_min_u32")
KERNEL(k_lshr_b32, "v_lshrrev_b32")
KERNEL(k_max_i16, "v_max_i16")
KERNEL(k_max_u16, "v_max_u16")
KERNEL(k_pk_max_u16, "v_pk_max_u16")
KERNEL(k_max_f16, "v_max_f16")
KERNEL(k_pk_max_f16, "v_pk_max_f16")

#define KERNEL3(NAME, INS)                                                                      \
    __global__ __launch_bounds__(256) void NAME(int *out, int seed) {                           \
        int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,  \
            a6 = a0 + 6, a7 = a0 + 7, b = seed, c = seed + 1;                                   \
        for (int i = 0; i < ITERS; ++i) {                                                       \
            _Pragma("unroll") for (int k = 0; k < 4; ++k)                                       \
            asm volatile(INS " %0, %0, %8, %9\n" INS " %1, %1, %8, %9\n" INS " %2, %2, %8, %9\n" \
                         INS " %3, %3, %8, %9\n" INS " %4, %4, %8, %9\n" INS " %5, %5, %8, %9\n" \
                         INS " %6, %6, %8, %9\n" INS " %7, %7, %8, %9\n"                        \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(b), "v"(c));                                                     \
        }                                                                                       \
        out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;            \
    }
KERNEL3(k_max3_f32, "v_max3_f32")
KERNEL3(k_add3_u32, "v_add3_u32")
KERNEL3(k_bfi_b32, "v_bfi_b32")
KERNEL3(k_perm_b32, "v_perm_b32")
KERNEL3(k_bfe_u32, "v_bfe_u32")
KERNEL3(k_med3_i32, "v_med3_i32")
KERNEL3(k_and_or_b32, "v_and_or_b32")
KERNEL3(k_mad_u24, "v_mad_u32_u24")
KERNEL3(k_lshl_add, "v_lshl_add_u32")
KERNEL3(k_max3_i16, "v_max3_i16")
KERNEL3(k_max3_u32, "v_max3_u32")
KERNEL3(k_or3_b32, "v_or3_b32")

// compare + select pattern, mask rewritten every pair (realistic DP usage)
__global__ __launch_bounds__(256) void k_cmp_cnd(int *out, int seed) {
    int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, b = seed;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            asm volatile("v_cmp_gt_i32 vcc, %0, %4\nv_cndmask_b32 %0, %0, %4, vcc\n"
                         "v_cmp_gt_i32 vcc, %1, %4\nv_cndmask_b32 %1, %1, %4, vcc\n"
                         "v_cmp_gt_i32 vcc, %2, %4\nv_cndmask_b32 %2, %2, %4, vcc\n"
                         "v_cmp_gt_i32 vcc, %3, %4\nv_cndmask_b32 %3, %3, %4, vcc\n"
                         "v_cmp_gt_i32 vcc, %0, %4\nv_cndmask_b32 %0, %0, %4, vcc\n"
                         "v_cmp_gt_i32 vcc, %1, %4\nv_cndmask_b32 %1, %1, %4, vcc\n"
                         "v_cmp_gt_i32 vcc, %2, %4\nv_cndmask_b32 %2, %2, %4, vcc\n"
                         "v_cmp_gt_i32 vcc, %3, %4\nv_cndmask_b32 %3, %3, %4, vcc\n"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
                         : "v"(b)
                         : "vcc");
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3;
}

// e64 compares into distinct SGPR pairs, then e64 selects (what hipcc emits)
__global__ __launch_bounds__(256) void k_cmp_cnd64(int *out, int seed) {
    int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, b = seed;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            asm volatile("v_cmp_gt_i32_e64 s[40:41], %0, %4\nv_cmp_gt_i32_e64 s[42:43], %1, %4\n"
                         "v_cmp_gt_i32_e64 s[44:45], %2, %4\nv_cmp_gt_i32_e64 s[46:47], %3, %4\n"
                         "v_cndmask_b32_e64 %0, %0, %4, s[40:41]\nv_cndmask_b32_e64 %1, %1, %4, s[42:43]\n"
                         "v_cndmask_b32_e64 %2, %2, %4, s[44:45]\nv_cndmask_b32_e64 %3, %3, %4, s[46:47]\n"
                         "v_cmp_gt_i32_e64 s[40:41], %0, %4\nv_cmp_gt_i32_e64 s[42:43], %1, %4\n"
                         "v_cmp_gt_i32_e64 s[44:45], %2, %4\nv_cmp_gt_i32_e64 s[46:47], %3, %4\n"
                         "v_cndmask_b32_e64 %0, %0, %4, s[40:41]\nv_cndmask_b32_e64 %1, %1, %4, s[42:43]\n"
                         "v_cndmask_b32_e64 %2, %2, %4, s[44:45]\nv_cndmask_b32_e64 %3, %3, %4, s[46:47]\n"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
                         : "v"(b)
                         : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3;
}

__global__ __launch_bounds__(256) void k_max3_i32(int *out, int seed) {
    int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
        a7 = a0 + 7, b = seed, c = seed + 1;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            asm volatile("v_max3_i32 %0, %0, %8, %9\nv_max3_i32 %1, %1, %8, %9\nv_max3_i32 %2, %2, %8, %9\n"
                         "v_max3_i32 %3, %3, %8, %9\nv_max3_i32 %4, %4, %8, %9\nv_max3_i32 %5, %5, %8, %9\n"
                         "v_max3_i32 %6, %6, %8, %9\nv_max3_i32 %7, %7, %8, %9\n"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(b), "v"(c));
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

__global__ __launch_bounds__(256) void k_cndmask(int *out, int seed) {
    int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
        a7 = a0 + 7, b = seed;
    asm volatile("v_cmp_gt_i32 vcc, %0, %1" ::"v"(a0), "v"(b) : "vcc");
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            asm volatile("v_cndmask_b32 %0, %0, %8, vcc\nv_cndmask_b32 %1, %1, %8, vcc\nv_cndmask_b32 %2, %2, %8, vcc\n"
                         "v_cndmask_b32 %3, %3, %8, vcc\nv_cndmask_b32 %4, %4, %8, vcc\nv_cndmask_b32 %5, %5, %8, vcc\n"
                         "v_cndmask_b32 %6, %6, %8, vcc\nv_cndmask_b32 %7, %7, %8, vcc\n"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(b)
                         : "vcc");
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

typedef void (*kfn)(int *, int);

static double run(kfn k, const char *name, int *d, int blocks_per_cu) {
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
    const double waves = 3.0 * blocks * 4;                   // 4 waves per block
    const double instrs = waves * ITERS * 32;                // 32 per iteration
    const double per_simd = instrs / 1024.0;                 // 256 CU x 4 SIMD
    const double cycles = ms * 1e-3 * 2.4e9;
    const double lane_ops = instrs * 64 / (ms * 1e-3) / 1e12;
    printf("%-14s blocks/CU=%d  %.3f ms  %.3f wave-instr/cycle/SIMD (at 2.4 GHz)  %.1f T lane-instr/s\n", name,
           blocks_per_cu, ms, per_simd / cycles, lane_ops);
    return per_simd / cycles;
}

int main() {
    int *d;
    hipMalloc(&d, 256 * 8 * 256 * sizeof(int));
    struct { kfn k; const char *n; } ks[] = {{k_add_u32, "v_add_u32"},   {k_max_i32, "v_max_i32"},
                                              {k_or_b32, "v_or_b32"},     {k_add_f32, "v_add_f32"},
                                              {k_max3_i32, "v_max3_i32"}, {k_cndmask, "v_cndmask_b32"},
                                              {k_pk_add_u16, "v_pk_add_u16"}, {k_pk_max_i16, "v_pk_max_i16"},
                                              {k_max_f32, "v_max_f32"}, {k_max_u32, "v_max_u32"},
                                              {k_sub_u32, "v_sub_u32"}, {k_xor_b32, "v_xor_b32"},
                                              {k_and_b32, "v_and_b32"}, {k_min_u32, "v_min_u32"},
                                              {k_lshr_b32, "v_lshrrev_b32"}, {k_max3_f32, "v_max3_f32"},
                                              {k_add3_u32, "v_add3_u32"}, {k_bfi_b32, "v_bfi_b32"},
                                              {k_perm_b32, "v_perm_b32"}, {k_bfe_u32, "v_bfe_u32"},
                                              {k_med3_i32, "v_med3_i32"}, {k_and_or_b32, "v_and_or_b32"},
                                              {k_mad_u24, "v_mad_u32_u24"}, {k_lshl_add, "v_lshl_add_u32"},
                                              {k_cmp_cnd, "cmp+cndmask32"}, {k_cmp_cnd64, "cmp+cndmask64"},
                                              {k_max_i16, "v_max_i16"}, {k_max_u16, "v_max_u16"}, {k_pk_max_u16, "v_pk_max_u16"},
                                              {k_max_f16, "v_max_f16"}, {k_pk_max_f16, "v_pk_max_f16"}, {k_max3_i16, "v_max3_i16"},
                                              {k_max3_u32, "v_max3_u32"}, {k_or3_b32, "v_or3_b32"}};
    for (auto &k : ks)
        for (int b : {2, 4}) run(k.k, k.n, d, b);
    hipFree(d);
    return 0;
}
