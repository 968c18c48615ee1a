// Replay microbenchmark of the dominant kernel's inner column (tools/, not product code; VERDICT r04
// item 3). tools/make_replay_k24.py extracts k_align<24, true, TAGGED>'s cross-mode column loop from
// the compiler's gfx950 assembly VERBATIM (profiles/r05/k_align24_inner_column.s) into
// replay_k24_body.inc; this kernel runs exactly that loop -- the same instructions, registers,
// dependency chains, LDS substitution-table reads and tile-layout look-ahead loads -- with the real
// kernel's block shape (256 threads, the 4 x 8 x 24-int LDS table), wave count (blocks = tiles x
// adapters), VGPR count (72: 7 waves per SIMD) and trip count (n - 1 = 149 columns of a 150-column
// window), and nothing else: no table fill from the adapter, no last column, no result store, no
// window tails. Its issue rate (SQ_INSTS_VALU per SIMD-cycle under rocprofv3 --pmc, and by events)
// is the ceiling of the kernel's loop on this hardware; variant `nolds` drops the LDS reads and
// their waits (the VALU + SALU mix alone).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/replay_k24 tools/replay_k24.hip
//   tools/replay_k24 [blocks=17986] [n=150] [reps=20]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "replay_k24_body.inc"

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

constexpr int kTabInts = 8 * 24;   // one wave's substitution table: 8 read codes x 24 slots
constexpr int kQuads = 40;         // tile rows (4-column chunks) per tile: >= n / 4 + 3

// Loop-register setup shared by the variants: every VGPR / SGPR the loop touches defined, then its
// live-ins -- window dwords (lo, hi, look-ahead) loaded from the lane's tile column, the tile stride
// (256 dwords), the LDS table base, row stride, window length, column counter, exit mask, shift,
// a8 = 0 and the first read code. Inputs only through SGPRs, so the kernel's VGPRs are the loop's 72.
#define RP_SETUP                                                                                          \
    "v_mov_b32 v0, 0\n v_mov_b32 v1, 0\n v_mov_b32 v2, 0\n v_mov_b32 v3, 0\n v_mov_b32 v4, 0\n"          \
    "v_mov_b32 v5, 0\n v_mov_b32 v11, 0\n v_mov_b32 v12, 0\n v_mov_b32 v13, 0\n v_mov_b32 v14, 0\n"      \
    "v_mov_b32 v15, 0\n v_mov_b32 v17, 0\n v_mov_b32 v19, 0\n v_mov_b32 v20, 0\n v_mov_b32 v21, 0\n"    \
    "v_mov_b32 v22, 0\n v_mov_b32 v23, 0\n v_mov_b32 v24, 0\n v_mov_b32 v25, 0\n v_mov_b32 v26, 0\n"    \
    "v_mov_b32 v27, 0\n v_mov_b32 v28, 0\n v_mov_b32 v29, 0\n v_mov_b32 v30, 0\n v_mov_b32 v31, 0\n"    \
    "v_mov_b32 v32, 0\n v_mov_b32 v33, 0\n v_mov_b32 v34, 0\n v_mov_b32 v35, 0\n v_mov_b32 v36, 0\n"    \
    "v_mov_b32 v37, 0\n v_mov_b32 v38, 0\n v_mov_b32 v39, 0\n v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n"    \
    "v_mov_b32 v42, 0\n v_mov_b32 v43, 0\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v46, 0\n"    \
    "v_mov_b32 v47, 0\n v_mov_b32 v48, 0\n v_mov_b32 v49, 0\n v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n"    \
    "v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n v_mov_b32 v54, 0\n v_mov_b32 v55, 0\n v_mov_b32 v56, 0\n"    \
    "v_mov_b32 v57, 0\n v_mov_b32 v58, 0\n v_mov_b32 v59, 0\n v_mov_b32 v60, 0\n v_mov_b32 v61, 0\n"    \
    "v_mov_b32 v62, 0\n v_mov_b32 v63, 0\n v_mov_b32 v64, 0\n v_mov_b32 v65, 0\n v_mov_b32 v66, 0\n"    \
    "v_mov_b32 v67, 0\n v_mov_b32 v68, 0\n v_mov_b32 v70, 0\n v_mov_b32 v71, 0\n"                         \
    "s_mov_b32 s16, 0xfffe0000\n s_mov_b32 s28, 0xfb000000\n s_mov_b32 s52, 0\n s_mov_b32 s54, 0\n"     \
    "s_mov_b32 s55, 0\n s_mov_b32 s58, 0\n s_mov_b32 s59, 0\n s_mov_b32 s60, 0\n"                        \
    "v_mbcnt_lo_u32_b32 v6, -1, 0\n v_mbcnt_hi_u32_b32 v6, -1, v6\n v_lshlrev_b32 v6, 2, v6\n"          \
    "v_mov_b32 v7, %[qhi]\n v_add_co_u32 v6, vcc, %[qlo], v6\n v_addc_co_u32 v7, vcc, 0, v7, vcc\n"   \
    "global_load_dword v8, v[6:7], off\n global_load_dword v9, v[6:7], off offset:1024\n"               \
    "global_load_dword v69, v[6:7], off offset:2048\n"                                                  \
    "v_mov_b32 v10, 256\n v_mov_b32 v16, %[ldsb]\n s_movk_i32 s57, 0x60\n v_mov_b32 v18, %[n]\n"       \
    "s_mov_b32 s53, 1\n s_mov_b64 s[2:3], 0\n s_mov_b32 s56, 8\n"                                       \
    "s_waitcnt vmcnt(0)\n v_and_b32 v0, 3, v8\n"

// tiles: n_tiles x kQuads x 256 dwords, every byte a Dna5 code 0..4 (the table rows the loop reads)
template <int V>
__global__ __launch_bounds__(256) void k_replay(const uint32_t *tiles, int n_tiles, int n) {
    __shared__ __attribute__((aligned(16))) int32_t tab[4 * kTabInts];
    for (int e = threadIdx.x; e < 4 * kTabInts; e += 256) tab[e] = (int32_t)((e * 2654435761u) >> 8);
    __syncthreads();
    const int tile = (int)(blockIdx.x % (unsigned)n_tiles);
    // this wave's 64 windows of the tile: column q of window w at dword q * 256 + w
    const uint64_t qa = (uint64_t)(uintptr_t)(tiles + ((int64_t)tile * kQuads * 256 + (threadIdx.x & ~63u)));
    const uint32_t qlo = __builtin_amdgcn_readfirstlane((uint32_t)qa), qhi = __builtin_amdgcn_readfirstlane((uint32_t)(qa >> 32));
    // the only static LDS array starts at LDS address 0
    const uint32_t ldsb = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) * kTabInts * 4);
    if constexpr (V == 0) {
        asm volatile(RP_SETUP "s_branch " RP_HEADER_EXACT "\n" RP_LOOP_EXACT ".Lrp_exact_exit:\n"
                     "s_or_b64 exec, exec, s[2:3]\n"
                     :
                     : [qlo] "s"(qlo), [qhi] "s"(qhi), [ldsb] "s"(ldsb), [n] "s"(n)
                     : RP_CLOBBER_V, RP_CLOBBER_S, "vcc", "scc", "memory");
    } else {
        asm volatile(RP_SETUP "s_branch " RP_HEADER_NOLDS "\n" RP_LOOP_NOLDS ".Lrp_nolds_exit:\n"
                     "s_or_b64 exec, exec, s[2:3]\n"
                     :
                     : [qlo] "s"(qlo), [qhi] "s"(qhi), [ldsb] "s"(ldsb), [n] "s"(n)
                     : RP_CLOBBER_V, RP_CLOBBER_S, "vcc", "scc", "memory");
    }
}

int main(int argc, char **argv) {
    const int blocks = argc > 1 ? std::atoi(argv[1]) : 17986;   // 391 tiles x 46 adapters: the headline launch
    const int n = argc > 2 ? std::atoi(argv[2]) : 150;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 20;
    const int n_tiles = 391;
    if (n < 2 || n / 4 + 3 > kQuads) {
        std::fprintf(stderr, "n must be in 2 .. %d\n", (kQuads - 3) * 4);
        return 1;
    }
    std::vector<uint32_t> h((size_t)n_tiles * kQuads * 256);
    uint32_t x = 12345;
    for (auto &w : h) {
        uint32_t v = 0;
        for (int b = 0; b < 4; ++b) {
            x = x * 1103515245u + 12345u;
            v |= ((x >> 16) % 5u) << (8 * b);
        }
        w = v;
    }
    uint32_t *d = nullptr;
    CHECK(hipMalloc(&d, h.size() * 4));
    CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double waves = 4.0 * blocks;
    const double passes = n - 1, loads = (n - 1 + 3) / 4;   // columns 1 .. n-1; a look-ahead every 4th
    for (int v = 0; v < 2; ++v) {
        auto launch = [&]() {
            if (v == 0) hipLaunchKernelGGL(k_replay<0>, dim3(blocks), dim3(256), 0, 0, d, n_tiles, n);
            else hipLaunchKernelGGL(k_replay<1>, dim3(blocks), dim3(256), 0, 0, d, n_tiles, n);
        };
        for (int w = 0; w < 3; ++w) launch();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) launch();
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        const double valu_main = (v == 0 ? RP_VALU_PER_PASS_MAIN : RP_VALU_PER_PASS_MAIN);
        const double valu = waves * (passes * valu_main + loads * RP_VALU_PER_PASS_LOAD);
        const double cells = waves * 64.0 * passes * 24.0;
        // wave-instructions per SIMD-cycle at a given clock: 256 CUs x 4 SIMDs
        std::printf("{\"variant\": \"%s\", \"blocks\": %d, \"n\": %d, \"ms\": %.4f, \"valu_wave_instr\": %.0f, "
                    "\"valu_per_simd_cycle_at_2.4GHz\": %.4f, \"cells_per_s\": %.4e}\n",
                    v == 0 ? "exact" : "nolds", blocks, n, ms, valu, valu / (1024.0 * ms * 1e-3 * 2.4e9),
                    cells / (ms * 1e-3));
    }
    CHECK(hipFree(d));
    return 0;
}
