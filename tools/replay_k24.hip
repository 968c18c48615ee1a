// Replay microbenchmark of the dominant kernel's inner column, and issue-rate probes, with the
// clock the chip holds measured inside every wave (tools/, not product code; VERDICT r04 item 3,
// r05 item 1). tools/make_replay_k24.py extracts k_align<24, true, TAGGED>'s cross-mode column loop
// from the compiler's gfx950 assembly VERBATIM (profiles/r05/k_align24_inner_column.s) into
// replay_k24_body.inc, as that loop and six edited copies:
//
//   exact      the loop as emitted
//   nolds      its ds_reads and their lgkmcnt waits dropped
//   nowait     the ds_reads kept, the waits dropped
//   sgprlit    the 49 VOP2 literals per column taken from SGPRs (196 B less code per column)
//   max3split  every v_max3_i32 as two v_max_i32
//   maxadd     every 32-bit max as full-rate v_add_u32 (max3 as two adds): same chains, no max
//   inter2     a second copy of every vector instruction on v72..v143, interleaved one by one:
//              two independent columns per lane (the row chain broken), the loop control shared
//
// Each runs with the real kernel's block shape (256 threads, the 4 x 8 x 24-int LDS table), wave
// count (blocks = tiles x adapters) and trip count (n - 1 = 149 columns of a 150-column window),
// and nothing else (no table fill, no last column, no result store). `waves` caps the waves per
// SIMD through dynamic LDS (a 256-thread block is one wave per SIMD).
//
// Clock: every wave reads s_memtime (shader cycles) and s_memrealtime (100 MHz) around its loop;
// the effective clock is sum(d memtime) / sum(d realtime) x 100 MHz, and the issue rates below are
// per SIMD per cycle AT THAT CLOCK (not the nominal 2.4 GHz).
//
// Rate probes (k_rate<OP>): 8 independent chains per lane of one instruction, 8 waves per SIMD,
// 2048 iterations -- the sustained issue rate of that instruction alone.
//
//   python tools/make_replay_k24.py && hipcc --offload-arch=gfx950 -O3 -o tools/replay_k24 tools/replay_k24.hip
//   tools/replay_k24 [reps=20]     (one JSON line per measurement)
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

// inter2: copy B's registers start as copies of A's (valid tile address, LDS base, codes)
#define RP_SETUP_INTER2                                                                                    \
    "v_mov_b32 v72, v0\n v_mov_b32 v73, v1\n v_mov_b32 v74, v2\n v_mov_b32 v75, v3\n"                    \
    "v_mov_b32 v76, v4\n v_mov_b32 v77, v5\n v_mov_b32 v78, v6\n v_mov_b32 v79, v7\n"                    \
    "v_mov_b32 v80, v8\n v_mov_b32 v81, v9\n v_mov_b32 v82, v10\n v_mov_b32 v83, v11\n"                  \
    "v_mov_b32 v84, v12\n v_mov_b32 v85, v13\n v_mov_b32 v86, v14\n v_mov_b32 v87, v15\n"                \
    "v_mov_b32 v88, v16\n v_mov_b32 v89, v17\n v_mov_b32 v90, v18\n v_mov_b32 v91, v19\n"                \
    "v_mov_b32 v92, v20\n v_mov_b32 v93, v21\n v_mov_b32 v94, v22\n v_mov_b32 v95, v23\n"                \
    "v_mov_b32 v96, v24\n v_mov_b32 v97, v25\n v_mov_b32 v98, v26\n v_mov_b32 v99, v27\n"                \
    "v_mov_b32 v100, v28\n v_mov_b32 v101, v29\n v_mov_b32 v102, v30\n v_mov_b32 v103, v31\n"            \
    "v_mov_b32 v104, v32\n v_mov_b32 v105, v33\n v_mov_b32 v106, v34\n v_mov_b32 v107, v35\n"            \
    "v_mov_b32 v108, v36\n v_mov_b32 v109, v37\n v_mov_b32 v110, v38\n v_mov_b32 v111, v39\n"            \
    "v_mov_b32 v112, v40\n v_mov_b32 v113, v41\n v_mov_b32 v114, v42\n v_mov_b32 v115, v43\n"            \
    "v_mov_b32 v116, v44\n v_mov_b32 v117, v45\n v_mov_b32 v118, v46\n v_mov_b32 v119, v47\n"            \
    "v_mov_b32 v120, v48\n v_mov_b32 v121, v49\n v_mov_b32 v122, v50\n v_mov_b32 v123, v51\n"            \
    "v_mov_b32 v124, v52\n v_mov_b32 v125, v53\n v_mov_b32 v126, v54\n v_mov_b32 v127, v55\n"            \
    "v_mov_b32 v128, v56\n v_mov_b32 v129, v57\n v_mov_b32 v130, v58\n v_mov_b32 v131, v59\n"            \
    "v_mov_b32 v132, v60\n v_mov_b32 v133, v61\n v_mov_b32 v134, v62\n v_mov_b32 v135, v63\n"            \
    "v_mov_b32 v136, v64\n v_mov_b32 v137, v65\n v_mov_b32 v138, v66\n v_mov_b32 v139, v67\n"            \
    "v_mov_b32 v140, v68\n v_mov_b32 v141, v69\n v_mov_b32 v142, v70\n v_mov_b32 v143, v71\n"

// One replay kernel per variant; PAD = ".p2align 8\n" (+ "s_nop 0\n" for the 4-byte phase).
#define RP_KERNEL(NAME, TAG, SETUP_EXTRA, PAD, ...)                                                      \
    __global__ __launch_bounds__(256) void NAME(const uint32_t *tiles, int n_tiles, int n,              \
                                                unsigned long long *clk) {                            \
        __shared__ __attribute__((aligned(16))) int32_t tab[4 * kTabInts];                            \
        for (int e = threadIdx.x; e < 4 * kTabInts; e += 256) tab[e] = (int32_t)((e * 2654435761u) >> 8); \
        __syncthreads();                                                                              \
        const int tile = (int)(blockIdx.x % (unsigned)n_tiles);                                       \
        const uint64_t qa = (uint64_t)(uintptr_t)(tiles + ((int64_t)tile * kQuads * 256 + (threadIdx.x & ~63u))); \
        const uint32_t qlo = __builtin_amdgcn_readfirstlane((uint32_t)qa);                            \
        const uint32_t qhi = __builtin_amdgcn_readfirstlane((uint32_t)(qa >> 32));                    \
        const uint32_t ldsb = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) * kTabInts * 4);      \
        unsigned long long *cp = clk + 2 * (size_t)__builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)); \
        /* the clock is read and stored inside the asm: no VGPR lives across the loop */               \
        asm volatile("s_memtime s[66:67]\n s_memrealtime s[68:69]\n"                                  \
                     RP_SETUP SETUP_EXTRA "s_branch " RP_HEADER_##TAG "\n" PAD RP_LOOP_##TAG           \
                     RP_EXIT_##TAG                                                                     \
                     "s_or_b64 exec, exec, s[2:3]\n"                                                   \
                     "s_memtime s[70:71]\n s_memrealtime s[72:73]\n s_waitcnt lgkmcnt(0)\n"           \
                     "s_sub_u32 s70, s70, s66\n s_subb_u32 s71, s71, s67\n"                            \
                     "s_sub_u32 s72, s72, s68\n s_subb_u32 s73, s73, s69\n"                            \
                     "s_mov_b64 s[74:75], exec\n s_mov_b64 exec, 1\n"                                  \
                     "v_mov_b32 v0, s70\n v_mov_b32 v1, s71\n v_mov_b32 v2, s72\n v_mov_b32 v3, s73\n" \
                     "v_mov_b32 v4, 0\n global_store_dwordx4 v4, v[0:3], %[cp]\n"                     \
                     "s_waitcnt vmcnt(0)\n s_mov_b64 exec, s[74:75]\n"                                 \
                     :                                                                                 \
                     : [qlo] "s"(qlo), [qhi] "s"(qhi), [ldsb] "s"(ldsb), [n] "s"(n), [cp] "s"(cp)      \
                     : __VA_ARGS__, "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74",     \
                       "s75", "vcc", "scc", "memory");                                                 \
    }

#define PAD0 ".p2align 8\n"
#define PAD4 ".p2align 8\n s_nop 0\n"

RP_KERNEL(k_exact, EXACT, "", PAD0, RP_CLOBBER_V, RP_CLOBBER_S)
RP_KERNEL(k_exact4, EXACT4, "", PAD4, RP_CLOBBER_V, RP_CLOBBER_S)
RP_KERNEL(k_nolds, NOLDS, "", PAD0, RP_CLOBBER_V, RP_CLOBBER_S)
RP_KERNEL(k_nolds4, NOLDS4, "", PAD4, RP_CLOBBER_V, RP_CLOBBER_S)
RP_KERNEL(k_nowait, NOWAIT, "", PAD0, RP_CLOBBER_V, RP_CLOBBER_S)
RP_KERNEL(k_sgprlit, SGPRLIT, RP_SGPRLIT_SETUP, PAD0, RP_CLOBBER_V, RP_CLOBBER_S, RP_CLOBBER_LIT)
RP_KERNEL(k_max3split, MAX3SPLIT, "", PAD0, RP_CLOBBER_V, RP_CLOBBER_S)
RP_KERNEL(k_maxadd, MAXADD, "", PAD0, RP_CLOBBER_V, RP_CLOBBER_S)
RP_KERNEL(k_inter2, INTER2, RP_SETUP_INTER2, PAD0, RP_CLOBBER_V, RP_CLOBBER_V2, RP_CLOBBER_S)
RP_KERNEL(k_nolds_mov, NOLDS_MOV, "", PAD0, RP_CLOBBER_V, RP_CLOBBER_S)
RP_KERNEL(k_vgconst, VGCONST, "v_mov_b32 v72, s16\n v_mov_b32 v73, s28\n", PAD0, RP_CLOBBER_V, "v72", "v73",
          RP_CLOBBER_S)

// ---- issue-rate probes: 8 independent chains per lane, one instruction ----
#define P8(T) T(0) T(1) T(2) T(3) T(4) T(5) T(6) T(7)
#define I_ADD(i) "v_add_u32 %" #i ", %" #i ", %8\n"
#define I_ANDLIT(i) "v_and_b32 %" #i ", 0xff01ffff, %" #i "\n"
#define I_ANDSG(i) "v_and_b32 %" #i ", %10, %" #i "\n"
#define I_MAX(i) "v_max_i32 %" #i ", %" #i ", %8\n"
#define I_MAX3(i) "v_max3_i32 %" #i ", %" #i ", %8, %9\n"
#define I_MAXU(i) "v_max_u32 %" #i ", %" #i ", %8\n"
#define I_MAXI16(i) "v_max_i16 %" #i ", %" #i ", %8\n"
#define I_PKMAX(i) "v_pk_max_i16 %" #i ", %" #i ", %8\n"
#define I_ADD3(i) "v_add3_u32 %" #i ", %" #i ", %8, %9\n"
#define I_CND(i) "v_cndmask_b32 %" #i ", %" #i ", %8, vcc\n"
#define I_MED3(i) "v_med3_i32 %" #i ", %" #i ", %8, %9\n"
#define I_SUBREV(i) "v_subrev_u32 %" #i ", %8, %" #i "\n"
#define I_MINI(i) "v_min_i32 %" #i ", %" #i ", %8\n"
#define I_MAXF(i) "v_max_f32 %" #i ", %" #i ", %8\n"
#define I_CELL(i) I_ADD(i) I_MAX(i) I_ADD(i) I_ANDLIT(i) I_MAX(i) I_ADD(i) I_MAX3(i) I_ANDLIT(i) I_ADD(i)
#define I_CMPCND(i) "v_cmp_eq_u32 vcc, %" #i ", %8\n v_cndmask_b32 %" #i ", %9, %8, vcc\n"
#define I_CND64(i) "v_cndmask_b32_e64 %" #i ", %" #i ", %8, %11\n"
#define I_BFE(i) "v_bfe_u32 %" #i ", %8, %" #i ", 4\n"
#define I_CMPS(i) "v_cmp_gt_i32 %11, %" #i ", %8\n"
#define I_XORMIN(i) "v_xor_b32 %" #i ", %" #i ", %8\n v_min_u32 %" #i ", 1, %" #i "\n"

template <int OP>
__global__ __launch_bounds__(256) void k_rate(int *out, int seed, int iters, unsigned long long *clk) {
    const unsigned long long m64 = __builtin_amdgcn_read_exec() & 0x5555555555555555ull;
    int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    int b = seed, c = ~seed;
    const int sg = __builtin_amdgcn_readfirstlane(seed * 3);
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if (OP == 8) asm volatile("v_cmp_gt_i32 vcc, %0, %1\n" ::"v"(b), "v"(c) : "vcc");
    for (int i = 0; i < iters; ++i) {
#define RATE_CASE(K, BODY) \
        if (OP == K) asm volatile(P8(BODY) P8(BODY) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), \
                                  "+v"(a6), "+v"(a7) : "v"(b), "v"(c), "s"(sg), "s"(m64) : "vcc");
        RATE_CASE(0, I_ADD)
        RATE_CASE(1, I_ANDLIT)
        RATE_CASE(2, I_ANDSG)
        RATE_CASE(3, I_MAX)
        RATE_CASE(4, I_MAX3)
        RATE_CASE(5, I_MAXU)
        RATE_CASE(6, I_MAXI16)
        RATE_CASE(7, I_PKMAX)
        RATE_CASE(8, I_CND)
        RATE_CASE(9, I_ADD3)
        RATE_CASE(10, I_MED3)
        RATE_CASE(11, I_SUBREV)
        RATE_CASE(12, I_MINI)
        RATE_CASE(13, I_MAXF)
        RATE_CASE(14, I_CELL)
        RATE_CASE(15, I_CMPCND)
        RATE_CASE(16, I_CND64)
        RATE_CASE(17, I_BFE)
        RATE_CASE(18, I_XORMIN)
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
        clk[2 * w] = t1 - t0;
        clk[2 * w + 1] = r1 - r0;
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

using ReplayFn = void (*)(const uint32_t *, int, int, unsigned long long *);
struct Variant {
    const char *name;
    ReplayFn fn;
    int valu_main, valu_load, valu_half, cols_per_pass;
};

// effective clock (GHz) from the per-wave counters of the last launch
static double eff_clock(const unsigned long long *d_clk, size_t waves) {
    std::vector<unsigned long long> h(2 * waves);
    CHECK(hipMemcpy(h.data(), d_clk, h.size() * 8, hipMemcpyDeviceToHost));
    double t = 0, r = 0;
    for (size_t w = 0; w < waves; ++w) {
        t += (double)h[2 * w];
        r += (double)h[2 * w + 1];
    }
    return r > 0 ? t / r * 0.1 : 0.0;
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
    const int blocks = 17986;   // 391 tiles x 46 adapters: the headline launch
    const int n = 150;
    const int n_tiles = 391;
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
    unsigned long long *d_clk = nullptr;
    CHECK(hipMalloc(&d, h.size() * 4));
    CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&d_clk, (size_t)blocks * 4 * 16));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double passes = n - 1, loads = (n - 1 + 3) / 4;   // columns 1 .. n-1; a look-ahead every 4th

    const Variant vs[] = {
        {"exact", k_exact, RP_VALU_MAIN_EXACT, RP_VALU_LOAD_EXACT, RP_VALU_HALF_EXACT, 1},
        {"exact4", k_exact4, RP_VALU_MAIN_EXACT4, RP_VALU_LOAD_EXACT4, RP_VALU_HALF_EXACT4, 1},
        {"nolds", k_nolds, RP_VALU_MAIN_NOLDS, RP_VALU_LOAD_NOLDS, RP_VALU_HALF_NOLDS, 1},
        {"nolds4", k_nolds4, RP_VALU_MAIN_NOLDS4, RP_VALU_LOAD_NOLDS4, RP_VALU_HALF_NOLDS4, 1},
        {"nowait", k_nowait, RP_VALU_MAIN_NOWAIT, RP_VALU_LOAD_NOWAIT, RP_VALU_HALF_NOWAIT, 1},
        {"sgprlit", k_sgprlit, RP_VALU_MAIN_SGPRLIT, RP_VALU_LOAD_SGPRLIT, RP_VALU_HALF_SGPRLIT, 1},
        {"max3split", k_max3split, RP_VALU_MAIN_MAX3SPLIT, RP_VALU_LOAD_MAX3SPLIT, RP_VALU_HALF_MAX3SPLIT, 1},
        {"maxadd", k_maxadd, RP_VALU_MAIN_MAXADD, RP_VALU_LOAD_MAXADD, RP_VALU_HALF_MAXADD, 1},
        {"inter2", k_inter2, RP_VALU_MAIN_INTER2, RP_VALU_LOAD_INTER2, RP_VALU_HALF_INTER2, 2},
        {"nolds_mov", k_nolds_mov, RP_VALU_MAIN_NOLDS_MOV, RP_VALU_LOAD_NOLDS_MOV, RP_VALU_HALF_NOLDS_MOV, 1},
        {"vgconst", k_vgconst, RP_VALU_MAIN_VGCONST, RP_VALU_LOAD_VGCONST, RP_VALU_HALF_VGCONST, 1},
    };
    // waves per SIMD: 0 = as many as the registers allow; else capped through dynamic LDS (a block
    // is one wave per SIMD, 160 KiB of LDS per CU, the static table 3 KiB)
    auto lds_for = [](int w) { return w <= 0 ? 0 : (int)(160 * 1024 / w - 4 * kTabInts * 4 - 512); };
    struct Run {
        int v, waves;
    };
    std::vector<Run> runs;
    for (int v = 0; v < (int)(sizeof(vs) / sizeof(vs[0])); ++v) runs.push_back({v, 0});
    for (int w : {3, 4, 5, 6}) runs.push_back({0, w});
    runs.push_back({10, 5});
    for (const Run &r : runs) {
        const Variant &v = vs[r.v];
        const int lds = lds_for(r.waves);
        auto launch = [&]() { hipLaunchKernelGGL(v.fn, dim3(blocks), dim3(256), lds, 0, d, n_tiles, n, d_clk); };
        for (int w = 0; w < 3; ++w) launch();
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0, 0));
        for (int k = 0; k < reps; ++k) launch();
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        const double ghz = eff_clock(d_clk, (size_t)blocks * 4);
        const double waves = 4.0 * blocks;
        const double valu = waves * (passes * v.valu_main + loads * v.valu_load);
        const double half = waves * passes * v.valu_half;
        const double cells = waves * 64.0 * passes * 24.0 * v.cols_per_pass;
        const double simd_cycles = 1024.0 * ms * 1e-3 * ghz * 1e9;
        // issue model: full-rate 2 cycles per wave64 instruction, half-rate (32-bit max, VOP3) 4
        const double model_cycles = (2.0 * (valu - half) + 4.0 * half) / 1024.0;
        std::printf("{\"kind\": \"replay\", \"variant\": \"%s\", \"waves_per_simd_cap\": %d, \"lds_bytes\": %d, "
                    "\"ms\": %.4f, \"clock_ghz\": %.4f, \"valu_wave_instr\": %.0f, \"half_rate_instr\": %.0f, "
                    "\"valu_per_simd_cycle\": %.4f, \"valu_per_simd_cycle_at_2.4GHz\": %.4f, "
                    "\"issue_model_frac\": %.4f, \"cells_per_s\": %.4e, \"k24_frac_equiv\": %.4f}\n",
                    v.name, r.waves, lds, ms, ghz, valu, half, valu / simd_cycles,
                    valu / (1024.0 * ms * 1e-3 * 2.4e9), model_cycles / (simd_cycles / 1024.0), cells / (ms * 1e-3),
                    cells * 10.0 / (ms * 1e-3) / 78.6e12);
        std::fflush(stdout);
    }

    // rate probes
    int *d_out = nullptr;
    const int rblocks = 256 * 8, iters = 1024;
    CHECK(hipMalloc(&d_out, (size_t)rblocks * 256 * 4));
    unsigned long long *d_rclk = nullptr;
    CHECK(hipMalloc(&d_rclk, (size_t)rblocks * 4 * 16));
    const char *names[] = {"v_add_u32", "v_and_b32 literal", "v_and_b32 sgpr", "v_max_i32", "v_max3_i32",
                           "v_max_u32", "v_max_i16", "v_pk_max_i16", "v_cndmask_b32", "v_add3_u32",
                           "v_med3_i32", "v_subrev_u32", "v_min_i32", "v_max_f32", "tagged cell (6 full + 3 max)",
                           "v_cmp_eq + v_cndmask (vcc) pair", "v_cndmask_b32_e64 (sgpr-pair mask)", "v_bfe_u32",
                           "v_xor + v_min_u32 pair"};
    void (*rk[])(int *, int, int, unsigned long long *) = {k_rate<0>, k_rate<1>, k_rate<2>, k_rate<3>, k_rate<4>,
                                                            k_rate<5>, k_rate<6>, k_rate<7>, k_rate<8>, k_rate<9>,
                                                            k_rate<10>, k_rate<11>, k_rate<12>, k_rate<13>,
                                                            k_rate<14>, k_rate<15>, k_rate<16>, k_rate<17>,
                                                            k_rate<18>};
    for (int op = 0; op < 19; ++op) {
        // wave-instructions per asm statement (8 chains x 2 copies x instructions per chain step)
        const int per_iter = op == 14 ? 9 * 16 : ((op == 15 || op == 18) ? 2 * 16 : 16);
        auto launch = [&]() { hipLaunchKernelGGL(rk[op], dim3(rblocks), dim3(256), 0, 0, d_out, 3, iters, d_rclk); };
        launch();
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0, 0));
        for (int k = 0; k < 3; ++k) launch();
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 3;
        const double ghz = eff_clock(d_rclk, (size_t)rblocks * 4);
        const double instrs = (double)rblocks * 4 * iters * per_iter;
        std::printf("{\"kind\": \"rate\", \"op\": \"%s\", \"waves_per_simd\": 8, \"ms\": %.4f, \"clock_ghz\": %.4f, "
                    "\"wave_instr_per_simd_cycle\": %.4f, \"cycles_per_wave_instr\": %.3f}\n",
                    names[op], ms, ghz, instrs / (1024.0 * ms * 1e-3 * ghz * 1e9),
                    (1024.0 * ms * 1e-3 * ghz * 1e9) / instrs);
        std::fflush(stdout);
    }
    CHECK(hipFree(d));
    CHECK(hipFree(d_clk));
    CHECK(hipFree(d_out));
    CHECK(hipFree(d_rclk));
    return 0;
}
