// pcabi_kern.h -- INTERNAL header of libpcabi (not the public ABI, see include/pcabi.h): the
// device-side types and kernel templates shared by the engine (pcabi_engine.hip) and the
// kernel translation units that instantiate them (pcabi_k_*.hip), split so that the heavy
// template instantiations compile in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "../../include/pcabi.h"
#include "pcabi_dp.h"

#ifndef PCABI_WAVES
#define PCABI_WAVES 1
#endif

// PCABI_POISON=1 (debug, pcabi_engine.hip): fresh device scratch is filled with 0xFF bytes, on the
// host's behalf (pcabi_poison) or stream-ordered for hipMallocAsync scratch (pcabi_poison_async)
void pcabi_poison(void *p, size_t bytes);
void pcabi_poison_async(void *p, size_t bytes, hipStream_t st);

namespace pcabi_eng {

// thread-local error message (pcabi_last_error), defined in pcabi_engine.hip
int fail(int code, const std::string &msg);

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(PCABI_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// Register buckets. FAST (branch-free core, pcabi_dp.h align_lane_fast): every multiple of 4 up
// to 64, used whenever pcabi::fast_ok holds (and served by the packed-key core when every
// adapter of the bucket is pcabi::packed_ok). WIDE (packed-key core only, wide key layout
// pk::Lay<RPL > 64>): every multiple of 4 from 68 to 88, for the 65-88 bp adapters (native
// barcoding "full sequence" adapters) whenever packed_ok holds. GENERIC (guarded core, any
// scoring): a few sizes, the path for everything else up to 128.
// LONG (two-pass packed core, pk::LayL): 96 / 112 / 128 rows for the 89-128 bp adapters (the
// 102 / 111 bp full rapid-barcode sequences) whenever pcabi::long_ok holds.
// STRIPED (pcabi_dp.h align_lane_striped, k_align_striped): every adapter longer than kMaxRPL, any
// scoring, rows in stripes of kStripeRows with the boundary row in global scratch; its table pads
// every adapter to the bucket's longest, rounded up to kStripeTab rows (pcabi_adapters::rt).
enum Kind { FAST = 0, GENERIC = 1, PACKED = 2, WIDE = 3, LONG = 4, STRIPED = 5,
            TAGGED = 6 };   // TAGGED: PACKED with the run-tagged key layout (pcabi_dp.h pk::LayT), a launch-time choice
struct BucketDef {
    int rpl;
    Kind kind;
};
constexpr BucketDef kBuckets[] = {
    {4, FAST},  {8, FAST},  {12, FAST}, {16, FAST}, {20, FAST}, {24, FAST}, {28, FAST}, {32, FAST},
    {36, FAST}, {40, FAST}, {44, FAST}, {48, FAST}, {52, FAST}, {56, FAST}, {60, FAST}, {64, FAST},
    {68, WIDE}, {72, WIDE}, {76, WIDE}, {80, WIDE}, {84, WIDE}, {88, WIDE},
    {96, LONG}, {112, LONG}, {128, LONG},
    {16, GENERIC}, {32, GENERIC}, {64, GENERIC}, {96, GENERIC}, {128, GENERIC},
    {256, STRIPED}};
constexpr int kNumBuckets = sizeof(kBuckets) / sizeof(kBuckets[0]);
constexpr int kStripedBucket = kNumBuckets - 1;
constexpr int kMaxRPL = 128;                          // longest adapter a register-resident core holds
constexpr int kStripeRows = 32;
constexpr int kStripeTab = 64;

struct KParams {
    const uint8_t *codes;      // pairs mode: windows read in place
    const int64_t *win_off;
    const int32_t *win_len;
    int64_t n_win;
    const uint32_t *tiles;     // cross mode: windows in tile layout (pcabi_tile_windows_dev)
    const int64_t *tile_off;   // [n_tiles + 1] dword offsets
    // bucket-local adapter table: RPL bytes per adapter, top padded (slot s-1 <-> byte s-1)
    const uint32_t *adp_pad;
    const int32_t *adp_len;
    const int32_t *adp_id;     // global adapter index (result row in cross mode)
    int32_t n_adp;
    // pairs mode
    const int32_t *task_win;   // [n_waves*64], -1 = idle lane
    const int32_t *task_out;   // [n_waves*64] result index
    const int32_t *wave_adp;   // [n_waves] bucket-local adapter
    int64_t n_waves;
    int32_t *out;
    int64_t out_stride;
    pcabi::Scoring sc;
    int32_t *compat;           // != nullptr: write check_compatibility flags instead of results
    int32_t chunk_split;       // k_align_chunk: lanes per chunk task (0 / 1: one; 2, 4: the row-split core)
    const int4 *task_chunk;    // k_align_chunk: per task slot (read offset, columns, owned lo, hi)
    // striped bucket (k_align_striped)
    int32_t rt;                // table rows per adapter (multiple of kStripeTab)
    int32_t max_cols;          // host value: no window / chunk of the launch is longer
    int32_t *scratch;          // boundary rows: per wave slot max_cols x fields x 64 lanes
    int64_t n_items;           // waves of work (cross: 64-window groups x adapters)
    // k_align_chunk planned on the device (the middle scan's queued rounds): dev_waves[0] = the
    // launch's first wave in the task arrays, dev_waves[1] = its wave count; the grid is n_waves
    // blocks that stride over the waves
    const int32_t *dev_waves;
};

// Window reader: one dword per lane every 4 columns (a wave-uniform branch -- j is the same in
// every lane), fetched one chunk ahead. Two layouts share it:
//   tiles (cross mode): chunk q of the lane's window at base[q * 256], so a wave's load is 256
//                       contiguous bytes (pcabi_tile_windows_dev builds the layout);
//   codes (pairs mode): the window's own bytes, base = its aligned dword, stride 1, a8 = 8 x
//                       misalignment; reads at most 12 bytes past the window end.
struct WindowReader {
    const uint32_t *q;
    int64_t stride;      // dwords between consecutive chunks
    int a8;
    uint32_t lo, hi, nx;
    __device__ __forceinline__ WindowReader() : q(nullptr), stride(0), a8(0), lo(0), hi(0), nx(0) {}   // no window
    __device__ __forceinline__ WindowReader(const uint32_t *base, int64_t stride_, int a8_)
        : q(base), stride(stride_), a8(a8_) {
        lo = q[0]; hi = q[stride]; nx = q[2 * stride];
    }
    __device__ __forceinline__ int operator()(int j) {   // called with j = 1, 2, 3, ... in order
        const int k = j - 1;
        if (k > 0 && (k & 3) == 0) { lo = hi; hi = nx; nx = q[(int64_t)(k / 4 + 2) * stride]; }
        return (int)(((((uint64_t)hi << 32) | lo) >> (8 * (k & 3) + a8)) & 0xFFu);
    }
};

template <int RPL>
struct AdapterRegs {
    uint32_t w[RPL / 4];
    __device__ __forceinline__ void load(const uint32_t *src) {
#pragma unroll
        for (int k = 0; k < RPL / 4; ++k) w[k] = __builtin_amdgcn_readfirstlane(src[k]);
    }
    __device__ __forceinline__ int operator()(int s) const {   // s: 1-based slot, compile-time
        return (int)((w[(s - 1) >> 2] >> (8 * ((s - 1) & 3))) & 0xFFu);
    }
};

__device__ __forceinline__ void store_result(int32_t *out, int64_t stride, int64_t idx,
                                             const pcabi::Result &r) {
    out[0 * stride + idx] = r.rs;
    out[1 * stride + idx] = r.re;
    out[2 * stride + idx] = r.as;
    out[3 * stride + idx] = r.ae;
    out[4 * stride + idx] = r.score;
    out[5 * stride + idx] = r.m;
    out[6 * stride + idx] = r.l1;
    out[7 * stride + idx] = r.l2;
}

__device__ __forceinline__ pcabi::Result empty_result() {
    pcabi::Result r;
    r.rs = -1; r.re = 0; r.as = -1; r.ae = 0;
    r.score = (int)0x80000000; r.m = 0; r.l1 = 0; r.l2 = 0;
    return r;
}

// Packed-core substitution table in LDS: one (RPL+2) x 8 int32 table per wave (its adapter).
constexpr int kTabW = pcabi::pk::TAB_W;

struct LdsRow {
    const int32_t *p;   // &tab[wave][c][0]: slot s at p[s - 1], 16-byte aligned
    __device__ __forceinline__ int32_t operator()(int s) const { return p[s - 1]; }
    __device__ __forceinline__ void quad(int q, int32_t *dst) const {
        const int4 v = *reinterpret_cast<const int4 *>(p + 4 * q);
        dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
    }
};

// This wave's packed-core substitution table (every lane of the block reaches the barrier).
template <int RPL, typename Y = pcabi::pk::Lay<RPL>>
__device__ __forceinline__ void fill_wave_tab(const KParams &p, int a_local, int L, int32_t *wave_tab) {
    const int off = RPL - L;
    const int lane = threadIdx.x & 63;
    for (int e = lane; e < kTabW * RPL; e += 64) {
        const int c = e / RPL, srow = e % RPL + 1;
        const uint32_t *ap = p.adp_pad + (int64_t)a_local * (RPL / 4);
        auto code = [&](int sl) { return (int)((ap[(sl - 1) / 4] >> (8 * ((sl - 1) & 3))) & 0xFFu); };
        wave_tab[e] = pcabi::pk::sub_key<RPL, decltype(code), Y>(srow, c, code, off, p.sc);
    }
    __syncthreads();
}

// The two tables of a long bucket's wave: pass 0 (c, nD) then pass 1 (m), kTabW x RPL each.
template <int RPL>
__device__ __forceinline__ void fill_wave_tab_long(const KParams &p, int a_local, int L, int32_t *wave_tab) {
    const int off = RPL - L;
    const int lane = threadIdx.x & 63;
    const uint32_t *ap = p.adp_pad + (int64_t)a_local * (RPL / 4);
    auto code = [&](int sl) { return (int)((ap[(sl - 1) / 4] >> (8 * ((sl - 1) & 3))) & 0xFFu); };
    for (int e = lane; e < kTabW * RPL; e += 64) {
        const int c = e / RPL, srow = e % RPL + 1;
        wave_tab[e] = pcabi::pk::sub_key<RPL, decltype(code), pcabi::pk::LayL<RPL, 0>>(srow, c, code, off, p.sc);
        wave_tab[kTabW * RPL + e] =
            pcabi::pk::sub_key<RPL, decltype(code), pcabi::pk::LayL<RPL, 1>>(srow, c, code, off, p.sc);
    }
    __syncthreads();
}

template <int RPL, bool AFFINE, int KIND>
__device__ __forceinline__ void run_lane(const KParams &p, int a_local, int64_t w, int64_t out_idx,
                                         int32_t *wave_tab, int64_t tile_off) {
    AdapterRegs<RPL> adp;
    if constexpr (KIND != LONG) adp.load(p.adp_pad + (int64_t)a_local * (RPL / 4));
    const int L = __builtin_amdgcn_readfirstlane(p.adp_len[a_local]);
    if constexpr (KIND == PACKED) fill_wave_tab<RPL>(p, a_local, L, wave_tab);
    if constexpr (KIND == TAGGED) fill_wave_tab<RPL, pcabi::pk::LayT<RPL>>(p, a_local, L, wave_tab);
    if constexpr (KIND == LONG) fill_wave_tab_long<RPL>(p, a_local, L, wave_tab);
    if (w < 0) return;
    const int n = p.win_len[w];
    pcabi::Result r;
    if (n <= 0) {
        r = empty_result();
    } else {
        WindowReader rd = tile_off >= 0
            ? WindowReader(p.tiles + tile_off + (threadIdx.x & 255), 256, 0)
            : [&] {
                  const uint8_t *b = p.codes + p.win_off[w];
                  const int a0 = (int)((uintptr_t)b & 3);
                  return WindowReader(reinterpret_cast<const uint32_t *>(b - a0), 1, 8 * a0);
              }();
        if constexpr (KIND == PACKED) {
            auto tabfn = [&](int rc) { return LdsRow{wave_tab + rc * RPL}; };
            r = pcabi::align_lane_packed<(RPL <= pcabi::pk::MAX_RPL ? RPL : 4), AFFINE>(rd, n, tabfn, L, p.sc);
        } else if constexpr (KIND == TAGGED) {
            static_assert(RPL <= 32 && AFFINE, "run-tagged layout: affine buckets of <= 32 rows");
            auto tabfn = [&](int rc) { return LdsRow{wave_tab + rc * RPL}; };
            r = pcabi::align_lane_packed<RPL, true, false, pcabi::pk::LayT<RPL>>(rd, n, tabfn, L, p.sc);
        } else if constexpr (KIND == LONG) {
            WindowReader rd1 = rd;   // the second pass reads the window again from its start
            auto tab0 = [&](int rc) { return LdsRow{wave_tab + rc * RPL}; };
            auto tab1 = [&](int rc) { return LdsRow{wave_tab + kTabW * RPL + rc * RPL}; };
            r = pcabi::align_lane_packed_long<RPL, AFFINE>(rd, rd1, n, tab0, tab1, L, p.sc);
        } else if constexpr (KIND == FAST) {
            r = pcabi::align_lane_fast<RPL, AFFINE>(rd, n, adp, L, p.sc);
        } else {
            r = pcabi::align_lane_generic<RPL, AFFINE>(rd, n, adp, L, p.sc);
        }
    }
    if (p.compat) {
        // pairs mode only: the window is read in place, the adapter from its padded row
        int en_match = 0;
        if (r.rs >= 0 && r.diag_en && r.l1 > 0) {
            const uint8_t *ab = reinterpret_cast<const uint8_t *>(p.adp_pad + (int64_t)a_local * (RPL / 4));
            en_match = p.codes[p.win_off[w] + r.re] == ab[RPL - L + r.ae];
        }
        p.compat[out_idx] = pcabi::compat_flag(r, n, en_match);
        return;
    }
    store_result(p.out, p.out_stride, out_idx, r);
}

// One kernel for both work shapes (uniform branch on p.task_win):
//  cross: 1-D grid of (window tile of 256, adapter) blocks in XCD-aware order; lane = window
//  pairs: grid (ceil(n_waves/4)); wave = one adapter, lanes = host-grouped tasks
template <int KIND, int RPL>
constexpr int wave_tab_ints() {
    return (KIND == PACKED || KIND == TAGGED) ? kTabW * RPL : (KIND == LONG ? 2 * kTabW * RPL : 1);
}

// Cross mode, block b of a (window tiles x adapters) grid. XCD-aware order: workgroups are dealt to
// the 8 XCDs round-robin, so block b runs on XCD b % 8. Each XCD takes every 8th tile of 256 windows
// and runs ALL adapters of a tile back to back, so a tile is fetched into one L2 once instead of once
// per adapter. (The grid is the tiles padded to a multiple of 8, times the adapters.)
template <int RPL, bool AFFINE, int KIND>
__device__ __forceinline__ void cross_block(const KParams &p, int64_t b, int32_t *wave_tab) {
    const int64_t k = b >> 3;
    const int a_local = (int)(k % p.n_adp);
    const int64_t tile = (k / p.n_adp) * 8 + (b & 7);
    const int64_t w = tile * 256 + threadIdx.x;
    const int a_glob = p.adp_id[a_local];
    const int64_t toff = w < p.n_win ? p.tile_off[tile] : 0;
    run_lane<RPL, AFFINE, KIND>(p, a_local, w < p.n_win ? w : -1, (int64_t)a_glob * p.n_win + w, wave_tab, toff);
}

template <int RPL, bool AFFINE, int KIND>
__global__ __launch_bounds__(256, PCABI_WAVES) void k_align(KParams p) {
    __shared__ __attribute__((aligned(16))) int32_t tab[4 * wave_tab_ints<KIND, RPL>()];
    int32_t *wave_tab = tab + (threadIdx.x >> 6) * wave_tab_ints<KIND, RPL>();
    if (p.task_win == nullptr) {
        cross_block<RPL, AFFINE, KIND>(p, blockIdx.x, wave_tab);
    } else {
        int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
        const bool live = wave < p.n_waves;            // dead waves still join the table barrier
        if (!live) wave = p.n_waves - 1;
        const int64_t slot = wave * 64 + (threadIdx.x & 63);
        const int a_local = __builtin_amdgcn_readfirstlane(p.wave_adp[wave]);
        const int32_t tw = live ? p.task_win[slot] : -1;
        run_lane<RPL, AFFINE, KIND>(p, a_local, tw, tw >= 0 ? p.task_out[slot] : 0, wave_tab, -1);
    }
}

// Cross mode over tiles, TWO adapters of a FAST bucket per wave (packed 16-bit lanes): block =
// (tile of 256 windows, adapter pair) in the XCD-aware order of k_align. Writes the best score of
// every (adapter, window) as int16: s16[a_glob * n_win + w].
struct FParams {
    const uint32_t *tiles;
    const int64_t *tile_off;
    const int32_t *win_len;
    int64_t n_win;
    const uint32_t *adp_pad;   // bucket table (RPL bytes per adapter)
    const int32_t *adp_len;
    const int32_t *adp_id;
    int32_t n_adp;             // adapters in the bucket (pairs = ceil(n_adp / 2))
    int16_t *s16;
    pcabi::Scoring sc;
};

struct LdsRow16 {
    const int32_t *p;
    __device__ __forceinline__ void quad(int q, pcabi::sf::v2 *dst) const {
        const int4 v = *reinterpret_cast<const int4 *>(p + 4 * q);
        dst[0] = __builtin_bit_cast(pcabi::sf::v2, v.x);
        dst[1] = __builtin_bit_cast(pcabi::sf::v2, v.y);
        dst[2] = __builtin_bit_cast(pcabi::sf::v2, v.z);
        dst[3] = __builtin_bit_cast(pcabi::sf::v2, v.w);
    }
};

template <int RPL, bool AFFINE>
__global__ __launch_bounds__(256) void k_score_filter(FParams p) {
    __shared__ __attribute__((aligned(16))) int32_t tab[4 * kTabW * RPL];
    int32_t *wave_tab = tab + (threadIdx.x >> 6) * kTabW * RPL;
    const int n_pair = (p.n_adp + 1) / 2;
    const int64_t b = blockIdx.x;
    const int64_t k = b >> 3;
    const int pr = (int)(k % n_pair);
    const int64_t tile = (k / n_pair) * 8 + (b & 7);
    const int64_t w = tile * 256 + threadIdx.x;
    const int ia = 2 * pr, ib = (2 * pr + 1 < p.n_adp) ? 2 * pr + 1 : 2 * pr;
    const int La = __builtin_amdgcn_readfirstlane(p.adp_len[ia]);
    const int Lb = __builtin_amdgcn_readfirstlane(p.adp_len[ib]);
    {
        const int lane = threadIdx.x & 63;
        const uint32_t *pa = p.adp_pad + (int64_t)ia * (RPL / 4), *pb = p.adp_pad + (int64_t)ib * (RPL / 4);
        for (int e = lane; e < kTabW * RPL; e += 64) {
            const int c = e / RPL, sl = e % RPL + 1;
            const int ca = (int)((pa[(sl - 1) / 4] >> (8 * ((sl - 1) & 3))) & 0xFFu);
            const int cb = (int)((pb[(sl - 1) / 4] >> (8 * ((sl - 1) & 3))) & 0xFFu);
            const int va = sl <= RPL - La ? 0 : (c == ca ? p.sc.ma : p.sc.mi);
            const int vb = sl <= RPL - Lb ? 0 : (c == cb ? p.sc.ma : p.sc.mi);
            const uint32_t lo = (uint16_t)(int16_t)(va - p.sc.go), hi = (uint16_t)(int16_t)(vb - p.sc.go);
            wave_tab[e] = (int32_t)(lo | (hi << 16));
        }
        __syncthreads();
    }
    if (w >= p.n_win) return;
    const int n = p.win_len[w];
    WindowReader rd(p.tiles + p.tile_off[tile] + threadIdx.x, 256, 0);
    auto tabfn = [&](int rc) { return LdsRow16{wave_tab + rc * RPL}; };
    const pcabi::sf::v2 r = pcabi::filter_lane<RPL, AFFINE>(rd, n, tabfn, p.sc);
    p.s16[(int64_t)p.adp_id[ia] * p.n_win + w] = r[0];
    if (ib != ia) p.s16[(int64_t)p.adp_id[ib] * p.n_win + w] = r[1];
}

// Pairs mode over CHUNKS of long reads (middle-scan candidates, pcabi_dp.h sf::chunk_plan): the
// packed core on (read offset, columns) of the task's read with the end cell restricted to the
// owned columns. Wave = one adapter, as k_align's pairs mode; results unmerged, one per task.
template <int RPL, bool AFFINE, int KIND>
__device__ __forceinline__ void chunk_wave(const KParams &p, int64_t wave, bool live, int32_t *wave_tab) {
    const int64_t slot = wave * 64 + (threadIdx.x & 63);
    const int a_local = __builtin_amdgcn_readfirstlane(p.wave_adp[wave]);
    const int L = __builtin_amdgcn_readfirstlane(p.adp_len[a_local]);
    if constexpr (KIND == PACKED) fill_wave_tab<RPL>(p, a_local, L, wave_tab);
    if constexpr (KIND == TAGGED) fill_wave_tab<RPL, pcabi::pk::LayT<RPL>>(p, a_local, L, wave_tab);
    if constexpr (KIND == LONG) fill_wave_tab_long<RPL>(p, a_local, L, wave_tab);
    const int32_t tw = live ? p.task_win[slot] : -1;
    if (tw < 0) return;
    const int4 ck = p.task_chunk[slot];
    const uint8_t *b = p.codes + p.win_off[tw] + ck.x;
    const int a0 = (int)((uintptr_t)b & 3);
    WindowReader rd(reinterpret_cast<const uint32_t *>(b - a0), 1, 8 * a0);
    pcabi::Result r;
    if constexpr (KIND == PACKED) {
        auto tabfn = [&](int rc) { return LdsRow{wave_tab + rc * RPL}; };
        r = pcabi::align_lane_packed<RPL, AFFINE, true>(rd, ck.y, tabfn, L, p.sc, ck.z, ck.w);
    } else if constexpr (KIND == TAGGED) {
        static_assert(RPL <= 32 && AFFINE, "run-tagged layout: affine buckets of <= 32 rows");
        auto tabfn = [&](int rc) { return LdsRow{wave_tab + rc * RPL}; };
        r = pcabi::align_lane_packed<RPL, true, true, pcabi::pk::LayT<RPL>>(rd, ck.y, tabfn, L, p.sc, ck.z, ck.w);
    } else if constexpr (KIND == LONG) {
        WindowReader rd1 = rd;
        auto tab0 = [&](int rc) { return LdsRow{wave_tab + rc * RPL}; };
        auto tab1 = [&](int rc) { return LdsRow{wave_tab + kTabW * RPL + rc * RPL}; };
        r = pcabi::align_lane_packed_long<RPL, AFFINE, true>(rd, rd1, ck.y, tab0, tab1, L, p.sc, ck.z, ck.w);
    } else {
        AdapterRegs<RPL> adp;
        adp.load(p.adp_pad + (int64_t)a_local * (RPL / 4));
        r = pcabi::align_lane_generic<RPL, AFFINE, true>(rd, ck.y, adp, L, p.sc, ck.z, ck.w);
    }
    store_result(p.out, p.out_stride, p.task_out[slot], r);
}

// W: the launch's minimum waves per SIMD (amdgpu_waves_per_eu; 1 = no bound). WPB: waves per block
// -- with 4, a block's
// waves meet at every table barrier and the block holds its CU slot until its slowest wave (the
// longest chunk of its 4 x 64 tasks) ends; with 1 (the device-planned default) every wave retires alone.
template <int RPL, bool AFFINE, int KIND, int W = 1, int WPB = 4>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(W))) void k_align_chunk(KParams p) {
    __shared__ __attribute__((aligned(16))) int32_t tab[WPB * wave_tab_ints<KIND, RPL>()];
    int32_t *wave_tab = tab + (threadIdx.x >> 6) * wave_tab_ints<KIND, RPL>();
    if (!p.dev_waves) {
        int64_t wave = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
        const bool live = wave < p.n_waves;        // dead waves still join the table barrier
        if (!live) wave = p.n_waves - 1;
        chunk_wave<RPL, AFFINE, KIND>(p, wave, live, wave_tab);
        return;
    }
    // planned on the device: the launch's waves from dev_waves, the blocks striding over them
    // (block-uniform trip count: every wave joins every table barrier); a wave rewrites only its
    // own table, after its own reads of the previous one
    const int64_t w0 = p.dev_waves[0], nw = p.dev_waves[1];
    for (int64_t wb = blockIdx.x; wb * WPB < nw; wb += gridDim.x) {
        int64_t wave = wb * WPB + (threadIdx.x >> 6);
        const bool live = wave < nw;
        if (!live) wave = nw - 1;
        chunk_wave<RPL, AFFINE, KIND>(p, w0 + wave, live, wave_tab);
    }
}

// ---- striped bucket: adapters longer than kMaxRPL (pcabi_dp.h align_lane_striped) ----------------
// The boundary row between stripes lives in global scratch, [column][field][lane] per wave slot,
// so a wave's access to one field of one column is 256 contiguous bytes.
template <bool AFFINE>
struct StripeBnd {
    static constexpr int NF = AFFINE ? 6 : 3;   // linear gaps carry no V state
    int32_t *p;                                 // this lane's column-1 field-0 entry
    __device__ __forceinline__ void load(int j, pcabi::BndCell &c) const {
        const int32_t *q = p + (int64_t)(j - 1) * (NF * 64);
        c.s = q[0];
        c.sc = q[64];
        c.sn = (uint32_t)q[128];
        if (AFFINE) {
            c.v = q[192];
            c.vc = q[256];
            c.vn = (uint32_t)q[320];
        } else {
            c.v = pcabi::NEG;
            c.vc = 0;
            c.vn = 0;
        }
    }
    __device__ __forceinline__ void store(int j, const pcabi::BndCell &c) const {
        int32_t *q = p + (int64_t)(j - 1) * (NF * 64);
        q[0] = c.s;
        q[64] = c.sc;
        q[128] = (int32_t)c.sn;
        if (AFFINE) {
            q[192] = c.v;
            q[256] = c.vc;
            q[320] = (int32_t)c.vn;
        }
    }
};

// The current stripe's R adapter codes in SGPRs (the adapter is wave-uniform).
template <int R>
struct StripeAdp {
    const uint32_t *base;   // the adapter's rt-byte table row (top-padded)
    uint32_t w[R / 4];
    __device__ __forceinline__ void load(int k) {
#pragma unroll
        for (int q = 0; q < R / 4; ++q) w[q] = __builtin_amdgcn_readfirstlane(base[k * (R / 4) + q]);
    }
    __device__ __forceinline__ int operator()(int s) const { return (int)((w[(s - 1) >> 2] >> (8 * ((s - 1) & 3))) & 0xFFu); }
};

// Persistent grid: wave slot = blockIdx * 4 + wave owns one scratch region and walks the work
// items (cross: 64 windows of a tile x one adapter; pairs: one host-built wave of tasks, chunks
// included) with a stride of the slot count. Every lane reaches the loop's end: no barriers.
template <int R, bool AFFINE>
__global__ __launch_bounds__(256) void k_align_striped(KParams p) {
    const int64_t slot = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t n_slots = (int64_t)gridDim.x * 4;
    StripeBnd<AFFINE> bnd{p.scratch + slot * (int64_t)p.max_cols * (StripeBnd<AFFINE>::NF * 64) + lane};
    for (int64_t item = slot; item < p.n_items; item += n_slots) {
        const bool cross = p.task_win == nullptr;
        int a_local;
        int64_t w, out_idx, q = 0;
        int4 ck = make_int4(0, 0, 1, -1);
        if (cross) {
            a_local = (int)(item % p.n_adp);
            q = item / p.n_adp;
            w = q * 64 + lane;
            if (w >= p.n_win) continue;
            out_idx = (int64_t)p.adp_id[a_local] * p.n_win + w;
        } else {
            a_local = p.wave_adp[item];
            const int64_t sl = item * 64 + lane;
            w = p.task_win[sl];
            if (w < 0) continue;
            out_idx = p.task_out[sl];
            if (p.task_chunk) ck = p.task_chunk[sl];
        }
        a_local = __builtin_amdgcn_readfirstlane(a_local);
        const int L = __builtin_amdgcn_readfirstlane(p.adp_len[a_local]);
        const int n = p.task_chunk ? ck.y : p.win_len[w];
        pcabi::Result r;
        if (n <= 0) {
            r = empty_result();
        } else {
            WindowReader rd = cross
                ? WindowReader(p.tiles + p.tile_off[q >> 2] + (q & 3) * 64 + lane, 256, 0)
                : [&] {
                      const uint8_t *b = p.codes + p.win_off[w] + ck.x;
                      const int a0 = (int)((uintptr_t)b & 3);
                      return WindowReader(reinterpret_cast<const uint32_t *>(b - a0), 1, 8 * a0);
                  }();
            StripeAdp<R> adp{p.adp_pad + (int64_t)a_local * (p.rt / 4)};
            r = pcabi::align_lane_striped<R, AFFINE>(rd, n, adp, L, p.rt, p.sc, bnd, ck.z, ck.w);
        }
        if (p.compat) {
            int en_match = 0;
            if (r.rs >= 0 && r.diag_en && r.l1 > 0) {
                const uint8_t *ab = reinterpret_cast<const uint8_t *>(p.adp_pad + (int64_t)a_local * (p.rt / 4));
                en_match = p.codes[p.win_off[w] + r.re] == ab[p.rt - L + r.ae];
            }
            p.compat[out_idx] = pcabi::compat_flag(r, n, en_match);
            continue;
        }
        store_result(p.out, p.out_stride, out_idx, r);
    }
}

// ---- row-split cross mode (pcabi_dp.h LaneSplit): launches too small to fill the chip ---------
// K consecutive lanes share one window, lane l holding rows l R + 1 .. (l + 1) R (R = RPL / K):
// block = (tile of 256 windows, one of its K sub-ranges of 256 / K windows, adapter), in the
// XCD-aware order of k_align (the K blocks of a tile on one XCD). The lanes run as a systolic
// pipeline: at step t lane l computes column t - l from what lane l - 1 computed at step t - 1,
// received by one DPP row shift (row_shr:1: lane i reads lane i - 1; a group of K lanes never
// straddles a row of 16); lane 0 takes row 0 instead. The last column runs in K phases. Packed and
// run-tagged layouts (the end-window buckets), affine and linear gaps.
__device__ __forceinline__ int32_t lane_from_below(int32_t v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
}

template <int RPL, int K, bool AFFINE, int KIND>
__global__ __launch_bounds__(256, PCABI_WAVES) void k_align_split(KParams p) {
    constexpr int R = RPL / K;
    static_assert(RPL % K == 0 && 16 % K == 0 && R >= 2, "split geometry");
    using Y = typename std::conditional<KIND == TAGGED, pcabi::pk::LayT<RPL>, pcabi::pk::Lay<RPL>>::type;
    __shared__ __attribute__((aligned(16))) int32_t tab[4 * kTabW * RPL];
    int32_t *wave_tab = tab + (threadIdx.x >> 6) * (kTabW * RPL);
    const int64_t b = blockIdx.x;
    const int64_t k = b >> 3;
    const int a_local = (int)(k % p.n_adp);
    const int64_t q = k / p.n_adp;
    const int64_t tile = (q / K) * 8 + (b & 7);
    const int l = (int)(threadIdx.x % K);
    const int64_t w = tile * 256 + (q % K) * (256 / K) + threadIdx.x / K;
    const int L = __builtin_amdgcn_readfirstlane(p.adp_len[a_local]);
    fill_wave_tab<RPL, Y>(p, a_local, L, wave_tab);
    const bool live = w < p.n_win;
    const int n = live ? p.win_len[w] : 0;
    int nmax = n;                                        // the wave's step count: its longest window
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) nmax = max(nmax, __shfl_xor(nmax, o));
    WindowReader rd;
    if (n > 0) rd = WindowReader(p.tiles + p.tile_off[tile] + (w & 255), 256, 0);
    pcabi::LaneSplit<R, AFFINE, Y> st;
    st.init(l, K, L, RPL, p.sc);
    int32_t sg = st.gbot, sv = st.vbot;
    const int steps = nmax - 1 + K - 1;
#pragma unroll 1
    for (int t = 1; t <= steps; ++t) {
        int32_t rg = lane_from_below(sg), rv = lane_from_below(sv);
        if (l == 0) {
            rg = st.row0_g(t);
            rv = st.neg2;
        }
        const int j = t - l;
        if (j >= 1 && j < n) {
            const int c = rd(j);
            st.inner(LdsRow{wave_tab + c * RPL + st.r0}, j, rg, rv);
            sg = st.gbot;
            sv = st.vbot;
        }
    }
    // the last column, lane by lane
    st.out = pcabi::SplitIn{};
#pragma unroll
    for (int ph = 0; ph < K; ++ph) {
        pcabi::SplitIn in;
        in.gup = lane_from_below(st.out.gup);
        in.vup = lane_from_below(st.out.vup);
        in.slt = lane_from_below(st.out.slt);
        in.vt = lane_from_below(st.out.vt);
        in.vp = lane_from_below(st.out.vp);
        in.score = lane_from_below(st.out.score);
        in.bi = lane_from_below(st.out.bi);
        in.lt = lane_from_below(st.out.lt);
        in.trail = lane_from_below(st.out.trail);
        in.prec = lane_from_below(st.out.prec);
        in.attr = (uint32_t)lane_from_below((int32_t)st.out.attr);
        if (l == ph && n > 0) {
            if (l == 0) in = st.empty_in(n);
            const int c = rd(n);
            st.last_col(LdsRow{wave_tab + c * RPL + st.r0}, n, in);
        }
    }
    if (l == K - 1 && live)
        store_result(p.out, p.out_stride, (int64_t)p.adp_id[a_local] * p.n_win + w, n > 0 ? st.result(n) : empty_result());
}

// ---- row-split chunk mode: the middle scan's candidate DP with K lanes per chunk task ----------
// The device plan's wave w (64 task slots, one adapter) runs as K sub-waves: sub-wave k takes slots
// w * 64 + k * (64 / K) .. + 64 / K, K consecutive lanes per slot (LaneSplit as k_align_split). Inner
// columns gated by the owned range; the read's last chunk (own_hi < 0) ends with the K-phase last
// column, an inner chunk runs its last column as an inner one and materializes (packed_best's CHUNK
// rules, host model: tests/native/dp_model.cpp run_split_chunk). K x the waves of k_align_chunk
// for the same chunks: the plan's ~4,096 waves per bucket leave the one-lane kernel at ~3 waves
// per SIMD.
template <int RPL, int K, bool AFFINE, int KIND>
__device__ __forceinline__ void split_chunk_wave(const KParams &p, int64_t pw, int sub, bool live, int32_t *wave_tab) {
    constexpr int R = RPL / K;
    using Y = typename std::conditional<KIND == TAGGED, pcabi::pk::LayT<RPL>, pcabi::pk::Lay<RPL>>::type;
    const int lane = threadIdx.x & 63, l = lane % K;
    const int64_t slot = pw * 64 + sub * (64 / K) + lane / K;
    const int a_local = __builtin_amdgcn_readfirstlane(p.wave_adp[pw]);
    const int L = __builtin_amdgcn_readfirstlane(p.adp_len[a_local]);
    fill_wave_tab<RPL, Y>(p, a_local, L, wave_tab);
    const int32_t tw = live ? p.task_win[slot] : -1;
    int4 ck = make_int4(0, 0, 1, 0);
    if (tw >= 0) ck = p.task_chunk[slot];
    const int n = tw >= 0 ? ck.y : 0;
    const bool at_end = ck.w < 0;
    const int hi = at_end ? n + 1 : ck.w;
    const int n_in = at_end ? n - 1 : n;
    int nmax = n_in;                                      // the sub-wave's step count
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) nmax = max(nmax, __shfl_xor(nmax, o));
    WindowReader rd;
    if (n > 0) {
        const uint8_t *b = p.codes + p.win_off[tw] + ck.x;
        const int a0 = (int)((uintptr_t)b & 3);
        rd = WindowReader(reinterpret_cast<const uint32_t *>(b - a0), 1, 8 * a0);
    }
    pcabi::LaneSplit<R, AFFINE, Y> st;
    st.init(l, K, L, RPL, p.sc);
    int32_t sg = st.gbot, sv = st.vbot;
    const int steps = nmax + K - 1;
#pragma unroll 1
    for (int t = 1; t <= steps; ++t) {
        int32_t rg = lane_from_below(sg), rv = lane_from_below(sv);
        if (l == 0) {
            rg = st.row0_g(t);
            rv = st.neg2;
        }
        const int j = t - l;
        if (j >= 1 && j <= n_in) {
            const int c = rd(j);
            st.inner(LdsRow{wave_tab + c * RPL + st.r0}, j, rg, rv, j >= ck.z && j < hi);
            sg = st.gbot;
            sv = st.vbot;
        }
    }
    // the read's last chunk: its last column, lane by lane; an inner chunk: the scout's best
    st.out = pcabi::SplitIn{};
#pragma unroll
    for (int ph = 0; ph < K; ++ph) {
        pcabi::SplitIn in;
        in.gup = lane_from_below(st.out.gup);
        in.vup = lane_from_below(st.out.vup);
        in.slt = lane_from_below(st.out.slt);
        in.vt = lane_from_below(st.out.vt);
        in.vp = lane_from_below(st.out.vp);
        in.score = lane_from_below(st.out.score);
        in.bi = lane_from_below(st.out.bi);
        in.lt = lane_from_below(st.out.lt);
        in.trail = lane_from_below(st.out.trail);
        in.prec = lane_from_below(st.out.prec);
        in.attr = (uint32_t)lane_from_below((int32_t)st.out.attr);
        if (l == ph && n > 0 && at_end) {
            if (l == 0) in = st.empty_in(n);
            const int c = rd(n);
            st.last_col(LdsRow{wave_tab + c * RPL + st.r0}, n, in);
        }
    }
    if (!at_end) st.materialize();
    if (l == K - 1 && tw >= 0)
        store_result(p.out, p.out_stride, p.task_out[slot], n > 0 ? st.result(at_end ? n : n + 1) : empty_result());
}

template <int RPL, int K, bool AFFINE, int KIND>
__global__ __launch_bounds__(256) void k_align_split_chunk(KParams p) {
    static_assert(RPL % K == 0 && 16 % K == 0 && RPL / K >= 2, "split geometry");
    __shared__ __attribute__((aligned(16))) int32_t tab[4 * kTabW * RPL];
    int32_t *wave_tab = tab + (threadIdx.x >> 6) * (kTabW * RPL);
    // planned on the device: the bucket's waves from dev_waves, K sub-waves each, the blocks
    // striding over them (block-uniform trip count: every wave joins every table barrier)
    const int64_t w0 = p.dev_waves[0], nsub = (int64_t)p.dev_waves[1] * K;
    for (int64_t wb = blockIdx.x; wb * 4 < nsub; wb += gridDim.x) {
        int64_t sw = wb * 4 + (threadIdx.x >> 6);
        const bool live = sw < nsub;
        if (!live) sw = nsub - 1;
        split_chunk_wave<RPL, K, AFFINE, KIND>(p, w0 + sw / K, (int)(sw % K), live, wave_tab);
    }
}

template <int RPL, int KIND>
void launch(const KParams &p, bool affine, dim3 grid, hipStream_t st) {
    if (affine) hipLaunchKernelGGL((k_align<RPL, true, KIND>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((k_align<RPL, false, KIND>), grid, dim3(256), 0, st, p);
}

// ---- grouped cross launches (pcabi_k_group.hip) ---------------------------------------------
// Several (window set, register bucket) units of one core family in ONE launch: a unit is the cross
// product of one region's windows (tile layout) with one register bucket of its adapter table, as a
// k_align launch would run it; the launch's blocks are the units' grids back to back (each a
// multiple of 8 blocks, so block b of a unit keeps k_align's XCD order), longest rows first. A
// bucket of one or two adapters is a grid of ~400 blocks (1.5 waves per SIMD for 100k windows):
// alone it is latency-bound; grouped, its waves share the SIMDs with the other units'.
//   class 0: the run-tagged core (affine, 4..32 rows)    class 1: the packed core (affine, 36..64 rows)
constexpr int kMaxGroupSegs = 16;
constexpr int kGroupClasses = 2;
struct GroupSeg {
    const uint32_t *tiles;
    const int64_t *tile_off;
    const int32_t *win_len;
    int64_t n_win;
    const uint32_t *adp_pad;
    const int32_t *adp_len;
    const int32_t *adp_id;
    int32_t *out;
    int64_t out_stride;
    int64_t block0;            // the unit's first block in the launch
    int32_t n_adp;
    int32_t rpl;
};
struct GroupParams {
    GroupSeg seg[kMaxGroupSegs];
    int32_t n_seg;
    pcabi::Scoring sc;
};
constexpr int group_max_rpl(int cls) { return cls == 0 ? 32 : 64; }
// the class a cross-mode unit belongs to, -1: launched on its own (bucket_pack_mode: 1 packed, 2 tagged)
inline int group_class(int rpl, int pack_mode, bool affine) {
    if (!affine) return -1;
    if (pack_mode == 2 && rpl <= 32) return 0;
    if (pack_mode == 1 && rpl >= 36 && rpl <= 64) return 1;
    return -1;
}
void dispatch_group(int cls, const GroupParams &p, int64_t blocks, hipStream_t st);

// ---- grouped candidate-DP launches (pcabi_k_chunk.hip) ----------------------------------------
// The run-tagged chunk buckets (<= 28 rows: the 32-row case alone sets 101 VGPRs, 4 waves per SIMD;
// up to 28 the group holds 5) of one device plan in ONE launch: one-wave blocks
// stride over the buckets' device-planned waves back to back (each bucket's (first wave, waves) on
// the device), the bucket found by a scalar walk, its core by a wave-uniform switch -- so the
// buckets' waves share the SIMDs instead of running as separate launches (side by side in round 1,
// one after the other in the serial later rounds). The common task arrays stay in `p`.
constexpr int kMaxChunkSegs = 8;
constexpr int kChunkGroupRpl = 28;
struct ChunkSeg {
    const uint32_t *adp_pad;
    const int32_t *adp_len;
    const int32_t *adp_id;
    const int32_t *dev_waves;  // the bucket's (first wave, waves) from the device plan
    int32_t n_adp;
    int32_t rpl;
};
struct ChunkGroupParams {
    KParams p;
    ChunkSeg seg[kMaxChunkSegs];
    int32_t n_seg;
};
void dispatch_chunk_group(const ChunkGroupParams &gp, unsigned blocks, hipStream_t st);

// ---- kernel translation units (pcabi_k_*.hip) ----------------------------------------------
// k_align launches by core, grid as k_align expects (cross: XCD-ordered tiles x adapters;
// pairs: ceil(waves / 4) blocks).
// PACKED <= 32 rows; tagged (affine only): the run-tagged layout, every adapter passing layt_ok
void dispatch_packed_small(int rpl, const KParams &p, bool affine, dim3 grid, hipStream_t st, bool tagged);
void dispatch_packed_large(int rpl, bool long_kind, const KParams &p, bool affine, dim3 grid,
                           hipStream_t st);                                                   // PACKED 36..88, LONG
void dispatch_fast(int rpl, bool generic, const KParams &p, bool affine, dim3 grid, hipStream_t st);
// k_align_chunk launches (middle-scan candidates in owned-column chunks), striped bucket included;
// tagged: the bucket runs the run-tagged layout (bucket_pack_mode 2)
int dispatch_chunk(int b, const KParams &p, bool affine, hipStream_t st, bool tagged = false);
// k_score_filter launches
void dispatch_filter(int rpl, const FParams &p, bool affine, hipStream_t st);
// k_align_split launches (cross mode; grid = padded tiles x adapters x K); false: no such kernel
bool dispatch_split(int rpl, int K, const KParams &p, bool affine, bool tagged, hipStream_t st);
// k_align_split_chunk launches (device-planned chunk tasks, K lanes each); false: no such kernel
bool dispatch_split_chunk(int rpl, int K, const KParams &p, bool affine, bool tagged, hipStream_t st);
// the striped bucket (k_align_striped): p.rt, p.max_cols set by the caller
int launch_striped(KParams p, bool affine, hipStream_t st);

}  // namespace pcabi_eng
