// pcabi_seed.hip -- exact seeding of the middle-adapter scan on the GPU (gfx950).
//
// Reference: porechop_abi/nanopore_read.py:219-252 (find_middle_adapters): every read against
// every middle adapter, a hit when the best alignment's full identity (pid2 = m / l2) reaches
// the threshold. The engine's score filter computes every pair's best score S* to find the
// pairs that can hit. This unit finds them from exact k-mer seeds instead and
// hands the engine the pairs whose bound reaches the filter threshold T.
//
// Why it is exact ("Seeds"):
//   * l2 counts the columns of the adapter span: every adapter base once (matched, mismatched,
//     against a gap, or hanging off a read end) plus the read bases inserted inside the span.
//     So e = l2 - m non-matching columns, and pid2 >= theta gives e <= L (1 - theta) / theta.
//   * Cut the adapter into e + 1 pieces. An error column touches at most one piece, so one
//     piece aligns as an unbroken run of matches: the read holds that piece exactly. Each piece
//     contributes its first K bases (K = min(8, piece length)) as a probe.
//   * A probe found at read position q for adapter offset o fixes the diagonal d0 = q - o of
//     that run, and the alignment never leaves the band d0 +- e (at most e gap columns shift
//     it). The score-only DP restricted to that band (free end gaps as the full DP: row 0,
//     column 0 and the read's last column) scores that alignment among others, so the band's
//     best S_b >= its score >= T (sf::filter_threshold). A wider band only raises S_b.
//   * Pairs with no probe hit get no bound (no alignment can reach theta); the others the
//     largest S_b. Pairs with a bound >= T go to the full attribute DP exactly as after the
//     filter. The engine re-seeds every later round on the masked reads (N never matches).
// Kernels (integer work, no MFMA):
//   k_seed_scan   reads grid-stride over blocks, 8 positions per lane: the 8-mer codes of the
//                 positions, and per probe length K (4..8) a bitmap test and a rank into the probe
//                 entries, all in LDS; hits become (read, adapter, diagonal) tasks per band class,
//                 staged per block in LDS and appended with one global atomic per chunk;
//   k_seed_band   one lane per task: the banded Gotoh score DP (2E+1 cells per adapter row in
//                 registers), atomicMax into the pair's bound;
//   k_cands       the pairs whose bound reaches T, compacted for the host (k_bound16: or all
//                 bounds as int16).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/pcabi.h"
#include "pcabi_dp.h"

namespace pcabi_internal {
int fail(int code, const std::string &msg);
}
using pcabi_internal::fail;

#define SD_TRY(expr)                                                                                          \
    do {                                                                                                      \
        hipError_t e_ = (expr);                                                                               \
        if (e_ != hipSuccess) return fail(PCABI_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

namespace pcabi_seed {

std::atomic<int64_t> g_runs{0};

constexpr int kMinK = 4, kMaxK = 8, kNK = kMaxK - kMinK + 1;
constexpr int kCls = 2;            // band classes: e <= E0, e <= E1
constexpr int kMaxE = 15;          // band half-width the kernels are built for
constexpr int kMaxL = 255;
constexpr int kMaxEnt = 8192;      // probe entries / distinct probes kept in LDS
#ifndef PCABI_SEED_BUF
#define PCABI_SEED_BUF 256
#endif

#ifndef PCABI_BAND_EXIT
#define PCABI_BAND_EXIT 1   // rows between the banded DP's early-exit checks (1: every row, r02 A/B)
#endif
constexpr int kBuf = PCABI_SEED_BUF;   // staged tasks per block and class
constexpr int kLdsMax = 64 * 1024; // per block: probe tables + stage
constexpr int kNeg = -(1 << 20);
constexpr int kPos = 8;            // read positions per lane and scan step (16 bases loaded)
constexpr int kNW = 4;             // dwords of bases per lane and step
#ifndef PCABI_SEED_SUB
#define PCABI_SEED_SUB 2
#endif
constexpr int kSub = PCABI_SEED_SUB;   // sub-steps per scan iteration
#ifndef PCABI_SEED_FLUSH
#define PCABI_SEED_FLUSH (8 / PCABI_SEED_SUB - 1)   // stage flush every 8 sub-steps
#endif

struct ScanArgs {
    const uint8_t *codes;
    const int64_t *v_off;
    const int32_t *v_len;
    int64_t n;
    const uint32_t *tabs;       // LDS image: bits | rank16 | estart16 | ent (dwords, copied as is)
    int32_t tab_dw;             // its dwords
    int32_t bits_off[kNK];      // dword offset of K's bitmap in the image, -1 when no probe has length K;
                                // K = 8 is the merged table: every 8-mer extending a probe of any K
    int32_t min_k;              // shortest probe
    int32_t rank_off, estart_off, ent_off;   // dword offsets of the other sections
                                             // (entries: adapter << 9 | band class << 8 | offset)
    int4 *task;                 // kCls regions of cap tasks: (read, adapter, diagonal, 0)
    int64_t cap;
    int32_t *cnt;               // tasks per class (may exceed cap: the caller grows and reruns)
};

struct Stage {
    int4 buf[kCls][kBuf];
    int cnt[kCls];
    int base[kCls];
};

__device__ __forceinline__ void stage_task(Stage &sg, int cls, int4 t, const ScanArgs &a) {
    const int slot = atomicAdd(&sg.cnt[cls], 1);
    if (slot < kBuf) {
        sg.buf[cls][slot] = t;
    } else {                                           // burst past the stage: straight out
        const int g = atomicAdd(&a.cnt[cls], 1);
        if (g < a.cap) a.task[cls * a.cap + g] = t;
    }
}

// Block-uniform: writes out the classes whose stage holds at least `at_least` tasks.
__device__ __forceinline__ void flush(Stage &sg, int at_least, const ScanArgs &a) {
    __syncthreads();
    bool any = false;
#pragma unroll
    for (int c = 0; c < kCls; ++c) any |= sg.cnt[c] >= at_least && sg.cnt[c] > 0;
    if (!any) return;                                  // uniform: every thread read the same counts
    if (threadIdx.x < kCls) {
        const int c = threadIdx.x;
        const int m = min(sg.cnt[c], kBuf);
        sg.base[c] = (sg.cnt[c] >= at_least && m > 0) ? atomicAdd(&a.cnt[c], m) : -1;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < kCls; ++c) {
        if (sg.base[c] < 0) continue;
        const int m = min(sg.cnt[c], kBuf);
        for (int i = threadIdx.x; i < m; i += 256) {
            const int64_t g = (int64_t)sg.base[c] + i;
            if (g < a.cap) a.task[c * a.cap + g] = sg.buf[c][i];
        }
    }
    __syncthreads();
    if (threadIdx.x < kCls && sg.base[threadIdx.x] >= 0) sg.cnt[threadIdx.x] = 0;
    __syncthreads();
}

__global__ __launch_bounds__(256) void k_seed_scan(ScanArgs a) {
    extern __shared__ uint32_t lds[];
    __shared__ Stage sg;
    for (int i = threadIdx.x; i < a.tab_dw; i += 256) lds[i] = a.tabs[i];
    if (threadIdx.x < kCls) sg.cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint16_t *rank = reinterpret_cast<const uint16_t *>(lds + a.rank_off);
    const uint16_t *estart = reinterpret_cast<const uint16_t *>(lds + a.estart_off);
    const int32_t *ent = reinterpret_cast<const int32_t *>(lds + a.ent_off);
    // The block walks its reads (blockIdx.x, + gridDim.x, ...) 2048 positions at a time; the
    // bytes of the next step (and the next read's length / offset) are loaded before the current
    // step is processed, so the global latency hides behind the lookups.
    int64_t k = blockIdx.x, nk = k;
    int len = 0, nlen = 0;
    const uint8_t *base = a.codes, *nbase = a.codes;
    auto next_read = [&](int64_t from, int &ln, const uint8_t *&bs) -> int64_t {
        for (; from < a.n; from += gridDim.x) {
            ln = a.v_len[from];
            if (ln > 0) {
                bs = a.codes + a.v_off[from];
                return from;
            }
        }
        return from;
    };
    auto fetch = [&](const uint8_t *bs, int ln, int p0b, uint32_t (&w)[kNW]) {
        const int p0 = p0b + kPos * (int)threadIdx.x;
#pragma unroll
        for (int d = 0; d < kNW; ++d) w[d] = 0x04040404u;
        if (p0 < ln) {   // bytes p0 .. p0 + 15 from five aligned dwords; past the read they stay
                         // inside the caller's >= 16 B tail padding (dword-aligned loads)
            const uint8_t *ad = bs + p0;
            const int a0 = (int)((uintptr_t)ad & 3);
            const uint32_t *q = reinterpret_cast<const uint32_t *>(ad - a0);
            uint32_t d[kNW + 1];
#pragma unroll
            for (int t = 0; t <= kNW; ++t) d[t] = q[t];
#pragma unroll
            for (int t = 0; t < kNW; ++t) w[t] = __builtin_amdgcn_alignbyte(d[t + 1], d[t], a0);
        }
    };
    k = next_read(k, len, base);
    if (k < a.n) nk = next_read(k + gridDim.x, nlen, nbase);
    int p0b = 0;
    // kSub sub-steps of 2048 positions per iteration, fetched together one iteration ahead:
    // more bytes in flight per latency
    uint32_t wn[kSub][kNW];
#pragma unroll
    for (int h = 0; h < kSub; ++h)
        if (k < a.n) fetch(base, len, h * 256 * kPos, wn[h]);
    int iter = 0;
    while (k < a.n) {                                  // block-uniform: every lane takes part
        const int64_t ck = k;
        const int clen = len, cp0b = p0b;
        uint32_t wc[kSub][kNW];
#pragma unroll
        for (int h = 0; h < kSub; ++h)
#pragma unroll
            for (int d = 0; d < kNW; ++d) wc[h][d] = wn[h][d];
        p0b += kSub * 256 * kPos;
        if (p0b >= len) {                              // on to the next read
            k = nk;
            len = nlen;
            base = nbase;
            p0b = 0;
            if (k < a.n) nk = next_read(k + gridDim.x, nlen, nbase);
        }
#pragma unroll
        for (int h = 0; h < kSub; ++h)
            if (k < a.n) fetch(base, len, p0b + h * 256 * kPos, wn[h]);
#pragma unroll
        for (int h = 0; h < kSub; ++h) {
        const int cp0 = cp0b + h * 256 * kPos + kPos * (int)threadIdx.x;
        const uint32_t *w = wc[h];
        // 16 bases (SWAR): c32 = their 2-bit codes, first base in the top bits; vmask bit t =
        // base t is A/C/G/T inside the read (Dna5 codes are 0..4: N has bit 2)
        uint32_t c32 = 0, vmask = 0;
#pragma unroll
        for (int d = 0; d < kNW; ++d) {
            const uint32_t c4 = ((w[d] & 0x03030303u) * 0x40100401u) >> 24;
            const uint32_t nb = (((~w[d]) >> 2) & 0x01010101u) * 0x10204080u >> 28;
            c32 = (c32 << 8) | c4;
            vmask |= nb << (4 * d);
        }
        const int rem = clen - cp0;
        vmask &= rem >= 16 ? 0xFFFFu : (rem > 0 ? (1u << rem) - 1u : 0u);
        // fast path: every probe is a prefix of the 8-mer at its position, and the K = 8 table
        // holds every 8-mer that extends a probe -- one LDS word per position
        uint32_t hits = 0, slow = 0;
        if (__all((vmask & 0x7FFFu) == 0x7FFFu)) {
            // every lane's 8 positions see 8 valid bases: one bitmap word each, the K = 8 bitmap
            // at LDS byte 0 (plan()), byte address (c8 >> 5) << 2 straight from c32
#pragma unroll
            for (int i = 0; i < kPos; ++i) {
                const int sh = 16 - 2 * i;
                const uint32_t word = *reinterpret_cast<const uint32_t *>(
                    reinterpret_cast<const char *>(lds) + ((c32 >> (sh + 3)) & 0x1FFCu));
                hits |= ((word >> ((c32 >> sh) & 31u)) & 1u) << i;
            }
        } else {
#pragma unroll
        for (int i = 0; i < kPos; ++i) {
            const uint32_t c8 = (c32 >> (16 - 2 * i)) & 0xFFFFu;
            const uint32_t word = lds[a.bits_off[kNK - 1] + (int)(c8 >> 5)];
            const bool full = ((vmask >> i) & 0xFFu) == 0xFFu;
            hits |= (full && ((word >> (c8 & 31)) & 1u)) ? 1u << i : 0u;
            // a valid run shorter than 8 bases (an N or the read end ahead): the short tables
            slow |= (!full && ((vmask >> i) & ((1u << a.min_k) - 1u)) == (1u << a.min_k) - 1u) ? 1u << i : 0u;
        }
        }
        while (hits | slow) {
            const bool fast = hits != 0;
            const int i = __builtin_ctz(fast ? hits : slow);
            if (fast) hits &= hits - 1;
            else slow &= slow - 1;
            const uint32_t c8 = (c32 >> (16 - 2 * i)) & 0xFFFFu;
            const int q = cp0 + i;
            const int run = __builtin_ctz(~(vmask >> i));
            for (int kk = fast ? kNK - 1 : 0; kk < (fast ? kNK : kNK - 1); ++kk) {
                const int K = kMinK + kk;
                if (a.bits_off[kk] < 0 || (!fast && K > run)) continue;
                const uint32_t code = c8 >> (2 * (kMaxK - K));
                const int dw = a.bits_off[kk] + (int)(code >> 5);
                const uint32_t word = lds[dw], bit = 1u << (code & 31);
                if (!(word & bit)) continue;
                const int r = rank[dw] + __popc(word & (bit - 1));
                const int e = estart[r + 1];
                for (int b = estart[r]; b < e; ++b) {
                    const int en = ent[b];                 // adapter << 9 | class << 8 | offset
                    stage_task(sg, (en >> 8) & 1, make_int4((int)ck, en >> 9, q - (en & 255), 0), a);
                }
            }
        }
        }
        if ((++iter & PCABI_SEED_FLUSH) == 0) flush(sg, kBuf / 2, a);
    }
    flush(sg, 1, a);
}

// Banded score DP of one task: rows i = 1..L of the adapter, per row the 2E+1 cells of the
// diagonals d0 - E .. d0 + E (cell x <-> read column j = i + d0 + x - E), free end gaps as the
// full DP: S(0, j) = 0, S(i, 0) = 0, ends in row L (j < len) or in the last column (j = len).
// CHECK: the band touches column 0 or the last column, or leaves the read.
// Early exit (inside bands, T > 0): no path gains more than `match` per remaining row (gaps cost),
// and an inside band holds no column-0 restart and no last-column end, so once every cell of row
// i satisfies S + match (L - i) < T the pair cannot reach T: the DP stops and returns that bound
// (below T, which is all the caller compares). Random probe hits -- most tasks -- stop early.
template <int E, bool CHECK>
__device__ __forceinline__ int band_best(const uint8_t *rd, int len, const uint8_t *ac, int L, int d0,
                                         const pcabi::Scoring &sc, int T) {
    constexpr int W = 2 * E + 1;
    int S[W], V[W], R[W];
#pragma unroll
    for (int x = 0; x < W; ++x) {
        const int j0 = d0 + x - E;                           // row 0
        S[x] = (!CHECK || (j0 >= 0 && j0 <= len)) ? 0 : kNeg;
        V[x] = kNeg;
        const int j1 = j0 + 1;                               // row 1's read column
        R[x] = (!CHECK || (j1 >= 1 && j1 <= len)) ? rd[j1 - 1] : 7;
    }
    int best = 0;                                            // S(L, 0) = 0 is always scouted
    for (int i = 1; i <= L; ++i) {
        const int ab = ac[i - 1];
        int h = kNeg, sl = kNeg;                             // H, S of the cell to the left
#pragma unroll
        for (int x = 0; x < W; ++x) {
            const int dg = S[x] + ((R[x] == ab) ? sc.ma : sc.mi);
            const int vu = (x + 1 < W) ? max(V[x + 1] + sc.ge, S[x + 1] + sc.go) : kNeg;
            h = max(h + sc.ge, sl + sc.go);
            int s = max(dg, max(vu, h)), v = vu;
            if (CHECK) {
                const int j = i + d0 + x - E;
                if (j == 0) { s = 0; v = kNeg; h = kNeg; }              // the adapter head hangs off
                else if (j < 0 || j > len) { s = kNeg; v = kNeg; h = kNeg; }
                if (j == len) best = max(best, s);                      // last column
            }
            S[x] = s;
            V[x] = v;
            sl = s;
        }
#pragma unroll
        for (int x = 0; x + 1 < W; ++x) R[x] = R[x + 1];
        const int jn = i + 1 + d0 + E;
        R[W - 1] = (!CHECK || (jn >= 1 && jn <= len)) ? rd[jn - 1] : 7;
        if (!CHECK && (i % PCABI_BAND_EXIT) == 0) {
            int mx = S[0];
#pragma unroll
            for (int x = 1; x < W; ++x) mx = max(mx, S[x]);
            const int ub = mx + pcabi::best_sub(sc) * (L - i);
            if (ub < T) return ub;
        }
    }
#pragma unroll
    for (int x = 0; x < W; ++x) {                            // last row, j < len
        const int j = L + d0 + x - E;
        if (!CHECK || (j >= 0 && j < len)) best = max(best, S[x]);
    }
    return best;
}

template <int E>
__global__ __launch_bounds__(256) void k_seed_band(const int4 *task, int32_t n_task, const uint8_t *codes,
                                                   const int64_t *v_off, const int32_t *v_len, const uint8_t *adp,
                                                   const int32_t *adp_off, const int32_t *adp_len, pcabi::Scoring sc,
                                                   const int32_t *thr, int32_t *bound, int64_t n) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n_task) return;
    const int4 tk = task[t];
    const int L = adp_len[tk.y];
    const int len = v_len[tk.x];
    const int d0 = tk.z;
    const uint8_t *rd = codes + v_off[tk.x];
    const uint8_t *ac = adp + adp_off[tk.y];
    const bool inside = d0 - E >= 1 && d0 + E + L + 1 < len;
    const int T = thr[tk.y];
    const int best = inside ? band_best<E, false>(rd, len, ac, L, d0, sc, T)
                            : band_best<E, true>(rd, len, ac, L, d0, sc, T);
    atomicMax(&bound[(int64_t)tk.y * n + tk.x], best);
}

// The pairs whose bound reaches their adapter's threshold T[a], as (a << 32 | read) keys
// (unordered; one atomic per wave).
__global__ __launch_bounds__(256) void k_cands(const int32_t *bound, int64_t n, int64_t total, const int32_t *T,
                                               int64_t *out, int64_t cap, unsigned long long *cnt) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t a = i / (n > 0 ? n : 1);
    const bool want = i < total && bound[i] >= T[a];
    const uint64_t m = __ballot(want);
    if (!m) return;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)m) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(cnt, (unsigned long long)__popcll(m));
    base = __shfl(base, leader);
    if (want) {
        const unsigned long long slot = base + __popcll(m & ((1ull << lane) - 1));
        if ((int64_t)slot < cap) out[slot] = (a << 32) | (i - a * n);
    }
}

__global__ __launch_bounds__(256) void k_bound16(const int32_t *bound, int64_t cnt, int16_t *s16) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < cnt) s16[i] = (int16_t)max(min(bound[i], 32767), -32768);
}

struct Buf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes, 1 << 16);
        if (hipMalloc(&p, want) != hipSuccess) return fail(PCABI_E_NOMEM, "hipMalloc failed (seeds)");
        cap = want;
        return 0;
    }
    ~Buf() {
        if (p) (void)hipFree(p);
    }
};

struct State {
    // the second band class runs beside the first on a side stream (fork / join by events)
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    ~State() {
        if (side) (void)hipStreamDestroy(side);
        if (fork) (void)hipEventDestroy(fork);
        if (join) (void)hipEventDestroy(join);
    }
    // plan cache key: the adapters themselves (a table at a reused address may hold others)
    std::vector<uint8_t> key_codes;
    std::vector<int32_t> key_len, key_rows;
    double threshold = -1.0;
    pcabi::Scoring sc{0, 0, 0, 0};
    bool planned = false, ok = false;
    double cost_seed = 0.0, cost_filter = 0.0;    // per read position (model units)
    int band[kCls] = {0, 0};                      // E of each class
    size_t lds_bytes = 0;
    ScanArgs a{};
    Buf tabs, adp, adp_off, adp_len, task, cnt, bound, thr, cands, ccnt;
    int64_t cap = 0, ccap = 0;
    int scan_blocks = 0;                          // resident k_seed_scan blocks (per plan)
};

State *create() { return new State(); }
void destroy(State *s) { delete s; }

namespace {
// Cost model per read position (VALU slots / issue rate, tools/valu_microbench.hip): the packed
// filter spends 4 packed ops per cell (rate 0.23), a band cell ~11 ops (~0.3), the scan ~60
// (~0.4) per position, and a random position hits a K-probe with probability 1 / 4^K.
constexpr double kFilterCell = 4.0 / 0.23, kBandCell = 11.0 / 0.3, kScanPos = 60.0 / 0.4;

int plan(State *s, const uint8_t *hcodes, const int32_t *hoff, const int32_t *hlen, int32_t n_adp,
         const std::vector<int> &fb_rows, const pcabi::Scoring &sc, double threshold) {
    s->planned = true;
    s->ok = false;
    if (!(threshold > 0.0) || sc.go >= 0 || sc.ge >= 0 || n_adp >= (1 << 22)) return 0;
    // band_best's early exit bounds the rows still to come by best_sub per row: sound only when no
    // row step can gain more (every gap step costs, checked above, and best_sub > 0 > go, ge)
    if (pcabi::best_sub(sc) <= 0) return 0;
    const double th = (threshold - 1e-5) / 100.0;
    if (th <= 0.0 || th > 1.0) return 0;
    std::vector<std::vector<std::vector<int32_t>>> lists(kNK);
    std::vector<int32_t> es((size_t)n_adp, -1);
    std::vector<int32_t> thr((size_t)n_adp, INT32_MAX);   // not under the filter: the caller adds them
    double filt = 0.0, seed = kScanPos;
    int e_lo = kMaxE + 1, e_hi = -1;
    for (int32_t a = 0; a < n_adp; ++a) {
        if (fb_rows[a] <= 0) continue;                 // not under the filter: always a candidate
        const int L = hlen[a];
        if (L <= 0 || L > kMaxL) return 0;
        for (int i = 0; i < L; ++i)
            if (hcodes[hoff[a] + i] > 3) return 0;
        const int T = pcabi::sf::filter_threshold(L, threshold, sc);
        if (T <= pcabi::sf::NEG16 || T <= 0) return 0;   // no usable bound: the filter / cross product
        const int e = (int)std::floor((double)L * (1.0 - th) / th + 1e-9);
        if (e > kMaxE) return 0;
        const int plen = L / (e + 1);
        const int K = std::min(kMaxK, plen);
        if (K < kMinK) return 0;
        es[a] = e;
        thr[a] = T;
        e_lo = std::min(e_lo, e);
        e_hi = std::max(e_hi, e);
        filt += kFilterCell * fb_rows[a];
        auto &lk = lists[K - kMinK];
        if (lk.empty()) lk.resize((size_t)1 << (2 * K));
        for (int p = 0; p <= e; ++p) {
            const int o = p * plen;
            uint32_t code = 0;
            for (int t = 0; t < K; ++t) code = (code << 2) | hcodes[hoff[a] + o + t];
            lk[code].push_back((a << 9) | o);   // the class bit (8) is set below
        }
    }
    if (e_hi < 0) return 0;
    // the merged K = 8 table: an 8-mer lists the entries of every probe it extends
    {
        std::vector<std::vector<int32_t>> merged((size_t)1 << 16);
        for (int kk = 0; kk < kNK; ++kk) {
            if (lists[kk].empty()) continue;
            const int sh = 2 * (kMaxK - (kMinK + kk));
            for (uint32_t c = 0; c < (1u << 16); ++c)
                for (int32_t x : lists[kk][c >> sh]) merged[c].push_back(x);
        }
        s->a.min_k = kMaxK;
        for (int kk = 0; kk < kNK - 1; ++kk)
            if (!lists[kk].empty()) s->a.min_k = std::min(s->a.min_k, kMinK + kk);
        lists[kNK - 1].swap(merged);
    }
    s->band[0] = std::max(1, e_lo);
    s->band[1] = std::max(s->band[0], e_hi);
    std::vector<int32_t> cls((size_t)n_adp, 0);
    for (int32_t a = 0; a < n_adp; ++a) cls[a] = es[a] > s->band[0] ? 1 : 0;
    // LDS image: bitmaps of the present K, per-dword rank (probes before the dword), the probe
    // entry ranges, the entries
    std::vector<uint32_t> bits;
    std::vector<uint16_t> estart;
    std::vector<int32_t> ent;
    ScanArgs &A = s->a;
    for (int kk = 0; kk < kNK; ++kk) A.bits_off[kk] = -1;
    // the merged K = 8 bitmap first: the scan's fast path addresses it from LDS byte 0
    for (int pass = 0; pass < kNK; ++pass) {
        const int kk = pass == 0 ? kNK - 1 : pass - 1;
        if (lists[kk].empty()) continue;
        const size_t nc = lists[kk].size();
        const int K = kMinK + kk;
        A.bits_off[kk] = (int32_t)bits.size();
        bits.resize(bits.size() + std::max<size_t>(nc / 32, 1), 0u);
        for (size_t c = 0; c < nc; ++c) {
            if (lists[kk][c].empty()) continue;
            bits[A.bits_off[kk] + c / 32] |= 1u << (c % 32);
            estart.push_back((uint16_t)ent.size());
            for (int32_t x : lists[kk][c]) {
                const int a = x >> 9;
                ent.push_back(x | (cls[a] << 8));
                if (kk == kNK - 1)                     // the merged table: each random hit costs a band
                    seed += kBandCell * (double)hlen[a] * (2.0 * s->band[cls[a]] + 1.0) / (double)((size_t)1 << (2 * K));
            }
            if (ent.size() >= (size_t)kMaxEnt) return 0;
        }
    }
    if (ent.empty()) return 0;
    estart.push_back((uint16_t)ent.size());
    std::vector<uint16_t> rank(bits.size());
    uint32_t run = 0;
    for (size_t d = 0; d < bits.size(); ++d) {
        rank[d] = (uint16_t)run;
        run += (uint32_t)__builtin_popcount(bits[d]);
    }
    std::vector<uint32_t> img(bits);
    auto append16 = [&](const std::vector<uint16_t> &v) {
        const int32_t off = (int32_t)img.size();
        img.resize(img.size() + (v.size() + 1) / 2, 0u);
        std::copy(v.begin(), v.end(), reinterpret_cast<uint16_t *>(img.data() + off));
        return off;
    };
    A.rank_off = append16(rank);
    A.estart_off = append16(estart);
    A.ent_off = (int32_t)img.size();
    for (int32_t x : ent) img.push_back((uint32_t)x);
    A.tab_dw = (int32_t)img.size();
    s->lds_bytes = 4 * img.size();
    if (s->lds_bytes + sizeof(Stage) > (size_t)kLdsMax) return 0;
    s->cost_seed = seed;
    s->cost_filter = filt;
    std::vector<int32_t> aoff((size_t)n_adp), alen((size_t)n_adp);
    int32_t tot = 0;
    for (int32_t a = 0; a < n_adp; ++a) {
        aoff[a] = tot;
        alen[a] = std::max(hlen[a], 0);
        tot += alen[a];
    }
    std::vector<uint8_t> flat((size_t)tot + 16, 0);
    for (int32_t a = 0; a < n_adp; ++a) std::copy(hcodes + hoff[a], hcodes + hoff[a] + alen[a], flat.begin() + aoff[a]);
    if (int rc = s->tabs.ensure(4 * img.size())) return rc;
    if (int rc = s->adp.ensure(flat.size())) return rc;
    if (int rc = s->adp_off.ensure(4 * aoff.size())) return rc;
    if (int rc = s->adp_len.ensure(4 * alen.size())) return rc;
    if (int rc = s->cnt.ensure(4 * kCls)) return rc;
    if (int rc = s->thr.ensure(4 * thr.size())) return rc;
    if (int rc = s->ccnt.ensure(8)) return rc;
    SD_TRY(hipMemcpy(s->tabs.p, img.data(), 4 * img.size(), hipMemcpyHostToDevice));
    SD_TRY(hipMemcpy(s->adp.p, flat.data(), flat.size(), hipMemcpyHostToDevice));
    SD_TRY(hipMemcpy(s->adp_off.p, aoff.data(), 4 * aoff.size(), hipMemcpyHostToDevice));
    SD_TRY(hipMemcpy(s->adp_len.p, alen.data(), 4 * alen.size(), hipMemcpyHostToDevice));
    SD_TRY(hipMemcpy(s->thr.p, thr.data(), 4 * thr.size(), hipMemcpyHostToDevice));
    A.tabs = (const uint32_t *)s->tabs.p;
    A.cnt = (int32_t *)s->cnt.p;
    s->ok = true;
    return 0;
}

void launch_band(const State *s, int E, int32_t cnt, int c, const uint8_t *codes, const int64_t *v_off,
                 const int32_t *v_len, const pcabi::Scoring &sc, int64_t n, hipStream_t st) {
    const dim3 grid((unsigned)((cnt + 255) / 256));
    const int4 *task = (const int4 *)s->task.p + c * s->cap;
    const uint8_t *adp = (const uint8_t *)s->adp.p;
    const int32_t *aoff = (const int32_t *)s->adp_off.p, *alen = (const int32_t *)s->adp_len.p;
    int32_t *bound = (int32_t *)s->bound.p;
    switch (E) {
#define C(X)                                                                                                   \
    case X:                                                                                                    \
        hipLaunchKernelGGL(k_seed_band<X>, grid, dim3(256), 0, st, task, cnt, codes, v_off, v_len, adp, aoff, \
                           alen, sc, (const int32_t *)s->thr.p, bound, n);                                    \
        break;
        C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13) C(14) C(15)
#undef C
    }
}
}  // namespace

// Middle-scan bounds from seeds. fb_rows[a]: register rows of adapter a's filter bucket (0: the
// adapter is not filtered). mode: 1 use seeds when the cost model prefers them, 2 whenever they
// apply. Returns 1 when done, 0 when seeds do not apply (the caller runs the score filter), < 0
// on error. Done: cands != nullptr receives the filtered pairs whose bound reaches their
// threshold, as sorted (a << 32 | read) keys (no bound array leaves the device); dcands !=
// nullptr receives the same keys unordered in device memory (valid until the next call) and
// n_dcands their count; otherwise s16 (int16, a * n + read) holds every bound (-8192: no seed).
int bounds(State *s, const void *adps_key, const uint8_t *hcodes, const int32_t *hoff, const int32_t *hlen,
           int32_t n_adp, const std::vector<int> &fb_rows, const uint8_t *codes, const int64_t *v_off,
           const int32_t *v_len, int64_t n, const pcabi::Scoring &sc, double threshold, int mode, int16_t *s16,
           std::vector<int64_t> *cands, const int64_t **dcands, int64_t *n_dcands, hipStream_t st) {
    if (mode <= 0 || n <= 0) return 0;
    (void)adps_key;
    bool same = s->planned && s->threshold == threshold && s->sc.ma == sc.ma && s->sc.mi == sc.mi &&
                s->sc.go == sc.go && s->sc.ge == sc.ge && (int32_t)s->key_len.size() == n_adp && s->key_rows == fb_rows;
    for (int32_t a = 0; same && a < n_adp; ++a) same = s->key_len[a] == hlen[a];
    if (same) {
        size_t q = 0;
        for (int32_t a = 0; same && a < n_adp; ++a)
            for (int32_t i = 0; same && i < hlen[a]; ++i) same = s->key_codes[q++] == hcodes[hoff[a] + i];
    }
    if (!same) {
        // a new plan: the old tables may still be read by work queued on `st`
        SD_TRY(hipStreamSynchronize(st));
        s->key_len.assign(hlen, hlen + n_adp);
        s->key_rows = fb_rows;
        s->key_codes.clear();
        for (int32_t a = 0; a < n_adp; ++a)
            s->key_codes.insert(s->key_codes.end(), hcodes + hoff[a], hcodes + hoff[a] + std::max(hlen[a], 0));
        s->threshold = threshold;
        s->sc = sc;
        s->scan_blocks = 0;
        if (int rc = plan(s, hcodes, hoff, hlen, n_adp, fb_rows, sc, threshold)) {
            s->planned = false;
            return rc;
        }
    }
    if (!s->ok) return 0;
    if (mode == 1 && !(s->cost_seed < 0.5 * s->cost_filter)) return 0;
    if (int rc = s->bound.ensure(sizeof(int32_t) * (size_t)n * n_adp)) return rc;
    ScanArgs A = s->a;
    A.codes = codes;
    A.v_off = v_off;
    A.v_len = v_len;
    A.n = n;
    for (int pass = 0; pass < 2; ++pass) {
        if (s->cap == 0) s->cap = 1 << 20;
        if (int rc = s->task.ensure(sizeof(int4) * kCls * (size_t)s->cap)) return rc;
        A.task = (int4 *)s->task.p;
        A.cap = s->cap;
        SD_TRY(hipMemsetAsync(A.cnt, 0, 4 * kCls, st));
        // every block resident at once (the blocks stride over the reads evenly: a second wave
        // of blocks would run on a partly idle chip)
        if (s->scan_blocks == 0) {
            int dev = 0, cus = 0, per_cu = 0;
            SD_TRY(hipGetDevice(&dev));
            SD_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            SD_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_seed_scan, 256, s->lds_bytes));
            s->scan_blocks = std::max(1, cus * std::max(1, per_cu));
        }
        const unsigned grid = (unsigned)std::min<int64_t>(n, s->scan_blocks);
        hipLaunchKernelGGL(k_seed_scan, dim3(grid), dim3(256), s->lds_bytes, st, A);
        SD_TRY(hipGetLastError());
        int32_t cnt[kCls];
        SD_TRY(hipMemcpyAsync(cnt, A.cnt, sizeof(cnt), hipMemcpyDeviceToHost, st));
        SD_TRY(hipStreamSynchronize(st));
        int64_t most = 0;
        for (int c = 0; c < kCls; ++c) {
            if (cnt[c] < 0) return fail(PCABI_E_DEVICE, "seed task counter overflow");
            most = std::max<int64_t>(most, cnt[c]);
        }
        if (most > s->cap) {
            if (pass == 1) return fail(PCABI_E_DEVICE, "seed tasks grew between passes");
            s->cap = most + most / 4;
            continue;
        }
        if (const char *dbg = std::getenv("PCABI_DEBUG"))
            if (dbg[0] == '1')
                std::fprintf(stderr, "[pcabi] seeds: %lld windows, band tasks %d (E=%d) + %d (E=%d), scan grid %u\n",
                             (long long)n, cnt[0], s->band[0], cnt[1], s->band[1], grid);
        SD_TRY(hipMemsetD32Async((hipDeviceptr_t)s->bound.p, pcabi::sf::NEG16, (size_t)n * n_adp, st));
        if (cnt[0] && cnt[1]) {   // both classes: side by side (atomicMax into one bound array)
            if (!s->side) {
                SD_TRY(hipStreamCreateWithFlags(&s->side, hipStreamNonBlocking));
                SD_TRY(hipEventCreateWithFlags(&s->fork, hipEventDisableTiming));
                SD_TRY(hipEventCreateWithFlags(&s->join, hipEventDisableTiming));
            }
            SD_TRY(hipEventRecord(s->fork, st));
            SD_TRY(hipStreamWaitEvent(s->side, s->fork, 0));
            launch_band(s, s->band[1], cnt[1], 1, codes, v_off, v_len, sc, n, s->side);
            launch_band(s, s->band[0], cnt[0], 0, codes, v_off, v_len, sc, n, st);
            SD_TRY(hipEventRecord(s->join, s->side));
            SD_TRY(hipStreamWaitEvent(st, s->join, 0));
        } else {
            for (int c = 0; c < kCls; ++c)
                if (cnt[c]) launch_band(s, s->band[c], cnt[c], c, codes, v_off, v_len, sc, n, st);
        }
        SD_TRY(hipGetLastError());
        const int64_t tot = n * (int64_t)n_adp;
        const unsigned grid_all = (unsigned)((tot + 255) / 256);
        if (!cands && !dcands) {
            hipLaunchKernelGGL(k_bound16, dim3(grid_all), dim3(256), 0, st, (const int32_t *)s->bound.p, tot, s16);
            SD_TRY(hipGetLastError());
            g_runs.fetch_add(1);
            return 1;
        }
        for (int cpass = 0; cpass < 2; ++cpass) {
            if (s->ccap == 0) s->ccap = 1 << 16;
            if (int rc = s->cands.ensure(sizeof(int64_t) * (size_t)s->ccap)) return rc;
            SD_TRY(hipMemsetAsync(s->ccnt.p, 0, 8, st));
            hipLaunchKernelGGL(k_cands, dim3(grid_all), dim3(256), 0, st, (const int32_t *)s->bound.p, n, tot,
                               (const int32_t *)s->thr.p, (int64_t *)s->cands.p, s->ccap,
                               (unsigned long long *)s->ccnt.p);
            SD_TRY(hipGetLastError());
            unsigned long long nc = 0;
            SD_TRY(hipMemcpyAsync(&nc, s->ccnt.p, 8, hipMemcpyDeviceToHost, st));
            SD_TRY(hipStreamSynchronize(st));
            if ((int64_t)nc > s->ccap) {
                s->ccap = (int64_t)nc + (int64_t)nc / 4;
                continue;
            }
            if (dcands) {                              // the keys stay on the device, unordered
                *dcands = (const int64_t *)s->cands.p;
                *n_dcands = (int64_t)nc;
                g_runs.fetch_add(1);
                return 1;
            }
            cands->resize((size_t)nc);
            if (nc) {
                SD_TRY(hipMemcpyAsync(cands->data(), s->cands.p, sizeof(int64_t) * nc, hipMemcpyDeviceToHost, st));
                SD_TRY(hipStreamSynchronize(st));
            }
            std::sort(cands->begin(), cands->end());
            g_runs.fetch_add(1);
            return 1;
        }
        return fail(PCABI_E_DEVICE, "seed candidates did not settle");
    }
    return fail(PCABI_E_DEVICE, "seed scan did not settle");
}

}  // namespace pcabi_seed

extern "C" int64_t pcabi_middle_seed_runs(void) { return pcabi_seed::g_runs.load(); }
