// pcabi_seed.hip -- exact seeding of the middle-adapter scan (round 1) on the GPU (gfx950).
//
// Reference: porechop_abi/nanopore_read.py:219-252 (find_middle_adapters): every read against
// every middle adapter, a hit when the best alignment's full identity (pid2 = m / l2) reaches
// the threshold. The engine's score filter computes every pair's best score S* to find the
// pairs that can hit. This unit finds them from exact k-mer seeds instead, and
// hands the engine the same kind of per-pair bound (int16 s16[a * n + k]).
//
// Why it is exact ("Seeds"):
//   * l2 counts the columns of the adapter span: every adapter base once (matched, mismatched,
//     against a gap, or hanging off a read end) plus the read bases inserted inside the span.
//     So e = l2 - m non-matching columns, and pid2 >= theta gives e <= L (1 - theta) / theta.
//   * Cut the adapter into e + 1 pieces. An error column touches at most one piece, so one
//     piece aligns as an unbroken run of matches: the read holds that piece exactly. Each piece
//     contributes its first K bases (K = min(8, piece length)) as a probe.
//   * A probe found at read position q with adapter offset o puts the whole alignment inside
//     read columns [q - o - e, q - o + L + e) (at most e insertions on either side), clipped
//     to the read. The score-only DP over that window (free end gaps, as the full DP) scores
//     every alignment inside it, in particular that one, so the window's best S_w >= its score
//     >= the filter bound T (sf::filter_threshold). A window starting inside the read lets the
//     adapter head hang off for free there, which only raises S_w: still a bound.
//   * Pairs with no probe hit get NEG16 (no alignment can reach theta); the others the largest
//     S_w. Pairs with a bound >= T go to the full attribute DP exactly as after the filter, and
//     masking in later rounds never creates a new theta-alignment, so the bounds carry over.
// Kernels (integer work, no MFMA):
//   k_seed_scan    one block per read (grid-stride), 4 positions per lane: the 8-mer codes of the
//                  positions, probe bitmaps (K = 4..8, 4^K bits each) in LDS, hits expanded into
//                  (read, adapter, window) tasks per row class, staged per block in LDS;
//   k_seed_window  one lane per task: Gotoh score DP over the window, rows in registers (32 or
//                  64 with pass-through padding rows), atomicMax into the pair's bound;
//   k_bound16      bound -> int16 s16.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
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
constexpr int kCls = 2;                        // row classes of k_seed_window
constexpr int kClsRows[kCls] = {32, 64};
constexpr int kMaxL = 64;
constexpr int kBitsDw = (1 << 16) / 32 + (1 << 14) / 32 + (1 << 12) / 32 + (1 << 10) / 32 + (1 << 8) / 32;
constexpr int kNeg = -(1 << 20);

struct ScanArgs {
    const uint8_t *codes;
    const int64_t *v_off;
    const int32_t *v_len;
    int64_t n;
    const uint32_t *bits;       // bitmaps of the probe k-mers, K = 4..8 (absent: no dwords)
    int32_t bits_off[kNK];      // dword offset of K's bitmap, -1 when no probe has length K
    int32_t n_bits;             // dwords in all bitmaps
    const int32_t *head;        // CSR over the probe codes, 4^K + 1 entries per present K
    int64_t head_off[kNK];
    const int32_t *ent;         // (adapter << 8) | piece offset o
    const int32_t *info;        // per adapter: L | e << 8 | cls << 16
    int4 *task;                 // kCls regions of cap tasks: (read, adapter, window start, columns)
    int64_t cap;
    int32_t *cnt;               // tasks per class (may exceed cap: the caller grows and reruns)
};

// Tasks are staged per block in LDS (LDS atomics) and appended to the global regions in
// chunks, one global atomic per chunk: a global atomic per task on the two class counters
// serialised the scan (76 ms for ~10 M tasks).
constexpr int kBuf = 512;

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
    __shared__ uint32_t bits[kBitsDw];
    __shared__ Stage sg;
    for (int i = threadIdx.x; i < a.n_bits; i += 256) bits[i] = a.bits[i];
    if (threadIdx.x < kCls) sg.cnt[threadIdx.x] = 0;
    __syncthreads();
    for (int64_t k = blockIdx.x; k < a.n; k += gridDim.x) {
        const int len = a.v_len[k];
        const uint8_t *base = a.codes + a.v_off[k];
        for (int p0b = 0; p0b < len; p0b += 1024) {      // block-uniform: every lane takes part
            const int p0 = p0b + 4 * (int)threadIdx.x;
            uint32_t valid = 0;
            uint32_t c2[11];
#pragma unroll
            for (int t = 0; t < 11; ++t) {
                const uint32_t b = (p0 + t < len) ? base[p0 + t] : 4u;
                valid |= (b < 4u ? 1u : 0u) << t;
                c2[t] = b & 3u;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t c8 = 0;
#pragma unroll
                for (int t = 0; t < 8; ++t) c8 = (c8 << 2) | c2[i + t];
                const int q = p0 + i;
#pragma unroll
                for (int kk = 0; kk < kNK; ++kk) {
                    if (a.bits_off[kk] < 0) continue;      // uniform
                    const int K = kMinK + kk;
                    const uint32_t need = (1u << K) - 1;
                    const uint32_t code = c8 >> (2 * (kMaxK - K));
                    if (((valid >> i) & need) != need) continue;
                    if (!((bits[a.bits_off[kk] + (code >> 5)] >> (code & 31)) & 1u)) continue;
                    const int e = a.head[a.head_off[kk] + code + 1];
                    for (int b = a.head[a.head_off[kk] + code]; b < e; ++b) {
                        const int en = a.ent[b];
                        const int ad = en >> 8, o = en & 255;
                        const int inf = a.info[ad];
                        const int L = inf & 255, er = (inf >> 8) & 255;
                        const int ws = max(q - o - er, 0);
                        const int we = min(q - o + L + er, len);
                        stage_task(sg, inf >> 16, make_int4((int)k, ad, ws, we - ws), a);
                    }
                }
            }
            flush(sg, kBuf / 2, a);
        }
    }
    flush(sg, 1, a);
}

// One lane per task: the best score of the adapter against the window (free end gaps on all
// four sides, as pcabi_dp.h / the oracle's build_rows), RPL rows with the adapter in the
// bottom L rows; the rows above it score 0 against anything, so they pass S = 0 through (row 0).
// Substitution scores come from one 6-bit signed field per read code (0..4) per row.
template <int RPL>
__global__ __launch_bounds__(256) void k_seed_window(const int4 *task, int32_t n_task, const uint8_t *codes,
                                                     const int64_t *v_off, const uint8_t *adp, const int32_t *adp_off,
                                                     const int32_t *info, pcabi::Scoring sc, int32_t *bound,
                                                     int64_t n) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n_task) return;
    const int4 tk = task[t];
    const int L = info[tk.y] & 255;
    const int pad = RPL - L;
    const uint8_t *ac = adp + adp_off[tk.y] - pad;
    uint32_t tab[RPL];
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
        uint32_t f = 0;
        if (i >= pad) {
            const int b = ac[i];
#pragma unroll
            for (int c = 0; c < 5; ++c) f |= ((uint32_t)((c == b) ? sc.ma : sc.mi) & 63u) << (6 * c);
        }
        tab[i] = f;
    }
    int S[RPL], H[RPL];
#pragma unroll
    for (int i = 0; i < RPL; ++i) { S[i] = 0; H[i] = kNeg; }
    int best = 0;                                        // S(L, 0)
    const uint8_t *w = codes + v_off[tk.x] + tk.z;
    const int nw = tk.w;
    for (int j = 0; j < nw; ++j) {
        const int sh = 6 * min((int)w[j], 4);
        int diag = 0, up = 0, V = kNeg;                  // row 0: S = 0
#pragma unroll
        for (int i = 0; i < RPL; ++i) {
            const int sub = __builtin_amdgcn_sbfe((int)tab[i], sh, 6);
            const int d = diag + sub;
            const int h = max(H[i] + sc.ge, S[i] + sc.go);
            V = max(V + sc.ge, up + sc.go);
            const int s = max(d, max(h, V));
            diag = S[i];
            S[i] = s;
            H[i] = h;
            up = s;
        }
        best = max(best, S[RPL - 1]);                    // last row
    }
#pragma unroll
    for (int i = 0; i < RPL; ++i) best = max(best, S[i]);   // last column
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
    // plan cache key
    const void *adps = nullptr;
    double threshold = -1.0;
    pcabi::Scoring sc{0, 0, 0, 0};
    bool planned = false, ok = false;
    double cost_seed = 0.0, cost_filter = 0.0;    // per read position (model units)
    ScanArgs a{};
    Buf bits, head, ent, info, adp, adp_off, task, cnt, bound, thr, cands, ccnt;
    int64_t cap = 0, ccap = 0;
};

State *create() { return new State(); }
void destroy(State *s) { delete s; }

namespace {
// Cost model per read position (VALU slots / issue rate, tools/valu_microbench.hip): the packed
// filter spends 4 packed ops per cell (rate 0.23), a window cell ~8 ops (~0.3), the scan ~60
// (~0.4) per position, and a random position hits a K-probe with probability 1 / 4^K.
constexpr double kFilterCell = 4.0 / 0.23, kWindowCell = 8.0 / 0.3, kScanPos = 60.0 / 0.4;

int plan(State *s, const uint8_t *hcodes, const int32_t *hoff, const int32_t *hlen, int32_t n_adp,
         const std::vector<int> &fb_rows, const pcabi::Scoring &sc, double threshold) {
    s->planned = true;
    s->ok = false;
    if (!(threshold > 0.0) || sc.ma > 31 || sc.ma < -32 || sc.mi > 31 || sc.mi < -32 || sc.go >= 0 || sc.ge >= 0)
        return 0;
    const double th = (threshold - 1e-5) / 100.0;
    if (th <= 0.0 || th > 1.0) return 0;
    std::vector<std::vector<std::vector<int32_t>>> lists(kNK);
    std::vector<int32_t> info((size_t)n_adp, 0);
    std::vector<int32_t> thr((size_t)n_adp, INT32_MAX);   // not under the filter: the caller adds them
    double filt = 0.0, seed = kScanPos;
    for (int32_t a = 0; a < n_adp; ++a) {
        if (fb_rows[a] <= 0) continue;                 // not under the filter: always a candidate
        const int L = hlen[a];
        if (L <= 0 || L > kMaxL) return 0;
        for (int i = 0; i < L; ++i)
            if (hcodes[hoff[a] + i] > 3) return 0;
        const int T = pcabi::sf::filter_threshold(L, threshold, sc);
        if (T <= pcabi::sf::NEG16) return 0;
        const int e = (int)std::floor((double)L * (1.0 - th) / th + 1e-9);
        if (e > 200) return 0;
        const int plen = L / (e + 1);
        const int K = std::min(kMaxK, plen);
        if (K < kMinK) return 0;
        const int cls = L <= kClsRows[0] ? 0 : 1;
        info[a] = L | (e << 8) | (cls << 16);
        thr[a] = T;
        filt += kFilterCell * fb_rows[a];
        auto &lk = lists[K - kMinK];
        if (lk.empty()) lk.resize((size_t)1 << (2 * K));
        for (int p = 0; p <= e; ++p) {
            const int o = p * plen;
            uint32_t code = 0;
            for (int t = 0; t < K; ++t) code = (code << 2) | hcodes[hoff[a] + o + t];
            lk[code].push_back((a << 8) | o);
            seed += kWindowCell * (double)(L + 2 * e) * kClsRows[cls] / (double)((size_t)1 << (2 * K));
        }
    }
    s->cost_seed = seed;
    s->cost_filter = filt;
    // device tables
    std::vector<uint32_t> bits;
    std::vector<int32_t> head, ent;
    ScanArgs &A = s->a;
    for (int kk = 0; kk < kNK; ++kk) {
        A.bits_off[kk] = -1;
        A.head_off[kk] = 0;
        if (lists[kk].empty()) continue;
        const size_t nc = lists[kk].size();
        A.bits_off[kk] = (int32_t)bits.size();
        A.head_off[kk] = (int64_t)head.size();
        bits.resize(bits.size() + std::max<size_t>(nc / 32, 1), 0u);
        for (size_t c = 0; c < nc; ++c) {
            head.push_back((int32_t)ent.size());
            if (!lists[kk][c].empty()) bits[A.bits_off[kk] + c / 32] |= 1u << (c % 32);
            for (int32_t x : lists[kk][c]) ent.push_back(x);
        }
        head.push_back((int32_t)ent.size());
    }
    if (ent.empty()) return 0;
    A.n_bits = (int32_t)bits.size();
    std::vector<int32_t> aoff((size_t)n_adp);
    int32_t tot = 0;
    for (int32_t a = 0; a < n_adp; ++a) { aoff[a] = tot; tot += std::max(hlen[a], 0); }
    if (int rc = s->bits.ensure(4 * bits.size())) return rc;
    if (int rc = s->head.ensure(4 * head.size())) return rc;
    if (int rc = s->ent.ensure(4 * ent.size())) return rc;
    if (int rc = s->info.ensure(4 * info.size())) return rc;
    if (int rc = s->adp.ensure((size_t)tot + 2 * kMaxL)) return rc;
    if (int rc = s->adp_off.ensure(4 * aoff.size())) return rc;
    if (int rc = s->cnt.ensure(4 * kCls)) return rc;
    if (int rc = s->thr.ensure(4 * thr.size())) return rc;
    if (int rc = s->ccnt.ensure(8)) return rc;
    SD_TRY(hipMemcpy(s->thr.p, thr.data(), 4 * thr.size(), hipMemcpyHostToDevice));
    // kMaxL bytes before the first adapter: the window kernel forms addresses of up to RPL - L
    // bytes before an adapter (padding rows it never reads)
    std::vector<uint8_t> flat((size_t)tot + 2 * kMaxL, 0);
    for (int32_t a = 0; a < n_adp; ++a)
        std::copy(hcodes + hoff[a], hcodes + hoff[a] + std::max(hlen[a], 0), flat.begin() + kMaxL + aoff[a]);
    SD_TRY(hipMemcpy(s->bits.p, bits.data(), 4 * bits.size(), hipMemcpyHostToDevice));
    SD_TRY(hipMemcpy(s->head.p, head.data(), 4 * head.size(), hipMemcpyHostToDevice));
    SD_TRY(hipMemcpy(s->ent.p, ent.data(), 4 * ent.size(), hipMemcpyHostToDevice));
    SD_TRY(hipMemcpy(s->info.p, info.data(), 4 * info.size(), hipMemcpyHostToDevice));
    SD_TRY(hipMemcpy((uint8_t *)s->adp.p, flat.data(), flat.size(), hipMemcpyHostToDevice));
    SD_TRY(hipMemcpy(s->adp_off.p, aoff.data(), 4 * aoff.size(), hipMemcpyHostToDevice));
    A.bits = (const uint32_t *)s->bits.p;
    A.head = (const int32_t *)s->head.p;
    A.ent = (const int32_t *)s->ent.p;
    A.info = (const int32_t *)s->info.p;
    A.cnt = (int32_t *)s->cnt.p;
    s->ok = true;
    return 0;
}

template <int RPL>
void launch_window(const State *s, int32_t cnt, int c, const uint8_t *codes, const int64_t *v_off,
                   const pcabi::Scoring &sc, int64_t n, hipStream_t st) {
    hipLaunchKernelGGL(k_seed_window<RPL>, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st,
                       (const int4 *)s->task.p + c * s->cap, cnt, codes, v_off, (const uint8_t *)s->adp.p + kMaxL,
                       (const int32_t *)s->adp_off.p, (const int32_t *)s->info.p, sc, (int32_t *)s->bound.p, n);
}
}  // namespace

// Middle-scan bounds from seeds. fb_rows[a]: register rows of adapter a's filter bucket (0: the
// adapter is not filtered). mode: 1 use seeds when the cost model prefers them, 2 whenever they
// apply. Returns 1 when done, 0 when seeds do not apply (the caller runs the score filter), < 0
// on error. Done: cands != nullptr receives the filtered pairs whose bound reaches their
// threshold, as sorted (a << 32 | read) keys (no bound array leaves the device); otherwise s16
// (int16, a * n + read) holds every bound.
int bounds(State *s, const void *adps_key, const uint8_t *hcodes, const int32_t *hoff, const int32_t *hlen,
           int32_t n_adp, const std::vector<int> &fb_rows, const uint8_t *codes, const int64_t *v_off,
           const int32_t *v_len, int64_t n, const pcabi::Scoring &sc, double threshold, int mode, int16_t *s16,
           std::vector<int64_t> *cands, hipStream_t st) {
    if (mode <= 0 || n <= 0) return 0;
    if (!s->planned || s->adps != adps_key || s->threshold != threshold || s->sc.ma != sc.ma || s->sc.mi != sc.mi ||
        s->sc.go != sc.go || s->sc.ge != sc.ge) {
        // a new plan: the old tables may still be read by work queued on `st`
        SD_TRY(hipStreamSynchronize(st));
        s->adps = adps_key;
        s->threshold = threshold;
        s->sc = sc;
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
        const unsigned grid = (unsigned)std::min<int64_t>(n, 8192);
        hipLaunchKernelGGL(k_seed_scan, dim3(grid), dim3(256), 0, st, A);
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
        SD_TRY(hipMemsetD32Async((hipDeviceptr_t)s->bound.p, pcabi::sf::NEG16, (size_t)n * n_adp, st));
        if (cnt[0]) launch_window<32>(s, cnt[0], 0, codes, v_off, sc, n, st);
        if (cnt[1]) launch_window<64>(s, cnt[1], 1, codes, v_off, sc, n, st);
        const int64_t tot = n * (int64_t)n_adp;
        const unsigned grid_all = (unsigned)((tot + 255) / 256);
        if (!cands) {
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
