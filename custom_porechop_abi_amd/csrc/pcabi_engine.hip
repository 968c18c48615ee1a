// pcabi_engine.hip -- gfx950 kernels + C ABI of the adapter-alignment engine (include/pcabi.h).
//
// Kernel map:
//   k_align<RPL, AFFINE, KIND>  one lane = one (window, adapter) DP with the adapter's RPL rows
//                               in VGPRs, one column (read base) per step (pcabi_dp.h). The
//                               wave's adapter is uniform. KIND picks the DP core: PACKED
//                               (score|tie-break|attributes in one int32 key, substitution keys
//                               from an LDS table), FAST (separate score/attribute registers,
//                               adapters <= 64) or GENERIC (any scoring, adapters <= 128).
//                               Two work shapes: cross (every window x every adapter of a
//                               bucket; XCD-aware tile order) and pairs (explicit tasks grouped
//                               into per-adapter waves on the host).
//   k_end_trim                  per-read decision epilogue (nanopore_read.py:175-217).
//   k_best_full_id              per-adapter max of the full-adapter identity
//                               (nanopore_read.py:158-173), deterministic (max is exact).
//   k_first_hit                 middle-scan round 1: first adapter over the threshold per read
//                               (nanopore_read.py:219-252).
//   k_tile_windows              window list -> tile layout (coalesced cross-mode reads).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdio>
#include <memory>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/pcabi.h"
#include "pcabi_dp.h"
#include "pcabi_kern.h"

namespace {
thread_local std::string g_err;
}  // namespace

namespace pcabi_eng {
int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
}  // namespace pcabi_eng

using namespace pcabi_eng;

namespace {


int bucket_of(int L, const pcabi::Scoring &sc, bool allow_wide = true) {
    if (L > kMaxRPL) return kStripedBucket;
    if (L <= 64) {
        const int rpl = (L + 3) & ~3;
        if (pcabi::fast_ok(L, rpl, sc)) return rpl / 4 - 1;
    } else if (allow_wide && L <= pcabi::pk::MAX_L) {
        const int rpl = (L + 3) & ~3;
        if (pcabi::packed_ok(L, rpl, sc)) return 16 + (rpl - 68) / 4;
    } else if (allow_wide && L <= pcabi::pk::MAX_L_LONG) {
        const int b = L <= 96 ? 22 : (L <= 112 ? 23 : 24);
        if (pcabi::long_ok(L, kBuckets[b].rpl, sc)) return b;
    }
    // The generic core keeps every row's state in registers: past 64 rows under affine gaps it
    // spills (k_align<96 / 128, true, 1>: hundreds of VGPRs to scratch) and runs slower than the
    // striped core, which holds 32 rows at a time.
    if (L > 64 && sc.go != sc.ge) return kStripedBucket;
    for (int b = 0; b < kNumBuckets; ++b)
        if (kBuckets[b].kind == GENERIC && L <= kBuckets[b].rpl) return b;
    return -1;
}

// ---- middle-scan score filter (pcabi_dp.h filter_lane) -------------------------------------------
// PCABI_MIDDLE_FILTER=0 in the environment turns it off (A/B timing; results are identical).
bool middle_filter_on() {
    const char *e = std::getenv("PCABI_MIDDLE_FILTER");
    return !(e && e[0] == '0');
}

// Owned end columns per chunk of the middle scan's candidate DP (pcabi_dp.h sf::chunk_plan):
// short enough that the longest read's chunks finish with the rest, long enough that the D-column
// lead-in of each chunk stays a few percent. A round with few candidates (later rounds: the
// reads that just hit) takes shorter chunks, down to kChunkColsMin, while the task list stays
// within kChunkTasks: a launch of a few waves runs as long as its longest chunk, one lane per
// column, so the chunk length is its latency.
constexpr int kChunkCols = 512;
constexpr int kChunkColsMin = 64;
constexpr int64_t kChunkTasks = 65536;

// PCABI_HOSTPROF=1: the middle scan prints its host-side time marks per call to stderr (where the
// host spends the time between the end trim's kernels and the scan's first launch).
struct HostMarks {
    bool on = false;
    std::vector<std::pair<const char *, std::chrono::steady_clock::time_point>> m;
    HostMarks() {
        const char *e = std::getenv("PCABI_HOSTPROF");
        on = e && e[0] == '1';
    }
    void mark(const char *what) {
        if (on) m.emplace_back(what, std::chrono::steady_clock::now());
    }
    ~HostMarks() {
        if (!on || m.empty()) return;
        std::string s;
        for (size_t k = 1; k < m.size(); ++k)
            s += std::string(" ") + m[k].first + "=" +
                 std::to_string(std::chrono::duration<double, std::micro>(m[k].second - m[k - 1].second).count());
        std::fprintf(stderr, "[pcabi hostprof] us:%s\n", s.c_str());
    }
};

thread_local HostMarks *g_hm = nullptr;
inline void hmark(const char *what) {
    if (g_hm) g_hm->mark(what);
}

// PCABI_DEBUG=1: the middle scan prints its candidate counts per round to stderr.
const bool g_debug = [] {
    const char *e = std::getenv("PCABI_DEBUG");
    return e && e[0] == '1';
}();

// Round 1 of the middle scan from exact seeds (pcabi_seed.hip) instead of the score filter:
// PCABI_MIDDLE_SEEDS=0 off, 1 (default) when the cost model prefers them, 2 whenever they apply.
int middle_seed_mode() {
    const char *e = std::getenv("PCABI_MIDDLE_SEEDS");
    if (!e || !e[0]) return 1;
    return e[0] == '0' ? 0 : (e[0] == '2' ? 2 : 1);
}

// Seeded rounds plan their candidate DP on the device (PCABI_MIDDLE_DEVPLAN=0: on the host).
bool middle_devplan_on() {
    const char *e = std::getenv("PCABI_MIDDLE_DEVPLAN");
    return !(e && e[0] == '0');
}

// Queued rounds run the candidate DP over the verified seeds' windows, with the whole read only for
// the candidates whose window winner is a hit the certificate cannot vouch for (k_certify). The
// windows pay on long reads only: the second plan's launches cost more than they save at 8 kb
// (2.90 -> 2.86 ms), break even at 12 kb and win 10-12 % from 16 kb (20 kb: 4.21 -> 3.70 ms,
// profiles/r03/final/windows_sweep/). So they run when the batch's mean read length reaches
// kWindowsMeanLen -- from the host lengths when the caller passes them, else from the previous
// call's round-1 segment total (pcabi_scan::last_mean). PCABI_MIDDLE_WINDOWS=1 / 0 forces them.
constexpr double kWindowsMeanLen = 10000.0;   // r05ac in-process A/B (graphs off): off 1.99 / on 2.03 ms at
                                              // 8 kb, off 2.50 / on 2.29 at 14 kb, off 3.21 / on 2.74 at 20 kb
bool middle_windows_on(double mean_len) {
    const char *e = std::getenv("PCABI_MIDDLE_WINDOWS");
    if (e && e[0] == '1') return true;
    if (e && e[0] == '0') return false;
    return mean_len >= kWindowsMeanLen;
}

// Queued rounds from this index on (0 = round 1) launch their band classes and candidate-DP
// buckets one after the other on the scan's stream: after round 1 only the reads that hit are
// left, their launches last a few microseconds, and each fork / join over side streams costs
// ~15-20 us of event latency (profiles/r03/final/kernel_trace_middle_8kb.csv). r05at (in-process
// A/B, profiles/r05/at/): from round 2 on (1) 1.93 ms at 8 kb / 2.53 at 20 kb, against 1.96-1.99 /
// 2.65-2.69 from round 3 on (2, the r03-r05 default, round 2 replayed from a graph) and 2.02 /
// 2.51 with round 1 serial too (0).
// round side by side). Captured round graphs (run_round) hold only serial rounds: a capture never
// records another caller's work on the shared side streams.
constexpr int kMiddleSerialFrom = 1;

// Device planning aims at this many waves per candidate-DP round (4 per SIMD): the chunk length
// is the longest of 512, 256, 128, 64 owned columns that still reaches it.
int64_t middle_plan_waves() {
    const char *e = std::getenv("PCABI_MIDDLE_PLAN_WAVES");
    return (e && e[0]) ? std::max<int64_t>(1, std::atoll(e)) : 4096;
}


// ---- decision epilogues --------------------------------------------------------------------

// One block per 64 reads: wave w takes adapters w, w + 4, ... of both sides (lane = read: the
// loads of one adapter's field are 256-B coalesced), the four partial maxima meet in LDS. (r03: one
// thread per read looped over every adapter -- 391 blocks for 100k reads, latency-bound.) r06: the
// four fields a decision reads (rs, re, m, l1: 16 of the result's 32 bytes) are loaded
// unconditionally, four adapters at a time, so a wave keeps 16 independent loads in flight instead
// of a dependent pair per adapter (the kernel reads 149 MB per headline step: HBM-bound, 42 us in r05).
struct EndFields {
    int rs, re, m, l1;
};
__device__ __forceinline__ EndFields end_fields(const int32_t *res, int64_t stride, int64_t i) {
    return EndFields{res[0 * stride + i], res[1 * stride + i], res[5 * stride + i], res[6 * stride + i]};
}

__global__ __launch_bounds__(256) void k_end_trim(const int32_t *sres, int64_t sstride, int32_t n_sa,
                                                  const int32_t *eres, int64_t estride, int32_t n_ea,
                                                  int64_t n_read, int end_size, int extra,
                                                  double thr, int min_trim,
                                                  int32_t *start_trim, int32_t *end_trim,
                                                  uint8_t *shit, uint8_t *ehit) {
    __shared__ int s_st[4][64], s_et[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t r = (int64_t)blockIdx.x * 64 + lane;
    const bool live = r < n_read;
    constexpr int U = 4;                              // adapters in flight per wave
    // find_start_trim (nanopore_read.py:175-195)
    int st = 0;
    for (int a0 = w; live && a0 < n_sa; a0 += 4 * U) {
        EndFields f[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int a = a0 + 4 * u;
            f[u] = a < n_sa ? end_fields(sres, sstride, (int64_t)a * n_read + r) : EndFields{-1, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int a = a0 + 4 * u;
            if (a >= n_sa) break;
            const int rs = f[u].rs;
            int re1 = 0, hit = 0;
            double partial = 0.0;
            if (rs != -1) {
                re1 = f[u].re + 1;
                partial = pcabi::pid6(f[u].m, f[u].l1);
            }
            if (partial > thr && re1 != end_size && re1 - rs >= min_trim) {
                st = max(st, re1 + extra);
                hit = 1;
            }
            if (shit) shit[(int64_t)a * n_read + r] = (uint8_t)hit;
        }
    }
    // find_end_trim (nanopore_read.py:197-217)
    int et = 0;
    for (int a0 = w; live && a0 < n_ea; a0 += 4 * U) {
        EndFields f[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int a = a0 + 4 * u;
            f[u] = a < n_ea ? end_fields(eres, estride, (int64_t)a * n_read + r) : EndFields{-1, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int a = a0 + 4 * u;
            if (a >= n_ea) break;
            const int rs = f[u].rs;
            int re1 = 0, hit = 0;
            double partial = 0.0;
            if (rs != -1) {
                re1 = f[u].re + 1;
                partial = pcabi::pid6(f[u].m, f[u].l1);
            }
            if (partial > thr && rs != 0 && re1 - rs >= min_trim) {
                et = max(et, (end_size - rs) + extra);
                hit = 1;
            }
            if (ehit) ehit[(int64_t)a * n_read + r] = (uint8_t)hit;
        }
    }
    s_st[w][lane] = st;
    s_et[w][lane] = et;
    __syncthreads();
    if (w == 0 && live) {
        start_trim[r] = max(max(s_st[0][lane], s_st[1][lane]), max(s_st[2][lane], s_st[3][lane]));
        end_trim[r] = max(max(s_et[0][lane], s_et[1][lane]), max(s_et[2][lane], s_et[3][lane]));
    }
}

// best[a] = max(best[a], max_w pid2): one block per adapter, uint64 ordering of non-negative
// doubles == numeric ordering, so the max is exact and order independent.
__global__ __launch_bounds__(256) void k_best_full_id(const int32_t *res, int64_t stride, int64_t n_win,
                                                      double *best) {
    const int a = blockIdx.x;
    __shared__ unsigned long long red[256];
    unsigned long long mx = 0;
    for (int64_t w = threadIdx.x; w < n_win; w += 256) {
        const int64_t i = (int64_t)a * n_win + w;
        const int rs = res[0 * stride + i];
        const double full = (rs == -1) ? 0.0 : pcabi::pid6(res[5 * stride + i], res[7 * stride + i]);
        const unsigned long long b = (unsigned long long)__double_as_longlong(full);
        mx = b > mx ? b : mx;
    }
    red[threadIdx.x] = mx;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] = red[threadIdx.x] > red[threadIdx.x + s] ? red[threadIdx.x] : red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const unsigned long long cur = (unsigned long long)__double_as_longlong(best[a]);
        best[a] = __longlong_as_double((long long)(red[0] > cur ? red[0] : cur));
    }
}

// Barcode call (porechop_abi/nanopore_read.py:408-482) over the barcode dicts that
// find_start_trim / find_end_trim fill (:193-195, :215-217). A side's dict is given as slots in
// insertion order: slot k holds barcode id name[k] with the full-adapter identity of adapter
// adp[k] (the LAST adapter of that name in set order -- a dict keeps a key's first position and
// its last value). The reference's stable sorts reduce to strict '>' scans in slot order:
//   per side  : best / second = first two of the descending stable sort
//   merged    : entries ordered by (-score, start before end, slot); best = the first, second =
//               the first entry whose name differs (the dedup keeps each name's first entry)
// Missing entries are ('none', 0.0), the reference's defaults (nanopore_read.py:58-61).
struct BcSide {
    const int32_t *res;
    int64_t stride;
    const int32_t *adp, *name;
    int32_t n;
};

__device__ __forceinline__ double bc_score(const BcSide &s, int k, int64_t n_read, int64_t r) {
    const int64_t i = (int64_t)s.adp[k] * n_read + r;
    return s.res[0 * s.stride + i] == -1 ? 0.0 : pcabi::pid6(s.res[5 * s.stride + i], s.res[7 * s.stride + i]);
}

__global__ __launch_bounds__(256) void k_barcode_call(BcSide st, BcSide en, int64_t n_read, double thr, double diff,
                                                      int require_two, int32_t *call, double *scores) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_read) return;
    int c = -1;
    if (require_two) {
        double b[2][2] = {{0.0, 0.0}, {0.0, 0.0}};   // [side][best, second]
        int bn[2] = {-1, -1};
        int cnt[2] = {0, 0};
        for (int side = 0; side < 2; ++side) {
            const BcSide &s = side ? en : st;
            for (int k = 0; k < s.n; ++k) {
                const double x = bc_score(s, k, n_read, r);
                if (cnt[side] == 0 || x > b[side][0]) {
                    if (cnt[side] > 0) b[side][1] = b[side][0];
                    b[side][0] = x;
                    bn[side] = s.name[k];
                } else if (cnt[side] == 1 || x > b[side][1]) {
                    b[side][1] = x;
                }
                ++cnt[side];
            }
        }
        if (b[0][0] >= thr && b[1][0] >= thr && b[0][0] >= b[0][1] + diff && b[1][0] >= b[1][1] + diff &&
            bn[0] == bn[1])
            c = bn[0];
        if (scores) {
            scores[4 * r + 0] = b[0][0]; scores[4 * r + 1] = b[0][1];
            scores[4 * r + 2] = b[1][0]; scores[4 * r + 3] = b[1][1];
        }
    } else {
        double b1 = 0.0, b2 = 0.0;
        int n1 = -1;
        bool has1 = false, has2 = false;
        for (int side = 0; side < 2; ++side) {
            const BcSide &s = side ? en : st;
            for (int k = 0; k < s.n; ++k) {
                const double x = bc_score(s, k, n_read, r);
                const int nm = s.name[k];
                if (!has1 || x > b1) {
                    // the previous best heads the entries of every other name
                    if (has1 && n1 != nm) { b2 = b1; has2 = true; }
                    b1 = x; n1 = nm; has1 = true;
                } else if (nm != n1 && (!has2 || x > b2)) {
                    b2 = x; has2 = true;
                }
            }
        }
        if (b1 >= thr && b1 >= b2 + diff) c = has1 ? n1 : -1;
        if (scores) {
            scores[4 * r + 0] = b1; scores[4 * r + 1] = b2;
            scores[4 * r + 2] = 0.0; scores[4 * r + 3] = 0.0;
        }
    }
    call[r] = c;
}

// Middle-scan round 1 (porechop_abi/nanopore_read.py:219-252): per read, the FIRST adapter in
// list order whose full-adapter identity is not below the threshold on the unmasked read. The
// reference's loop hits exactly that adapter first (the ones before it fail on this same
// sequence and are never revisited), so only this hit leaves the device: hits[f * hit_stride +
// w] for f = adapter (-1 = none), rs, re (inclusive), m, l2.
__global__ __launch_bounds__(256) void k_first_hit(const int32_t *res, int64_t stride, int64_t n_win,
                                                   int32_t n_adp, double thr, const int32_t *start_adp,
                                                   int32_t *hits, int64_t hit_stride) {
    const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (w >= n_win) return;
    int32_t fa = -1, frs = -1, fre = 0, fm = 0, fl = 0;
    for (int a = start_adp ? start_adp[w] : 0; a < n_adp; ++a) {
        const int64_t i = (int64_t)a * n_win + w;
        const int rs = res[0 * stride + i];
        const int m = res[5 * stride + i], l2 = res[7 * stride + i];
        const double full = (rs == -1) ? 0.0 : pcabi::pid6(m, l2);
        if (!(full < thr)) {   // Python: `if full < middle_threshold: break` (NaN does not break)
            fa = a; frs = rs; fre = res[1 * stride + i]; fm = m; fl = l2;
            break;
        }
    }
    hits[0 * hit_stride + w] = fa;
    hits[1 * hit_stride + w] = frs;
    hits[2 * hit_stride + w] = fre;
    hits[3 * hit_stride + w] = fm;
    hits[4 * hit_stride + w] = fl;
}

// Views of a subset of windows: sub[k] = window idx[k].
__global__ __launch_bounds__(256) void k_gather_views(const int64_t *win_off, const int32_t *win_len,
                                                      const int32_t *idx, int64_t n, int64_t *sub_off,
                                                      int32_t *sub_len) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    sub_off[k] = win_off[idx[k]];
    sub_len[k] = win_len[idx[k]];
}

// ---- input-preserving masking (r05) ------------------------------------------------------------
// The reference masks a COPY of the read (nanopore_read.py:225 masked_seq = the trimmed read, :234
// rebuilt with '-'), so the caller's sequence is never touched. The scan does the same on the
// device: the caller's codes are read-only, and a read's first hit copies the whole window into a
// shadow arena owned by the scan (16-byte aligned, zero tail padding for the window readers'
// look-ahead), with the hit's span masked as it is copied; from then on the read's effective offset
// eoff[w] (an offset from `codes`, like win_off) points at the copy, which later hits mask in place.
// Only reads that hit are ever copied (round 1: ~4.5 % of a batch); every round after round 1 runs
// on reads that hit in round 1 only.
__device__ __forceinline__ int64_t shadow_bytes(int32_t len) { return ((int64_t)max(len, 0) + 16 + 15) & ~(int64_t)15; }

// Masking of a round's hits (nanopore_read.py:245, the span becomes '-', Dna5 N): the blocks stride
// over the list (8 int32 per hit, k_round_hits' layout), a block's threads over the read. o[7] > 0:
// the read's first hit, shadow at arena byte (o[7] - 1) * 16 (k_round_hits' allocation): the window
// is copied from the caller's codes with the span masked, and eoff redirected; o[7] == 0: the read
// already has its copy (eoff), the span is masked there. *bump > cap (the round's allocations did
// not fit): nothing is copied or masked, the round is flagged (rflag bit 8) and holds no next round,
// so the host grows the arena and queues it again.
__global__ __launch_bounds__(256) void k_mask_list(const uint8_t *codes, const int64_t *win_off, int64_t *eoff,
                                                   const int32_t *win_len, const int32_t *list, int32_t *n_dev,
                                                   uint8_t *arena, int64_t arena_rel, int64_t cap,
                                                   const unsigned long long *bump, int32_t *rflag) {
    if ((int64_t)*bump > cap) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (rflag) *rflag |= 8;
            *n_dev = 0;
        }
        return;
    }
    const int64_t nh = *n_dev;
    for (int64_t j = blockIdx.x; j < nh; j += gridDim.x) {
        const int32_t *o = list + 8 * j;
        const int32_t w = o[0], rs = o[2], rend = rs == -1 ? 0 : o[3] + 1;
        if (o[7] > 0) {
            // 16 bytes per thread and pass: the source's aligned dwords (those holding a byte of the
            // window: the caller's padding is not assumed), shifted into place, the span masked,
            // bytes past the window zero, one 16-byte store
            const int64_t at = (int64_t)(o[7] - 1) * 16;
            const int32_t len = win_len[w];
            const int64_t nb = shadow_bytes(len);
            const uintptr_t sa = (uintptr_t)(codes + win_off[w]);
            const uint32_t *s4 = reinterpret_cast<const uint32_t *>(sa & ~(uintptr_t)3);
            const int a0 = (int)(sa & 3), sh = 8 * a0;
            const int64_t lim = (int64_t)len + a0;      // source dword k holds window bytes iff 4k < lim
            uint4 *dst = reinterpret_cast<uint4 *>(arena + at);
            for (int64_t c = threadIdx.x; c * 16 < nb; c += 256) {
                uint32_t d[5];
#pragma unroll
                for (int k = 0; k < 5; ++k) d[k] = (4 * (4 * c + k) < lim) ? s4[4 * c + k] : 0u;
                uint32_t v[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    uint32_t x = sh ? __builtin_amdgcn_alignbit(d[i + 1], d[i], sh) : d[i];
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const int64_t pos = 16 * c + 4 * i + b;
                        const uint32_t m = 0xFFu << (8 * b);
                        if (pos >= len) x &= ~m;
                        else if (pos >= rs && pos < rend) x = (x & ~m) | (4u << (8 * b));
                    }
                    v[i] = x;
                }
                dst[c] = make_uint4(v[0], v[1], v[2], v[3]);
            }
            if (threadIdx.x == 0) eoff[w] = arena_rel + at;
        } else {
            // the copy already exists: eoff[w] lies in the arena
            uint8_t *dst = arena + (eoff[w] - arena_rel);
            for (int64_t i = rs + threadIdx.x; i < rend; i += 256) dst[i] = 4;
        }
    }
}

// The arena moved (grown): every redirected offset follows it.
__global__ __launch_bounds__(256) void k_shadow_rebase(const int64_t *win_off, int64_t *eoff, int64_t n, int64_t delta) {
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256)
        if (eoff[k] != win_off[k]) eoff[k] += delta;
}

// ---- device-planned candidate DP (middle scan, seeded rounds) --------------------------------
// The seeds leave the candidate pairs on the device as unordered keys (adapter << 32 | window).
// k_plan_count counts each adapter's tasks for the four chunk lengths, the host lays the waves
// out (one adapter per wave, adapters in bucket order: n_adp numbers, not tasks), k_plan_place
// writes the task slots, the DP runs per bucket, and k_merge_* pick per candidate the first chunk
// (read order) with the largest score, then per window the first adapter (list order) whose
// full identity is not below the threshold -- the host path's rules (filtered_first_hits).
constexpr int kPlanC = 5;     // chunk lengths kPlanMin << c, c = 0..4
constexpr int kPlanMin = 32;  // (r05: 32-column chunks for the few whole reads a round certifies)

__device__ __forceinline__ int plan_tasks(int len, int span, int c) {
    if (span < 0) return 1;                          // whole windows
    const int C = kPlanMin << c;
    return (len + C - 1) / C;                        // sf::chunk_plan's chunk count
}

__device__ __forceinline__ bool plan_valid(int64_t key, const int32_t *v_len, const int32_t *start) {
    const int32_t a = (int32_t)(key >> 32), k = (int32_t)(key & 0xFFFFFFFF);
    return v_len[k] > 0 && (!start || a >= start[k]);
}

// Wave helpers (every lane of the wave takes part): sum, inclusive scan.
__device__ __forceinline__ int wave_sum(int x) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d);
    return x;
}
__device__ __forceinline__ int wave_incl_scan(int x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    return x;
}

// Candidates of one adapter are typically many (the reads' own adapter), so the per-adapter
// counters are updated once per (wave, adapter): the lanes of one adapter are reduced first.
// nc_dev != nullptr: the candidate count is on the device (at most nc); the blocks stride.
__global__ __launch_bounds__(256) void k_plan_count(const int64_t *cand, int64_t nc, const unsigned long long *nc_dev,
                                                    const int32_t *v_len, const int32_t *start, const int32_t *span,
                                                    int32_t *adp_tasks, const int32_t *cmask) {
    const int64_t ncl = nc_dev ? min((int64_t)*nc_dev, nc) : nc;
    const int lane = threadIdx.x & 63;
    for (int64_t b0 = (int64_t)blockIdx.x * 256; b0 < ncl; b0 += (int64_t)gridDim.x * 256) {   // uniform
        const int64_t i = b0 + threadIdx.x;
        const int64_t key = i < ncl ? cand[i] : 0;
        const bool active = i < ncl && plan_valid(key, v_len, start) && (!cmask || cmask[i]);
        const int32_t a = active ? (int32_t)(key >> 32) : -1;
        int nt[kPlanC] = {};
        if (active) {
            const int32_t k = (int32_t)(key & 0xFFFFFFFF);
#pragma unroll
            for (int c = 0; c < kPlanC; ++c) nt[c] = plan_tasks(v_len[k], span[a], c);
        }
        uint64_t pending = __ballot(active);
        while (pending) {                            // wave-uniform
            const int leader = __ffsll((unsigned long long)pending) - 1;
            const int32_t a0 = __shfl(a, leader);
            const bool mine = active && a == a0;
#pragma unroll
            for (int c = 0; c < kPlanC; ++c) {
                const int sum = wave_sum(mine ? nt[c] : 0);
                if (lane == leader) atomicAdd(&adp_tasks[a0 * kPlanC + c], sum);
            }
            pending &= ~__ballot(mine);
        }
    }
}

// Task slots: adapter a's tasks fill slots [wave_off[a] * 64, ...) in any order (a slot's result
// depends only on its own task); idle slots keep task_win = -1. cidx[a]: the chunk length of a's
// bucket (kPlanMin << cidx). nc_dev / slots_dev (device counts, nullptr: host values): the candidate
// count, and the slots the layout holds (a task past them is not written: the layout overflowed).
__global__ __launch_bounds__(256) void k_plan_place(const int64_t *cand, int64_t nc, const unsigned long long *nc_dev,
                                                    const int32_t *v_len, const int32_t *start, const int32_t *span,
                                                    const int32_t *cidx, const int64_t *wave_off, int32_t *fill,
                                                    int32_t *tw, int32_t *to, int4 *tck, int32_t *tcand,
                                                    const int64_t *slots_dev, int32_t *cbase_out, const int32_t *cmask) {
    const int64_t ncl = nc_dev ? min((int64_t)*nc_dev, nc) : nc;
    const int64_t slots = slots_dev ? *slots_dev : INT64_MAX;
    const int lane = threadIdx.x & 63;
    for (int64_t b0 = (int64_t)blockIdx.x * 256; b0 < ncl; b0 += (int64_t)gridDim.x * 256) {   // uniform
        const int64_t i = b0 + threadIdx.x;
        const int64_t key = i < ncl ? cand[i] : 0;
        const bool active = i < ncl && plan_valid(key, v_len, start) && (!cmask || cmask[i]);
        const int32_t a = active ? (int32_t)(key >> 32) : -1, k = (int32_t)(key & 0xFFFFFFFF);
        int n = 0, D = -1, c = 0, nt = 0;
        if (active) {
            n = v_len[k];
            D = span[a];
            c = cidx[a];
            nt = plan_tasks(n, D, c);
        }
        int64_t base = 0;
        uint64_t pending = __ballot(active);
        while (pending) {                            // wave-uniform: one atomic per (wave, adapter)
            const int leader = __ffsll((unsigned long long)pending) - 1;
            const int32_t a0 = __shfl(a, leader);
            const bool mine = active && a == a0;
            const int x = mine ? nt : 0;
            const int incl = wave_incl_scan(x);
            const int total = __shfl(incl, 63);
            int b1 = 0;
            if (lane == leader) b1 = atomicAdd(&fill[a0], total);
            b1 = __shfl(b1, leader);
            if (mine) base = wave_off[a0] * 64 + b1 + (incl - x);
            pending &= ~__ballot(mine);
        }
        if (cbase_out) {                             // the tasks are written by k_plan_fill
            if (i < ncl) cbase_out[i] = active ? (int32_t)base : -1;
            continue;
        }
        if (!active) continue;
        const int C = kPlanMin << c;
        for (int t = 0; t < nt; ++t) {
            const int64_t q = base + t;
            if (q >= slots) break;
            int4 ck = make_int4(0, 0, 0, 0);
            if (D >= 0) {                            // sf::chunk_plan, chunk t
                const int lo = 1 + t * C, hi = lo + C;
                const int st = max(0, lo - 1 - D);
                ck = hi > n ? make_int4(st, n - st, lo - st, -1) : make_int4(st, hi - 1 - st, lo - st, hi - st);
            }
            tw[q] = k;
            to[q] = (int32_t)q;
            tck[q] = ck;
            tcand[q] = (int32_t)i;
        }
    }
}

// The task slots of k_plan_place's candidates, one wave per candidate (its lanes over the chunks):
// a read of 8 kb has 63 chunks of 128 columns, which one lane wrote one after another.
__global__ __launch_bounds__(256) void k_plan_fill(const int64_t *cand, int64_t nc, const unsigned long long *nc_dev,
                                                   const int32_t *v_len, const int32_t *span, const int32_t *cidx,
                                                   const int32_t *cbase, int32_t *tw, int32_t *to, int4 *tck,
                                                   int32_t *tcand, const int64_t *slots_dev) {
    const int64_t ncl = nc_dev ? min((int64_t)*nc_dev, nc) : nc;
    const int64_t slots = *slots_dev;
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * 4;
    for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < ncl; i += waves) {
        const int32_t base = cbase[i];
        if (base < 0) continue;                      // wave-uniform
        const int64_t key = cand[i];
        const int32_t a = (int32_t)(key >> 32), k = (int32_t)(key & 0xFFFFFFFF);
        const int n = v_len[k], D = span[a], c = cidx[a];
        const int nt = plan_tasks(n, D, c), C = kPlanMin << c;
        for (int t = lane; t < nt; t += 64) {
            const int64_t q = (int64_t)base + t;
            if (q >= slots) break;
            int4 ck = make_int4(0, 0, 0, 0);
            if (D >= 0) {                            // sf::chunk_plan, chunk t
                const int lo = 1 + t * C, hi = lo + C;
                const int st = max(0, lo - 1 - D);
                ck = hi > n ? make_int4(st, n - st, lo - st, -1) : make_int4(st, hi - 1 - st, lo - st, hi - st);
            }
            tw[q] = k;
            to[q] = (int32_t)q;
            tck[q] = ck;
            tcand[q] = (int32_t)i;
        }
    }
}

// ---- candidate windows (device rounds, PCABI_MIDDLE_WINDOWS): one chunk per verified seed ------
// A verified seed (pcabi_seed.hip put_verified: read, adapter | E << 24, the diagonal's codes offset)
// is a band task of a candidate pair whose bound reached T. Every alignment of the pair scoring >= T
// holds an exact piece, whose task is verified, and stays within E diagonals of it: it ends in row L
// at a column of d0 + L - E .. d0 + L + E, or in the read's last column when the band reaches it. One
// chunk per verified seed that owns those columns (started D + 1 columns earlier: sf::chunk_plan's
// rule, so an owned cell >= T gets the whole read's score and attributes) replaces the pair's
// whole-read chunks -- 8 kb x L cells become ~(D + 2E) x L. The merge's rules are unchanged and
// still give the whole-read answer whenever it reaches T: the largest score, then the smallest first
// owned column (overlapping windows of one pair report the same first maximum of a shared cell).
__device__ __forceinline__ bool wseed_valid(const int4 &v, const int32_t *v_len, const int32_t *start) {
    const int32_t a = v.y & 0xFFFFFF, k = v.x;
    return v_len[k] > 0 && (!start || a >= start[k]);
}

__device__ __forceinline__ int4 wseed_chunk(const int4 &v, const int64_t *v_off, const int32_t *v_len,
                                            const int32_t *alen, const int32_t *span) {
    const int32_t a = v.y & 0xFFFFFF, E = (int32_t)((uint32_t)v.y >> 24), k = v.x;
    const int64_t dabs = (int64_t)(((uint64_t)(uint32_t)v.w << 32) | (uint32_t)v.z);
    const int d0 = (int)(dabs - v_off[k]);
    const int n = v_len[k], L = alen[a], D = span[a];
    int lo = max(1, d0 + L - E);
    const int hi = d0 + L + E + 1;
    if (hi > n) {                                    // the band reaches the read end: the last chunk
        lo = min(lo, n);
        const int st = max(0, lo - 1 - D);
        return make_int4(st, n - st, lo - st, -1);
    }
    const int st = max(0, lo - 1 - D);
    return make_int4(st, hi - 1 - st, lo - st, hi - st);
}

// Per adapter its windows (the same count under every chunk length, so k_plan_layout's choice does
// not matter): one atomic per (wave, adapter).
__global__ __launch_bounds__(256) void k_wplan_count(const int4 *vl, const int32_t *vcount, int64_t vcap,
                                                     const int32_t *v_len, const int32_t *start, int32_t *adp_tasks) {
    const int64_t nv = min((int64_t)*vcount, vcap);
    const int lane = threadIdx.x & 63;
    for (int64_t b0 = (int64_t)blockIdx.x * 256; b0 < nv; b0 += (int64_t)gridDim.x * 256) {   // uniform
        const int64_t i = b0 + threadIdx.x;
        const int4 v = i < nv ? vl[i] : make_int4(0, 0, 0, 0);
        const bool active = i < nv && wseed_valid(v, v_len, start);
        const int32_t a = active ? (v.y & 0xFFFFFF) : -1;
        uint64_t pending = __ballot(active);
        while (pending) {                            // wave-uniform
            const int leader = __ffsll((unsigned long long)pending) - 1;
            const int32_t a0 = __shfl(a, leader);
            const bool mine = active && a == a0;
            const int sum = wave_sum(mine ? 1 : 0);
            if (lane == leader)
                for (int c = 0; c < kPlanC; ++c) atomicAdd(&adp_tasks[a0 * kPlanC + c], sum);
            pending &= ~__ballot(mine);
        }
    }
}

// The window task slots (k_plan_place's layout: adapter a's tasks from wave_off[a] * 64), the
// candidate of each from the pair map k_cands wrote (pmap, row stride n).
__global__ __launch_bounds__(256) void k_wplan_place(const int4 *vl, const int32_t *vcount, int64_t vcap,
                                                     const int64_t *v_off, const int32_t *v_len, const int32_t *start,
                                                     const int32_t *alen, const int32_t *span, const int32_t *pmap,
                                                     int64_t n, const int64_t *wave_off, int32_t *fill, int32_t *tw,
                                                     int32_t *to, int4 *tck, int32_t *tcand, const int64_t *slots_dev) {
    const int64_t nv = min((int64_t)*vcount, vcap);
    const int64_t slots = *slots_dev;
    const int lane = threadIdx.x & 63;
    for (int64_t b0 = (int64_t)blockIdx.x * 256; b0 < nv; b0 += (int64_t)gridDim.x * 256) {   // uniform
        const int64_t i = b0 + threadIdx.x;
        const int4 v = i < nv ? vl[i] : make_int4(0, 0, 0, 0);
        const bool active = i < nv && wseed_valid(v, v_len, start);
        const int32_t a = active ? (v.y & 0xFFFFFF) : -1;
        int64_t q = 0;
        uint64_t pending = __ballot(active);
        while (pending) {                            // wave-uniform: one atomic per (wave, adapter)
            const int leader = __ffsll((unsigned long long)pending) - 1;
            const int32_t a0 = __shfl(a, leader);
            const bool mine = active && a == a0;
            const int x = mine ? 1 : 0;
            const int incl = wave_incl_scan(x);
            const int total = __shfl(incl, 63);
            int b1 = 0;
            if (lane == leader) b1 = atomicAdd(&fill[a0], total);
            b1 = __shfl(b1, leader);
            if (mine) q = wave_off[a0] * 64 + b1 + (incl - x);
            pending &= ~__ballot(mine);
        }
        if (!active || q >= slots) continue;
        tw[q] = v.x;
        to[q] = (int32_t)q;
        tck[q] = wseed_chunk(v, v_off, v_len, alen, span);
        tcand[q] = pmap[(int64_t)a * n + v.x];
    }
}

// Merge key of a task: larger score first, then the earlier chunk. Chunks are told apart by their
// first owned column (start + own_lo, unique per chunk), not by their start: near the read
// start several chunks begin at offset 0.
__device__ __forceinline__ uint64_t merge_key(int32_t score, int4 ck) {
    return ((uint64_t)((uint32_t)score ^ 0x80000000u) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)(ck.x + ck.z));
}

// A candidate's chunk tasks sit in consecutive slots, so a wave's lanes mostly share a few
// candidates: a segmented max over each run of equal candidates (shuffles) leaves one atomic per
// run instead of one per task (64 same-address atomics per wave serialised: ~48 us of round 1).
__global__ __launch_bounds__(256) void k_merge_best(const int32_t *tw, const int4 *tck, const int32_t *tcand,
                                                    const int32_t *res, int64_t slots, const int64_t *slots_dev,
                                                    unsigned long long *best) {
    const int64_t ns = slots_dev ? *slots_dev : slots;
    const int lane = threadIdx.x & 63;
    for (int64_t b0 = (int64_t)blockIdx.x * 256; b0 < ns; b0 += (int64_t)gridDim.x * 256) {   // block-uniform
        const int64_t q = b0 + threadIdx.x;
        const bool live = q < ns && tw[q] >= 0;
        const int32_t cand = live ? tcand[q] : -1 - lane;           // idle lanes: runs of their own
        unsigned long long key = live ? (unsigned long long)merge_key(res[4 * slots + q], tck[q]) : 0ull;
        const int32_t prev = __shfl_up(cand, 1);
        const uint64_t heads = __ballot(lane == 0 || prev != cand);
        const int start = 63 - __clzll(heads & ((2ull << lane) - 1ull));   // this lane's run head
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long o = __shfl_up(key, d);
            if (lane - d >= start) key = key > o ? key : o;
        }
        const bool tail = lane == 63 || ((heads >> (lane + 1)) & 1ull);
        if (live && tail) atomicMax(&best[cand], key);
    }
}

// The candidate windows' certificate, per window slot that holds its candidate's best (k_merge_best):
// only a winner that is a hit (full identity not below the threshold) needs one. If the whole
// read's best alignment A* were a hit, it would have an exact piece and stay in its band, so it
// would be in a window and be the windows' winner; so a winner that is no hit proves the pair has
// no hit. A winner that is a hit is the whole read's best when its score is above U[a] (pcabi_seed
// cert_bounds: every alignment without an exact piece, or with more gap columns than the band
// allows, scores at most U[a]; U[a] >= T - 1). Otherwise the candidate is flagged (cmask 1, its
// window best dropped) and its whole read runs in chunks. Block 0 also clears the plan counters for
// that second plan.
__global__ __launch_bounds__(256) void k_certify(const int64_t *cand, const int32_t *tw, const int4 *tck,
                                                 const int32_t *tcand, const int32_t *res, int64_t slots,
                                                 const int64_t *slots_dev, double thr, const int32_t *U,
                                                 unsigned long long *best, int32_t *cmask, int32_t *adp_tasks,
                                                 int32_t *fill, int32_t n_adp) {
    if (blockIdx.x == 0) {
        for (int i = threadIdx.x; i < n_adp * kPlanC; i += 256) adp_tasks[i] = 0;
        for (int i = threadIdx.x; i < n_adp; i += 256) fill[i] = 0;
    }
    const int64_t ns = *slots_dev;
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < ns; q += (int64_t)gridDim.x * 256) {
        if (tw[q] < 0) continue;
        const int32_t ci = tcand[q];
        const int32_t score = res[4 * slots + q];
        if ((unsigned long long)merge_key(score, tck[q]) != best[ci]) continue;
        const int rs = res[0 * slots + q];
        const double full = rs == -1 ? 0.0 : pcabi::pid6(res[5 * slots + q], res[7 * slots + q]);
        if (full < thr) continue;                    // no hit: the pair has none (NaN is a hit, as k_merge_hit)
        if (score > U[(int32_t)(cand[ci] >> 32)]) continue;
        cmask[ci] = 1;
        best[ci] = 0ull;
    }
}

// pass 0: per window the smallest adapter whose winning chunk reaches the threshold (atomicMin);
// pass 1: that candidate writes the window's hit (rs / re back to whole-window offsets).
// slots: the result rows' stride; slots_dev: the live slots (nullptr: all).
__global__ __launch_bounds__(256) void k_merge_hit(const int64_t *cand, const int32_t *tw, const int4 *tck,
                                                   const int32_t *tcand, const int32_t *res, int64_t slots,
                                                   const int64_t *slots_dev, const unsigned long long *best, double thr,
                                                   int pass, int32_t *hit_a, int32_t *hb, int64_t n,
                                                   const int32_t *cmask, int want) {
    const int64_t ns = slots_dev ? *slots_dev : slots;
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < ns; q += (int64_t)gridDim.x * 256) {
        if (tw[q] < 0) continue;
        const int32_t ci = tcand[q];
        if (cmask && cmask[ci] != want) continue;    // (candidate windows: this plan does not decide it)
        const int4 ck = tck[q];
        const int32_t st = ck.x;
        if ((unsigned long long)merge_key(res[4 * slots + q], ck) != best[ci]) continue;
        const int rs = res[0 * slots + q];
        const int m = res[5 * slots + q], l2 = res[7 * slots + q];
        const double full = rs == -1 ? 0.0 : pcabi::pid6(m, l2);
        if (full < thr) continue;                    // NaN goes on, as the reference's loop
        const int32_t k = tw[q], a = (int32_t)(cand[ci] >> 32);
        if (pass == 0) {
            atomicMin(&hit_a[k], a);
        } else if (hit_a[k] == a) {
            hb[0 * n + k] = a;
            hb[1 * n + k] = rs + st;
            hb[2 * n + k] = res[1 * slots + q] + st;
            hb[3 * n + k] = m;
            hb[4 * n + k] = l2;
        }
    }
}

// The windows that hit, compacted (window, adapter, rs, re, m, l2), in any order.
__global__ __launch_bounds__(256) void k_hits_compact(const int32_t *hb, int64_t n, int32_t *out,
                                                      unsigned int *cnt) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n || hb[k] < 0) return;
    const unsigned int j = atomicAdd(cnt, 1u);
    int32_t *o = out + 6 * (int64_t)j;
    o[0] = (int32_t)k;
#pragma unroll
    for (int f = 0; f < 5; ++f) o[1 + f] = hb[f * n + k];
}


// ---- queued middle-scan rounds (middle_device_rounds): the kernels between the seeded plan's ------
// steps, every count read on the device

// Start of a round: views of its windows (sub[k] = window cur[k], k < n_dev; cur == nullptr: none,
// round 1 reads the windows themselves) and the round's counters zeroed -- the next round's read
// count, the plan flag, the plan's per-adapter task counts (n_adp x kPlanC) and fill counters.
// n_first != nullptr (round 1): its read count, n_first_val, is written too.
__global__ __launch_bounds__(256) void k_round_views(const int64_t *win_off, const int32_t *win_len, const int32_t *cur,
                                                     const int32_t *n_dev, int64_t *sub_off, int32_t *sub_len,
                                                     int32_t *n_next, int32_t *plan_flag, int32_t *ptasks,
                                                     int32_t *pfill, int32_t n_adp, int32_t *n_first,
                                                     int32_t n_first_val) {
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            *n_next = 0;
            *plan_flag = 0;
            if (n_first) *n_first = n_first_val;
        }
        for (int i = threadIdx.x; i < n_adp * kPlanC; i += 256) ptasks[i] = 0;
        for (int i = threadIdx.x; i < n_adp; i += 256) pfill[i] = 0;
    }
    if (!cur) return;
    const int64_t n = *n_dev;
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256) {
        sub_off[k] = win_off[cur[k]];
        sub_len[k] = win_len[cur[k]];
    }
}

// Before the merges: the candidates' best keys zeroed (k < *n_cand), the round's per-window hit
// adapter (INT32_MAX) and hit table row 0 (-1) reset (k < *n_dev).
__global__ __launch_bounds__(256) void k_merge_reset(unsigned long long *best, const unsigned long long *n_cand, int64_t cap,
                                                     int32_t *hit_a, int32_t *hb, const int32_t *n_dev,
                                                     int32_t *cmask) {
    const int64_t nc = min((int64_t)*n_cand, cap), nr = *n_dev;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nc; i += (int64_t)gridDim.x * 256) {
        best[i] = 0ull;
        if (cmask) cmask[i] = 0;
    }
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < nr; k += (int64_t)gridDim.x * 256) {
        hit_a[k] = INT32_MAX;
        hb[k] = -1;
    }
}

// Profile counters (pcabi_scan_profile): a round's reads and bases, and a plan's tasks and DP cells
// (columns x adapter rows; a whole-window task, chunk (0, 0, 0, 0), computes its window).
__global__ __launch_bounds__(256) void k_prof_round(const int32_t *v_len, const int32_t *n_dev, unsigned long long *out) {
    const int64_t n = *n_dev;
    unsigned long long b = 0;
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256) b += (uint32_t)v_len[k];
    for (int d = 32; d > 0; d >>= 1) b += __shfl_xor(b, d);
    if ((threadIdx.x & 63) == 0) atomicAdd(&out[1], b);
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&out[0], (unsigned long long)n);
}

__global__ __launch_bounds__(256) void k_prof_cells(const int32_t *tw, const int4 *tck, const int32_t *tcand,
                                                    const int64_t *cand, const int32_t *v_len, const int32_t *alen,
                                                    const int64_t *slots_dev, unsigned long long *out) {
    const int64_t ns = *slots_dev;
    unsigned long long t = 0, c = 0;
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < ns; q += (int64_t)gridDim.x * 256) {
        const int32_t k = tw[q];
        if (k < 0) continue;
        const int4 ck = tck[q];
        const int32_t a = (int32_t)(cand[tcand[q]] >> 32);
        const int cols = (ck.x | ck.y | ck.z | ck.w) ? ck.y : v_len[k];
        t += 1;
        c += (unsigned long long)cols * (uint32_t)alen[a];
    }
    for (int d = 32; d > 0; d >>= 1) {
        t += __shfl_xor(t, d);
        c += __shfl_xor(c, d);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&out[2], t);
        atomicAdd(&out[3], c);
    }
}

// The device plan's layout (device_plan_hits' host part, on the device, one block): per bucket
// the longest chunk length whose waves reach `target` (else the shortest), every adapter's wave
// offset (buckets in order, a bucket's adapters in order, one adapter per wave), the wave ->
// bucket-local adapter table, the idle lanes of every adapter's last wave (task -1), and per
// bucket (first wave, waves). More slots than slots_cap: flag, need = the slots, no waves.
//   bk_first[n_bk + 1]: the buckets' ranges of bk_adp (global adapter ids) / bk_local (their
//   index in the bucket's table); tasks[a * kPlanC + c]: k_plan_count's counts.
__global__ __launch_bounds__(256) void k_plan_layout(const int32_t *tasks, int32_t n_bk, const int32_t *bk_first,
                                                     const int32_t *bk_adp, const int32_t *bk_local, int64_t target,
                                                     int64_t slots_cap, int32_t *cidx, int64_t *woff, int32_t *wa,
                                                     int32_t *tw, int32_t *bk_waves, int64_t *slots_total,
                                                     int32_t *flag, int64_t *need) {
    typedef hipcub::BlockScan<long long, 256> Scan;
    __shared__ typename Scan::TempStorage scan_tmp;
    __shared__ unsigned long long s_w[kNumBuckets][kPlanC];
    __shared__ int s_bc[kNumBuckets];
    __shared__ long long s_carry;
    const int32_t n_all = bk_first[n_bk];
    for (int i = threadIdx.x; i < kNumBuckets * kPlanC; i += 256) s_w[i / kPlanC][i % kPlanC] = 0;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    auto bucket_of = [&](int32_t j) {
        int32_t b = 0;
        while (b + 1 < n_bk && bk_first[b + 1] <= j) ++b;
        return b;
    };
    // per bucket the waves of each chunk length; the longest length whose waves reach the target
    for (int32_t j = threadIdx.x; j < n_all; j += 256) {
        const int32_t a = bk_adp[j], b = bucket_of(j);
#pragma unroll
        for (int c = 1; c < kPlanC; ++c) atomicAdd(&s_w[b][c], (unsigned long long)((tasks[a * kPlanC + c] + 63) / 64));
    }
    __syncthreads();
    for (int32_t b = threadIdx.x; b < n_bk; b += 256) {
        int bc = 0;
        for (int c = kPlanC - 1; c > 0; --c)
            if ((int64_t)s_w[b][c] >= target) {
                bc = c;
                break;
            }
        s_bc[b] = bc;
    }
    __syncthreads();
    // wave offsets: an exclusive scan over the adapters (buckets in order, a bucket's in order)
    for (int32_t j0 = 0; j0 < n_all; j0 += 256) {      // block-uniform
        const int32_t j = j0 + threadIdx.x;
        long long w = 0;
        int32_t a = -1, b = 0;
        if (j < n_all) {
            a = bk_adp[j];
            b = bucket_of(j);
            cidx[a] = s_bc[b];
            w = (tasks[a * kPlanC + s_bc[b]] + 63) / 64;
        }
        long long ex, tot;
        Scan(scan_tmp).ExclusiveSum(w, ex, tot);
        ex += s_carry;
        if (a >= 0) woff[a] = ex;
        __syncthreads();
        if (threadIdx.x == 0) s_carry += tot;
        __syncthreads();
    }
    const int64_t slots = s_carry * 64;
    for (int32_t b = threadIdx.x; b < n_bk; b += 256) {
        const int64_t lo = bk_first[b] < n_all ? woff[bk_adp[bk_first[b]]] : s_carry;
        const int64_t hi = bk_first[b + 1] < n_all ? woff[bk_adp[bk_first[b + 1]]] : s_carry;
        bk_waves[2 * b] = (int32_t)lo;
        bk_waves[2 * b + 1] = slots > slots_cap ? 0 : (int32_t)(hi - lo);
    }
    if (slots > slots_cap) {                         // too small: no waves, the round reruns larger
        if (threadIdx.x == 0) {
            *flag = 1;
            *need = slots;
            *slots_total = 0;
        }
        return;
    }
    if (threadIdx.x == 0) *slots_total = slots;
    // the wave -> bucket-local adapter table and the idle lanes of every adapter's last wave: one
    // wave per adapter
    const int lane = threadIdx.x & 63;
    for (int32_t j = threadIdx.x >> 6; j < n_all; j += 4) {
        const int32_t a = bk_adp[j];
        const int32_t nt = tasks[a * kPlanC + cidx[a]];
        const int64_t nw = (nt + 63) / 64, w0 = woff[a];
        for (int64_t w = lane; w < nw; w += 64) wa[w0 + w] = bk_local[j];
        const int64_t t = nt + lane;
        if (t < nw * 64) tw[w0 * 64 + t] = -1;
    }
}

// A round's hits (k_merge_hit's per-window table hb, row stride n) -> the round's list (8 int32
// each: read, adapter, rs, re, m, l2, position, 0), the next round's reads (those that hit, from
// the adapter that hit) and their count. A round whose seed / plan buffers overflowed keeps nothing
// (no hits, no next round, no masking): the host sees rflag and reruns it with larger buffers.
// (r04) The list is an ORDERED compaction -- a round's hits in the order of its reads, which round
// 1 takes in read order -- so every round's list is sorted by read and the host concatenates the
// rounds without sorting (an indirect std::sort of ~5 k hits cost ~0.1-0.4 ms of host time per
// call). k_round_count counts each 256-entry chunk's hits; a chunk's base is the sum of the counts
// before it (summed by the block: a few hundred chunks), its hits' places a block scan.
__global__ __launch_bounds__(256) void k_round_count(const int32_t *hb, const int32_t *n_dev, const int32_t *seed_flags,
                                                     const int32_t *plan_flag, int32_t *counts) {
    if (seed_flags[0] || seed_flags[1] || *plan_flag) return;
    const int64_t nr = *n_dev, nch = (nr + 255) / 256;
    for (int64_t c = blockIdx.x; c < nch; c += gridDim.x) {   // block-uniform
        const int64_t k = c * 256 + threadIdx.x;
        const int cnt = __syncthreads_count(k < nr && hb[k] >= 0);
        if (threadIdx.x == 0) counts[c] = cnt;
    }
}

// (r05) A read's first masked hit also takes its shadow-arena space here (k_mask_list copies it):
// one atomic per block over the block's scanned sizes; o[7] = 1 + the 16-byte unit it starts at.
__global__ __launch_bounds__(256) void k_round_hits(const int32_t *hb, int64_t n, const int32_t *n_dev, const int32_t *cur,
                                                    const int32_t *counts, int32_t *list, int32_t *n_next,
                                                    int32_t *cur_next, int32_t *start_next, const int32_t *seed_flags,
                                                    const int32_t *plan_flag, int32_t *rflag, const int64_t *win_off,
                                                    const int64_t *eoff, const int32_t *win_len,
                                                    unsigned long long *bump) {
    typedef hipcub::BlockScan<int, 256> Scan;
    typedef hipcub::BlockScan<long long, 256> Scan64;
    __shared__ typename Scan::TempStorage scan_tmp;
    __shared__ typename Scan64::TempStorage scan64_tmp;
    __shared__ unsigned long long s_at;
    __shared__ int s_part[4];
    const int32_t f = (seed_flags[0] ? 1 : 0) | (seed_flags[1] ? 2 : 0) | (*plan_flag ? 4 : 0);
    if (blockIdx.x == 0 && threadIdx.x == 0) *rflag = f;
    if (f) return;
    const int64_t nr = *n_dev, nch = (nr + 255) / 256;
    for (int64_t c = blockIdx.x; c < nch; c += gridDim.x) {   // block-uniform
        int part = 0;                                          // hits of the chunks before c
        for (int64_t i = threadIdx.x; i < c; i += 256) part += counts[i];
        for (int d = 32; d > 0; d >>= 1) part += __shfl_xor(part, d);
        if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = part;
        __syncthreads();
        const int base = s_part[0] + s_part[1] + s_part[2] + s_part[3];
        const int64_t k = c * 256 + threadIdx.x;
        const int32_t a = k < nr ? hb[k] : -1;
        int pos = 0, tot = 0;
        Scan(scan_tmp).ExclusiveSum(a >= 0 ? 1 : 0, pos, tot);
        const int32_t r = a >= 0 ? (cur ? cur[k] : (int32_t)k) : 0;
        const int32_t rs = a >= 0 ? hb[1 * n + k] : -1, re = a >= 0 ? hb[2 * n + k] : 0;
        // shadow space (16-byte units) of a first masked hit
        long long units = 0;
        if (a >= 0 && rs != -1 && re + 1 > rs && eoff[r] == win_off[r]) units = shadow_bytes(win_len[r]) / 16;
        long long uex = 0, utot = 0;
        Scan64(scan64_tmp).ExclusiveSum(units, uex, utot);
        if (threadIdx.x == 0) s_at = utot ? atomicAdd(bump, (unsigned long long)utot * 16ull) : 0ull;
        __syncthreads();
        if (a >= 0) {
            const int32_t j = base + pos;
            int32_t *o = list + 8 * (int64_t)j;
            o[0] = r;
            o[1] = a;
            o[2] = rs;
            o[3] = re;
            o[4] = hb[3 * n + k];
            o[5] = hb[4 * n + k];
            o[6] = (int32_t)k;
            const long long at = (long long)(s_at / 16ull) + uex;   // a unit index; < 2^31 (checked by the host's cap)
            o[7] = units ? (int32_t)min(at + 1, (long long)INT32_MAX) : 0;
            cur_next[j] = r;
            start_next[j] = a;
        }
        if (c == nch - 1 && threadIdx.x == 0) *n_next = base + tot;
        __syncthreads();                                       // s_part, scan_tmp reused
    }
}

// The reads with their end adapters trimmed (nanopore_read.py:44-49,
// get_seq_with_start_end_adapters_trimmed): view = [start_trim, len - end_trim), empty when the
// trims meet.
__global__ __launch_bounds__(256) void k_trim_views(const int64_t *read_off, const int32_t *read_len,
                                                    const int32_t *start_trim, const int32_t *end_trim, int64_t n,
                                                    int64_t *view_off, int32_t *view_len) {
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256) {
        const int32_t st = start_trim[k];
        view_off[k] = read_off[k] + st;
        view_len[k] = max(read_len[k] - st - end_trim[k], 0);
    }
}

// ---- launch plumbing -------------------------------------------------------------------------

// Tile layout of a window list (cross mode): windows [256t, 256t + 256) form tile t; dword
// (t, q, lane) = codes 4q..4q+3 of window 256t + lane, at tiles[tile_off[t] + 256q + lane].
// Zero past each window's end. Thread = window: it loads its window's 64-byte slab (17 dwords,
// independent loads, any offset: a byte funnel shift) and writes its 16 dwords down the tile's
// rows, so every row store of a wave is 256 contiguous bytes. (r01-r05: 16 threads per window and
// an LDS transpose, each thread 16 dependent load chains in turn: 25 us per 100k 150-bp windows.)
// grid (n_tiles, <= 1024): blockIdx.y strides over 16-chunk slabs.
__global__ __launch_bounds__(256) void k_tile_windows(const uint8_t *codes, const int64_t *win_off,
                                                      const int32_t *win_len, int64_t n_win,
                                                      const int64_t *tile_off, uint32_t *tiles) {
    const int64_t t = blockIdx.x;
    const int64_t base = tile_off[t];
    const int64_t nq = (tile_off[t + 1] - base) / 256;
    const int64_t w = t * 256 + threadIdx.x;
    int64_t n = 0;
    const uint8_t *wb = codes;
    if (w < n_win) {
        n = max(win_len[w], 0);
        wb = codes + win_off[w];
    }
    for (int64_t q0 = (int64_t)blockIdx.y * 16; q0 < nq; q0 += (int64_t)gridDim.y * 16) {
        const int64_t c0 = 4 * q0;
        const int64_t avail = n - c0;                 // window bytes from column c0 on
        const uint8_t *b = wb + c0;
        const int sh = (int)((uintptr_t)b & 3);
        const uint32_t *q = reinterpret_cast<const uint32_t *>(b - sh);
        uint32_t d[17];
#pragma unroll
        for (int k = 0; k < 17; ++k) d[k] = (avail > 0 && 4 * k < avail + sh) ? q[k] : 0u;   // dwords holding window bytes
        const int nqq = (int)std::min<int64_t>(16, nq - q0);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (k >= nqq) break;
            uint32_t v = sh ? __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh) : d[k];
            const int64_t rem = avail - 4 * k;
            v = rem >= 4 ? v : (rem > 0 ? v & ((1u << (8 * rem)) - 1u) : 0u);
            tiles[base + (q0 + k) * 256 + threadIdx.x] = v;
        }
    }
}

int64_t tile_layout(const int32_t *win_len, int64_t n_win, int64_t *tile_off, int64_t *max_nq) {
    const int64_t n_tiles = (n_win + 255) / 256;
    int64_t off = 0, mq = 0;
    for (int64_t t = 0; t < n_tiles; ++t) {
        int32_t mx = 0;
        for (int64_t w = t * 256; w < std::min<int64_t>(n_win, t * 256 + 256); ++w) mx = std::max(mx, win_len[w]);
        const int64_t nq = (mx + 3) / 4 + 2;   // + the reader's one-chunk-ahead fetch
        tile_off[t] = off;
        off += nq * 256;
        mq = std::max(mq, nq);
    }
    tile_off[n_tiles] = off;
    if (max_nq) *max_nq = mq;
    return off;
}

void launch_tiles(const uint8_t *codes, const int64_t *win_off, const int32_t *win_len, int64_t n_win,
                  const int64_t *tile_off, int64_t max_nq, uint32_t *tiles, hipStream_t st) {
    const int64_t n_tiles = (n_win + 255) / 256;
    if (n_tiles == 0) return;
    const dim3 grid((unsigned)n_tiles, (unsigned)std::min<int64_t>(std::max<int64_t>((max_nq + 15) / 16, 1), 1024));
    hipLaunchKernelGGL(k_tile_windows, grid, dim3(256), 0, st, codes, win_off, win_len, n_win, tile_off, tiles);
}

// Buckets the chunked candidate DP serves: the packed core's (FAST buckets laid out packed, WIDE)
// and the generic and striped cores' (long adapters).
bool chunkable(int b, bool packed) {
    return kBuckets[b].kind == WIDE || kBuckets[b].kind == LONG || kBuckets[b].kind == GENERIC ||
           kBuckets[b].kind == STRIPED || (kBuckets[b].kind == FAST && packed);
}

// Lanes per window of the row-split core (k_align_split) for a cross-mode launch of `waves`
// waves: 4 (2 under 16 rows) for launches under 1024 waves, else 1 (the one-lane core).
// PCABI_SPLIT=0 turns the split off, 2 / 4 force it (tests: the split core on any launch). The split costs ~1.3-1.7x the VALU work per
// cell (the per-step exchange and bookkeeping over R / K rows), so it pays only where a launch is
// latency-bound on its own: r04 A/B (profiles/r04/split_ab/), a threshold of 4096 waves split the
// headline's one-adapter buckets (1,564 waves), which run beside the other side's buckets anyway:
// 7.78 -> 7.98 ms per step; the set search of 10k reads (156 waves per adapter) gained 2.79 ->
// 2.53 ms.
int split_lanes(int rpl, int64_t waves) {
    const char *e = std::getenv("PCABI_SPLIT");
    const int forced = (e && e[0]) ? std::atoi(e) : -1;
    int K = 1;
    if (forced >= 0) K = forced;
    else if (waves < 1024) K = rpl < 16 ? 2 : 4;
    return (K == 2 || K == 4) && pcabi::split_ok(rpl, K) ? K : 1;
}

// packed: bucket_pack_mode (0 untagged cores off, 1 packed key layout, 2 run-tagged layout)
int dispatch(int b, const KParams &p, bool affine, hipStream_t st, int packed) {
    if (kBuckets[b].kind == STRIPED) return launch_striped(p, affine, st);
    const int64_t tiles8 = (p.n_win + 8 * 256 - 1) / (8 * 256) * 8;   // window tiles, padded to 8
    dim3 grid = p.task_win ? dim3((unsigned)((p.n_waves + 3) / 4))
                           : dim3((unsigned)(tiles8 * p.n_adp));
    const BucketDef d = kBuckets[b];
    if (!p.task_win && !p.compat && packed && d.kind == FAST && d.rpl <= 64) {
        // a launch too small to fill the chip: K lanes per window (pcabi_dp.h LaneSplit)
        const int K = split_lanes(d.rpl, (p.n_win + 255) / 256 * 4 * (int64_t)p.n_adp);
        if (K > 1 && dispatch_split(d.rpl, K, p, affine, packed == 2, st)) return 0;
    }
    if (d.kind == LONG || d.kind == WIDE || (d.kind == FAST && packed && d.rpl > 32))
        dispatch_packed_large(d.rpl, d.kind == LONG, p, affine, grid, st);
    else if (d.kind == FAST && packed)
        dispatch_packed_small(d.rpl, p, affine, grid, st, packed == 2);
    else
        dispatch_fast(d.rpl, d.kind == GENERIC, p, affine, grid, st);
    return 0;
}

// Packed-key kernels serve a fast bucket when every adapter in it satisfies the range
// conditions of pcabi_dp.h packed_ok (any window length).
bool bucket_packed_ok(int b, const std::vector<int32_t> &lens, const pcabi::Scoring &sc) {
    if (kBuckets[b].kind == WIDE || kBuckets[b].kind == LONG) return true;   // assigned only when packed_ok / long_ok holds
    if (kBuckets[b].kind != FAST || kBuckets[b].rpl > pcabi::pk::MAX_RPL) return false;
    for (int32_t L : lens)
        if (!pcabi::packed_ok(L, kBuckets[b].rpl, sc)) return false;
    return true;
}

// How k_align serves a bucket: 0 = not packed (fast / generic cores), 1 = packed key layout,
// 2 = the run-tagged layout (pcabi_dp.h pk::LayT: affine buckets of <= 32 rows whose adapters all
// pass layt_ok; one VALU op per cell less).
int bucket_pack_mode(int b, const std::vector<int32_t> &lens, const pcabi::Scoring &sc) {
    if (!bucket_packed_ok(b, lens, sc)) return 0;
    if (kBuckets[b].kind != FAST || kBuckets[b].rpl > 32) return 1;
    for (int32_t L : lens)
        if (!pcabi::layt_ok(L, kBuckets[b].rpl, sc)) return 1;
    return 2;
}

// Host-side layout of a bucket's adapter table.
struct BucketHost {
    std::vector<uint8_t> pad;   // n * RPL bytes (striped: n * rt)
    std::vector<int32_t> len, id;
    int rt = 0;                 // striped: table rows per adapter
};

// At most this many FAST buckets per adapter table: a cross product launches its buckets side by
// side (the caller's stream + SideStreams::N), and a bucket of one or two adapters is too small
// a grid to fill the GPU on its own.
constexpr int kMaxFastBuckets = 4;

// Bucket of every adapter: its own register bucket, then the cheapest merges of a FAST bucket
// into the next larger non-empty one (cost = adapters x added padding rows) until at most
// kMaxFastBuckets remain. Only merges the packed core can serve with the scoring `sc` (it
// passes scores through any number of padding rows; the fast core allows at most 3).
// all_striped: every adapter on the striped core (needs_striped: long windows under a scoring
// with no path-span bound).
std::vector<int> assign_buckets(const int32_t *adp_len, int32_t n_adp, const pcabi::Scoring &sc, bool merge,
                                bool allow_wide, bool all_striped = false) {
    std::vector<int> b_of(n_adp);
    int count[kNumBuckets] = {};
    for (int a = 0; a < n_adp; ++a) {
        b_of[a] = all_striped ? kStripedBucket : bucket_of(adp_len[a], sc, allow_wide);
        ++count[b_of[a]];
    }
    if (all_striped) return b_of;
    auto packed_all = [&](int b, int extra_from) {
        for (int a = 0; a < n_adp; ++a)
            if ((b_of[a] == b || b_of[a] == extra_from) && !pcabi::packed_ok(adp_len[a], kBuckets[b].rpl, sc))
                return false;
        return true;
    };
    const int max_fast = kMaxFastBuckets;
    while (merge) {
        std::vector<int> fast;
        for (int b = 0; b < kNumBuckets; ++b)
            if (count[b] && kBuckets[b].kind == FAST) fast.push_back(b);
        if ((int)fast.size() <= max_fast) break;
        int best = -1;
        int64_t best_cost = 0;
        for (size_t k = 0; k + 1 < fast.size(); ++k) {
            const int i = fast[k], j = fast[k + 1];
            // more than 3 padding rows: only the packed core passes scores through them
            if (!packed_all(j, i)) continue;
            const int64_t cost = (int64_t)count[i] * (kBuckets[j].rpl - kBuckets[i].rpl);
            if (best < 0 || cost < best_cost) { best = (int)k; best_cost = cost; }
        }
        if (best < 0) break;
        const int i = fast[best], j = fast[best + 1];
        for (int a = 0; a < n_adp; ++a)
            if (b_of[a] == i) b_of[a] = j;
        count[j] += count[i];
        count[i] = 0;
    }
    return b_of;
}

void build_buckets(const uint8_t *adp_codes, const int32_t *adp_off, const int32_t *adp_len,
                   int32_t n_adp, const pcabi::Scoring &sc, BucketHost (&bk)[kNumBuckets], bool merge = true,
                   bool allow_wide = true, bool all_striped = false) {
    const std::vector<int> b_of = assign_buckets(adp_len, n_adp, sc, merge, allow_wide, all_striped);
    for (int a = 0; a < n_adp; ++a)
        if (b_of[a] == kStripedBucket)
            bk[kStripedBucket].rt = std::max(bk[kStripedBucket].rt, (adp_len[a] + kStripeTab - 1) / kStripeTab * kStripeTab);
    for (int a = 0; a < n_adp; ++a) {
        const int L = adp_len[a];
        const int b = b_of[a];
        const int R = b == kStripedBucket ? bk[b].rt : kBuckets[b].rpl;
        BucketHost &h = bk[b];
        const size_t base = h.pad.size();
        h.pad.resize(base + R, (uint8_t)pcabi::PAD_CODE);
        const int off = R - L;
        for (int k = 0; k < L; ++k) h.pad[base + off + k] = adp_codes[adp_off[a] + k];
        h.len.push_back(L);
        h.id.push_back(a);
    }
}

}  // namespace

// error channel shared with the host I/O unit (csrc/pcabi_io.cpp)
namespace pcabi_internal {
int fail(int code, const std::string &msg) { return pcabi_eng::fail(code, msg); }
}  // namespace pcabi_internal

// ---- prepared adapter tables (device) ---------------------------------------------------------
std::atomic<uint64_t> g_table_serial{0};
struct pcabi_adapters {
    int32_t n_adp = 0;
    // a process-unique number (a new table may reuse a freed one's address): what the middle scan's
    // captured round graphs are keyed on, since they hold the table's device pointers
    uint64_t serial = g_table_serial.fetch_add(1) + 1;
    int rt[kNumBuckets] = {};        // striped bucket: table rows per adapter
    bool padded[kNumBuckets] = {};
    int max_off[kNumBuckets] = {};   // most padding rows above an adapter (> 3: packed core only)
    std::vector<int32_t> lens[kNumBuckets];
    std::vector<int32_t> ids[kNumBuckets];   // global adapter index of each bucket entry (host)
    bool has_n = false;                      // some adapter holds an N (code 4) base
    std::vector<uint8_t> hcodes;             // host copy of the adapters (middle-scan seeds)
    std::vector<int32_t> hoff, hlen;
    int32_t count[kNumBuckets] = {};
    uint32_t *pad[kNumBuckets] = {};
    int32_t *len[kNumBuckets] = {};
    int32_t *id[kNumBuckets] = {};
    // Other layouts of the same adapters, built on first use by adapters_for() for a scoring this
    // layout cannot serve (gap costs >= 0 under padded register buckets, a merge made for another
    // scoring) or for long windows that need the striped core; kept until the table is destroyed
    // (launches queued on a stream may still read them).
    std::mutex alt_mu;
    std::vector<std::pair<pcabi::Scoring, pcabi_adapters *>> alt_scored;
    pcabi_adapters *alt_striped = nullptr;
};

namespace {

}  // namespace
// Bumped by every device (re)allocation of the engine's and the seeds' scratch and by every new
// seed plan: a captured round graph (middle_device_rounds) holds their addresses and launch
// arguments, and is replayed only while the generation it was captured at holds.
std::atomic<uint64_t> g_buf_gen{0};

// Debug switch PCABI_POISON: every fresh scratch allocation and every growth (DeviceBuf, the
// seeds' Buf, the shadow arena, the stream-ordered scratch of the epilogues and the striped core)
// is filled with one byte before use, so a kernel or host path that reads scratch nothing wrote
// sees garbage instead of the zeros fresh hipMalloc memory usually holds (the
// r05 `need2` read went unnoticed for that reason). "1" fills 0xFF (every int -1); a hex byte such
// as "0x3f" fills that byte (0x3f: every int32 / int64 a huge positive count whose growth arithmetic
// -- need + need / 4 -- does not overflow; 0x7f wrapped there and hid the r05 need2 read).
int pcabi_poison_byte() {
    static const int b = [] {
        const char *e = std::getenv("PCABI_POISON");
        if (!e || !e[0] || (e[0] == '0' && !e[1])) return -1;
        if (e[0] == '1' && !e[1]) return 0xFF;
        return (int)(std::strtol(e, nullptr, 0) & 0xFF);
    }();
    return b;
}
void pcabi_poison(void *p, size_t bytes) {
    if (pcabi_poison_byte() < 0 || !p || !bytes) return;
    (void)hipMemset(p, pcabi_poison_byte(), bytes);
    (void)hipDeviceSynchronize();
}
void pcabi_poison_async(void *p, size_t bytes, hipStream_t st) {
    if (pcabi_poison_byte() >= 0 && p && bytes) (void)hipMemsetAsync(p, pcabi_poison_byte(), bytes, st);
}
namespace {
struct DeviceBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return 0;
        g_buf_gen.fetch_add(1);
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes, 1 << 16);
        const hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
            return fail(PCABI_E_NOMEM, "hipMalloc failed (" + std::to_string(want) + " bytes): " + hipGetErrorString(e));
        }
        cap = want;
        pcabi_poison(p, want);
        return 0;
    }
};

}  // namespace

// Scratch of the device-resident middle scan (pcabi_middle_scan_dev), grown on demand.
namespace pcabi_seed {   // pcabi_seed.hip
struct State;
State *create();
void destroy(State *s);
int bounds(State *s, const void *adps_key, const uint8_t *hcodes, const int32_t *hoff, const int32_t *hlen,
           int32_t n_adp, const std::vector<int> &fb_rows, const uint8_t *codes, const int64_t *v_off,
           const int32_t *v_len, int64_t n, const pcabi::Scoring &sc, double threshold, int mode, int16_t *s16,
           std::vector<int64_t> *cands, const int64_t **dcands, int64_t *n_dcands, hipStream_t st);
int plan_ready(State *s, const uint8_t *hcodes, const int32_t *hoff, const int32_t *hlen, int32_t n_adp,
               const std::vector<int> &fb_rows, const pcabi::Scoring &sc, double threshold, int mode, hipStream_t st);
int bounds_dev(State *s, const uint8_t *codes, const int64_t *v_off, const int32_t *v_len, int64_t n,
               const int32_t *n_dev, int32_t n_adp, const pcabi::Scoring &sc, const int64_t **dcands,
               const unsigned long long **dcount, const int32_t **flags, const int4 **vlist, const int32_t **vcount,
               const int32_t **pmap, int64_t *vcap, hipStream_t st);
bool grow_after_overflow(State *s, int raw_overflow, int task_overflow);
void shrink_next(State *s, int bits);
void serial_next(State *s);
const int64_t *seg_cum_dev(State *s);
int seg_positions();
void cert_bounds(State *s, std::vector<int32_t> &U);
int debug_counts(State *s, int64_t (&out)[5], hipStream_t st);
void profile_events(State *s, hipEvent_t *ev);
int profile_counts(State *s, int64_t (&out)[3], hipStream_t st);
int profile_band_stats(State *s, bool on);
int band_stats(State *s, unsigned long long (&out)[8]);
int band_e(State *s, int c);
}  // namespace pcabi_seed

// Per-phase profile of the device-resident middle scan (pcabi_scan_profile): events around the
// phases of every queued round, which is then synchronised on its own (a diagnostic pass, never
// the timed one), and the algorithmic units the rounds processed (profile kernels, counters).
enum MidPhase { kPhScan, kPhExpand, kPhBands, kPhCands, kPhPlan, kPhDp, kPhOther, kPhases };
struct MidProf {
    bool on = false;
    std::vector<hipEvent_t> pool;
    size_t used = 0;
    std::vector<std::tuple<int, hipEvent_t, hipEvent_t>> spans;   // this round's (phase, from, to)
    double ms[kPhases] = {};
    int64_t rounds = 0, reads = 0, bases = 0, raw = 0, band_in = 0, band_edge = 0, dp_tasks = 0, dp_cells = 0;
    double round1_ms = 0.0;                                        // round 1's runs (whole rounds)
    // the pinned band classes' work: per class lane-rows issued, active lane-rows, tasks, passes
    unsigned long long band[8] = {};
    hipEvent_t get() {
        if (used == pool.size()) {
            hipEvent_t e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            pool.push_back(e);
        }
        return pool[used++];
    }
    ~MidProf() {
        for (hipEvent_t e : pool) (void)hipEventDestroy(e);
    }
};

struct pcabi_scan {
    const pcabi_adapters *adps = nullptr;
    DeviceBuf tiles, toff, res, hits, idx, start, soff, slen, mwin;
    DeviceBuf s16, tw, to, wa, pres, tck;   // score filter + candidate pairs (chunks)
    DeviceBuf pspan, ptasks, pfill, pwoff, pcidx, pcand, pbest, phit, phb, plist, pcnt, plen;   // device planning
    DeviceBuf tw2, to2, tck2, pcand2, wa2, pres2, pcert, pucert, q_bk2, q_misc2;   // candidate windows' second plan
    pcabi_seed::State *seed = nullptr; // seeded round-1 bounds (pcabi_seed.hip)
    // queued rounds (middle_device_rounds): per round slot the reads, their start adapters and the
    // hit list; round counts and flags; the plan's bucket tables and scratch
    DeviceBuf q_cur, q_start, q_list, q_n, q_flags, q_bk, q_wave, q_misc, pcbase;
    int32_t *h_stage = nullptr;                     // pinned host staging of the queued rounds' hit lists
    size_t h_stage_cap = 0;                         // (int32 elements)
    int32_t *h_ctl = nullptr;                       // pinned: round counts, flags, plan needs of a batch
    int64_t spec_hits = 4096;                       // hits per round copied with the counts (grows to fit)
    double last_mean = 0.0;                         // the previous call's mean read length (round 1)
    int64_t q_slots_cap = 0;
    std::vector<int32_t> h_ucert;                   // the certificate bounds last uploaded to pucert
    std::vector<int32_t> h_up;                      // bucket tables | spans | lengths last uploaded
    const void *up_at[3] = {nullptr, nullptr, nullptr};   // ... into these buffers
    DeviceBuf pcount;                               // k_round_count's per-chunk hit counts
    // (r05) input-preserving masking: the reads' effective offsets and the shadow arena of the
    // masked copies (shadow_cap: its usable bytes), a zeroed bump for the host-driven loop
    DeviceBuf eoff, shadow, shadow_zero;
    int64_t shadow_cap = 0;
    MidProf prof;                                   // pcabi_scan_profile
    DeviceBuf pprof;                                // its device counters (4 x u64)
    // (r05) later rounds replayed from captured graphs, one per round slot: the key is everything
    // a round's launches take by value or address (middle_device_rounds, RoundKey)
    struct RoundGraph {
        std::vector<int64_t> key, seen;     // the captured graph's key; the last key queued directly
        hipGraphExec_t exec = nullptr;
    };
    RoundGraph graphs[32];
    int rounds_hint = 3;                            // rounds the last call needed (the first batch's size)
    uint64_t last_table = 0;                        // the adapter table (serial) of the last call
};

namespace {

// Side streams of a device for the fork / join of pcabi_align_cross_dev's bucket launches. A fork
// region takes its side streams from a rotating start, so two regions queued back to back (the
// headline's two sides, each a cross product on its own caller stream) use different side streams
// and their launches overlap (r04 trace: with 3 shared side streams the end side's small buckets
// queued behind the start side's).
struct SideStreams {
    static constexpr int N = 6;
    std::mutex mu;               // one fork / join region at a time per device
    bool init = false;
    int next = 0;                // the next region's first side stream
    hipStream_t s[N] = {};
    hipEvent_t fork = nullptr, join[N] = {};
};
SideStreams g_side[16];
std::mutex g_side_mu;

int side_streams(int dev, SideStreams **out) {
    if (dev < 0 || dev >= 16) return fail(PCABI_E_ARG, "bad device index");
    std::lock_guard<std::mutex> g(g_side_mu);
    SideStreams &ss = g_side[dev];
    if (!ss.init) {
        // plain streams on the process's GPU_MAX_HW_QUEUES (side streams with a CU mask, a hardware
        // queue each, measured slower in r04n)
        for (int i = 0; i < SideStreams::N; ++i) {
            HIP_TRY(hipStreamCreateWithFlags(&ss.s[i], hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&ss.join[i], hipEventDisableTiming));
        }
        HIP_TRY(hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming));
        ss.init = true;
    }
    *out = &ss;
    return 0;
}

// pcabi_set_side_streams: whether fork / join regions use the side streams (initially on)
constexpr int kSideStreamsDefault = 1;
std::atomic<int> g_side_on{kSideStreamsDefault};
bool side_streams_on() { return g_side_on.load(std::memory_order_relaxed) != 0; }

// Per-stream setting (pcabi_stream_side_streams, r05): a caller that runs cross products on several
// streams at once turns the side streams off for ITS streams only; streams without an entry follow
// the process-wide default (pcabi_set_side_streams).
std::mutex g_stream_side_mu;
std::vector<std::pair<hipStream_t, int>> g_stream_side;   // few entries: a linear scan
bool side_streams_on(hipStream_t st) {
    {
        std::lock_guard<std::mutex> g(g_stream_side_mu);
        for (const auto &e : g_stream_side)
            if (e.first == st) return e.second != 0;
    }
    return side_streams_on();
}

// Fork / join of independent launches: launch k runs on the caller's stream (k == 0) or on side
// stream (first + k - 1) % N, each side stream first waiting for the work already queued on the
// caller's stream; end() makes the caller's stream wait for every side stream used.
struct ForkJoin {
    hipStream_t main = nullptr;
    SideStreams *ss = nullptr;
    std::unique_lock<std::mutex> lock;
    int first = 0;
    unsigned used = 0;           // bit i: side stream i took a launch of this region
    int n_side = 0;              // side launches of this region
    int begin(hipStream_t m, size_t n_launch) {
        main = m;
        if (n_launch <= 1 || !side_streams_on(m)) return 0;  // off: every launch on the caller's stream
        int dev = 0;
        HIP_TRY(hipGetDevice(&dev));
        if (int rc = side_streams(dev, &ss)) return rc;
        lock = std::unique_lock<std::mutex>(ss->mu);
        first = ss->next;
        HIP_TRY(hipEventRecord(ss->fork, main));
        return 0;
    }
    hipStream_t at(size_t k) {
        if (k == 0 || !ss) return main;
        const int i = (int)((first + k - 1) % SideStreams::N);
        if (!(used & (1u << i))) (void)hipStreamWaitEvent(ss->s[i], ss->fork, 0);
        used |= 1u << i;
        n_side = std::max(n_side, (int)k);
        return ss->s[i];
    }
    int end() {
        for (int i = 0; i < SideStreams::N; ++i) {
            if (!(used & (1u << i))) continue;
            HIP_TRY(hipEventRecord(ss->join[i], ss->s[i]));
            HIP_TRY(hipStreamWaitEvent(main, ss->join[i], 0));
        }
        if (ss && n_side) ss->next = (first + n_side) % SideStreams::N;
        used = 0;
        n_side = 0;
        if (lock.owns_lock()) lock.unlock();
        return 0;
    }
};

// Per-device state for the host-buffer API (serialised by a mutex: the legacy ABI is called
// concurrently from the reference's ThreadPool workers, porechop_abi.py:228,418,504).
struct Engine {
    std::mutex mu;
    bool init = false;
    hipStream_t stream = nullptr;
    DeviceBuf codes, woff, wlen, out, tasks_win, tasks_out, wave_adp, tiles, toff, hits, bc;
    pcabi_scan *scan = nullptr;   // scratch of the middle scan (pcabi_middle_scan_host)
    DeviceBuf pad[kNumBuckets], len[kNumBuckets], id[kNumBuckets];
    // pcabi_end_decisions_host: both sides' windows, results, trims, flags and lists; the two
    // sides' prepared adapter tables, kept while the adapters and the scoring stay the same
    DeviceBuf dec[17];
    // pcabi_middle_scan_seqs: pinned staging slots the host strings are encoded into while the
    // previous slots' copies run (allocated on first use, kept)
    uint8_t *stage[4] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t stage_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    DeviceBuf stage_dev;          // the slots' device copies (2-bit codes + N masks), unpacked into place
    struct DTab {
        std::vector<uint8_t> codes;
        std::vector<int32_t> lens;
        pcabi::Scoring sc{0, 0, 0, 0};
        pcabi_adapters *t = nullptr;
    } dtab[2];
};

Engine g_engines[16];

int engine_init(Engine &e, int device) {
    if (e.init) return 0;
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(PCABI_E_DEVICE, std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950");
    HIP_TRY(hipStreamCreateWithFlags(&e.stream, hipStreamNonBlocking));
    e.init = true;
    return 0;
}

int check_common(const int32_t *adp_len, int32_t n_adp) {
    for (int a = 0; a < n_adp; ++a)
        if (adp_len[a] < 1 || adp_len[a] > pcabi::MAX_STRIPED_LEN)
            return fail(PCABI_E_ARG, "adapter length " + std::to_string(adp_len[a]) + " outside 1.." +
                                         std::to_string(pcabi::MAX_STRIPED_LEN));
    return 0;
}

// The register cores keep the path's start column mod 2^16 (pcabi_dp.h attribute word), which
// is exact only when every window is short or the path span is bounded (gap costs < 0). Any
// other scoring the reference accepts (arg_parser.py:229-236: any four integers, e.g. gap costs
// >= 0) on windows of 32 k and more runs on the striped core instead, whose two-word attributes
// never wrap (align_lane_striped): true when that routing is needed.
bool needs_striped(const pcabi::Scoring &sc, int max_L, int64_t max_win) {
    if (max_win < 32768 - 256) return false;
    const int b = pcabi::span_bound(max_L, sc.ma, sc.mi, sc.go, sc.ge);
    return b < 0 || b + max_L >= 32768;
}

}  // namespace

extern "C" {

const char *pcabi_last_error(void) { return g_err.c_str(); }
int pcabi_version(void) { return 1; }
int pcabi_max_adapter_len(void) { return pcabi::MAX_STRIPED_LEN; }
int pcabi_max_window_len(void) { return pcabi::MAX_WINDOW_LEN; }

int pcabi_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void pcabi_encode_dna5(const char *ascii, uint8_t *codes, int64_t n) {
    static const struct Tab {
        uint8_t t[256];
        Tab() {
            for (int c = 0; c < 256; ++c) t[c] = 4;
            t['A'] = t['a'] = 0;
            t['C'] = t['c'] = 1;
            t['G'] = t['g'] = 2;
            t['T'] = t['t'] = t['U'] = t['u'] = 3;
        }
    } tab;
    auto run = [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i) codes[i] = tab.t[(unsigned char)ascii[i]];
    };
    // whole batches of reads (hundreds of MB from the Python drivers) on up to 16 host threads
    const int64_t per = 8 << 20;
    const int nt = (int)std::min<int64_t>(16, std::max<int64_t>(1, n / per));
    if (nt <= 1) {
        run(0, n);
        return;
    }
    std::vector<std::thread> th;
    for (int k = 0; k < nt; ++k) th.emplace_back(run, n * k / nt, n * (k + 1) / nt);
    for (auto &t : th) t.join();
}

void pcabi_pid6_host(const int32_t *m, const int32_t *l, int64_t n, double *out) {
    for (int64_t k = 0; k < n; ++k) out[k] = pcabi::pid6(m[k], l[k]);
}

}  // extern "C"

namespace {

// Shared body of pcabi_align_host / pcabi_first_hits_host. first_thr != nullptr (cross mode
// only): out receives the k_first_hit fields (5 x n_win) instead of the raw results.
// All-vs-all link matrix from the cross product f[a * n + w] (window w as row 0, sequence a as
// rows): per pair the reference's orientation (row 0 = the longer, ties -> the first argument of
// consensus.py:90-97, i < j), mirrored; -1 on the diagonal. 32 x 32 tiles through LDS so both
// the direct and the transposed reads are coalesced.
__global__ __launch_bounds__(256) void k_orient(const int32_t *f, const int32_t *len, int64_t n, int32_t *mat) {
    __shared__ int32_t direct[32][33], trans[32][33];
    const int64_t r0 = (int64_t)blockIdx.y * 32, c0 = (int64_t)blockIdx.x * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8 threads
    for (int y = ty; y < 32; y += 8) {
        const int64_t r = r0 + y, c = c0 + tx;
        direct[y][tx] = (r < n && c < n) ? f[r * n + c] : 0;
        const int64_t rt = c0 + y, ct = r0 + tx;                 // f[c][r] for the tile, row-wise
        trans[tx][y] = (rt < n && ct < n) ? f[rt * n + ct] : 0;
    }
    __syncthreads();
    for (int y = ty; y < 32; y += 8) {
        const int64_t r = r0 + y, c = c0 + tx;
        if (r >= n || c >= n) continue;
        int32_t v = -1;
        if (r != c) {
            const int64_t i = r < c ? r : c, j = r < c ? c : r;
            // want f[j * n + i] when len[i] >= len[j], else f[i * n + j]
            const bool from_j = len[i] >= len[j];
            const bool j_is_r = (j == r);
            v = (from_j == j_is_r) ? direct[y][tx] : trans[y][tx];
        }
        mat[r * n + c] = v;
    }
}

int align_host_impl(int device, const uint8_t *codes, int64_t codes_len, const int64_t *win_off,
                    const int32_t *win_len, int64_t n_win, const uint8_t *adp_codes,
                    const int32_t *adp_off, const int32_t *adp_len, int32_t n_adp,
                    const int32_t *task_win, const int32_t *task_adp, int64_t n_task, int match,
                    int mismatch, int gap_open, int gap_extend, const double *first_thr, int32_t *out,
                    bool compat = false, bool orient = false, double *best = nullptr, bool best_dev = false) {
    if (device < 0 || device >= 16) return fail(PCABI_E_ARG, "bad device index");
    if (n_win < 0 || n_adp < 0 || n_task < 0) return fail(PCABI_E_ARG, "negative count");
    if (int rc = check_common(adp_len, n_adp)) return rc;
    for (int64_t w = 0; w < n_win; ++w) {
        if (win_len[w] < 0 || win_len[w] > pcabi::MAX_WINDOW_LEN)
            return fail(PCABI_E_ARG, "window length out of range");
        if (win_len[w] > 0 && (win_off[w] < 0 || win_off[w] + win_len[w] + 16 > codes_len))
            return fail(PCABI_E_ARG, "window outside the buffer or buffer not padded by 16 bytes");
    }
    const int64_t n_res = task_win ? n_task : (int64_t)n_adp * n_win;
    if (task_win)
        for (int64_t t = 0; t < n_task; ++t)
            if (task_win[t] < 0 || task_win[t] >= n_win || task_adp[t] < 0 || task_adp[t] >= n_adp)
                return fail(PCABI_E_ARG, "task index out of range");
    if (n_res == 0) return 0;

    Engine &e = g_engines[device];
    std::lock_guard<std::mutex> lock(e.mu);
    if (int rc = engine_init(e, device)) return rc;
    HIP_TRY(hipSetDevice(device));

    const pcabi::Scoring sc{match, mismatch, gap_open, gap_extend};
    int64_t max_win = 0;
    bool striped_only = false;
    {
        int max_L = 0;
        for (int a = 0; a < n_adp; ++a)
            if (adp_len[a] <= kMaxRPL) max_L = std::max(max_L, (int)adp_len[a]);   // striped: c never wraps
        for (int64_t w = 0; w < n_win; ++w) max_win = std::max<int64_t>(max_win, win_len[w]);
        striped_only = needs_striped(sc, max_L, max_win);
    }
    BucketHost bk[kNumBuckets];
    build_buckets(adp_codes, adp_off, adp_len, n_adp, sc, bk, true, true, striped_only);

    if (int rc = e.codes.ensure((size_t)codes_len)) return rc;
    if (int rc = e.woff.ensure(sizeof(int64_t) * (size_t)std::max<int64_t>(n_win, 1))) return rc;
    if (int rc = e.wlen.ensure(sizeof(int32_t) * (size_t)std::max<int64_t>(n_win, 1))) return rc;
    if (int rc = e.out.ensure(sizeof(int32_t) * PCABI_NFIELDS * (size_t)n_res)) return rc;
    HIP_TRY(hipMemcpyAsync(e.codes.p, codes, (size_t)codes_len, hipMemcpyHostToDevice, e.stream));
    HIP_TRY(hipMemcpyAsync(e.woff.p, win_off, sizeof(int64_t) * (size_t)n_win, hipMemcpyHostToDevice, e.stream));
    HIP_TRY(hipMemcpyAsync(e.wlen.p, win_len, sizeof(int32_t) * (size_t)n_win, hipMemcpyHostToDevice, e.stream));

    KParams p{};
    p.codes = (const uint8_t *)e.codes.p;
    p.win_off = (const int64_t *)e.woff.p;
    p.win_len = (const int32_t *)e.wlen.p;
    p.n_win = n_win;
    p.out = (int32_t *)e.out.p;
    p.out_stride = n_res;
    p.sc = sc;
    p.compat = compat ? (int32_t *)e.out.p : nullptr;   // pairs mode only (checked by the caller)
    const bool affine = gap_open != gap_extend;

    // host-side pair grouping (pairs mode): per bucket, per adapter, runs padded to 64 lanes
    std::vector<std::vector<int32_t>> per_adp;
    if (task_win) {
        per_adp.resize(n_adp);
        for (int64_t t = 0; t < n_task; ++t) per_adp[task_adp[t]].push_back((int32_t)t);
        // longest windows first: lanes of a wave then run near-equal column counts
        for (auto &v : per_adp)
            std::stable_sort(v.begin(), v.end(), [&](int32_t x, int32_t y) {
                return win_len[task_win[x]] > win_len[task_win[y]];
            });
    }
    std::vector<int32_t> tw, to, wa;
    struct CrossLaunch {
        int b;
        KParams p;
        int packed;   // bucket_pack_mode
    };
    std::vector<CrossLaunch> cross;
    for (int b = 0; b < kNumBuckets; ++b) {
        BucketHost &h = bk[b];
        if (h.len.empty()) continue;
        const int nb = (int)h.len.size();
        if (int rc = e.pad[b].ensure(h.pad.size())) return rc;
        if (int rc = e.len[b].ensure(sizeof(int32_t) * nb)) return rc;
        if (int rc = e.id[b].ensure(sizeof(int32_t) * nb)) return rc;
        HIP_TRY(hipMemcpyAsync(e.pad[b].p, h.pad.data(), h.pad.size(), hipMemcpyHostToDevice, e.stream));
        HIP_TRY(hipMemcpyAsync(e.len[b].p, h.len.data(), sizeof(int32_t) * nb, hipMemcpyHostToDevice, e.stream));
        HIP_TRY(hipMemcpyAsync(e.id[b].p, h.id.data(), sizeof(int32_t) * nb, hipMemcpyHostToDevice, e.stream));
        p.adp_pad = (const uint32_t *)e.pad[b].p;
        p.adp_len = (const int32_t *)e.len[b].p;
        p.adp_id = (const int32_t *)e.id[b].p;
        p.n_adp = nb;
        p.rt = h.rt;
        p.max_cols = (int32_t)std::min<int64_t>(max_win, INT32_MAX);
        if (!task_win) {
            p.task_win = nullptr;
            if (n_win > 0 && !p.tiles) {
                std::vector<int64_t> toff((size_t)((n_win + 255) / 256 + 1));
                int64_t max_nq = 0;
                const int64_t nd = tile_layout(win_len, n_win, toff.data(), &max_nq);
                if (int rc = e.toff.ensure(sizeof(int64_t) * toff.size())) return rc;
                if (int rc = e.tiles.ensure(sizeof(uint32_t) * (size_t)nd)) return rc;
                HIP_TRY(hipMemcpyAsync(e.toff.p, toff.data(), sizeof(int64_t) * toff.size(), hipMemcpyHostToDevice, e.stream));
                launch_tiles(p.codes, p.win_off, p.win_len, n_win, (const int64_t *)e.toff.p, max_nq,
                             (uint32_t *)e.tiles.p, e.stream);
                // toff (host) must outlive the async copy
                HIP_TRY(hipStreamSynchronize(e.stream));
                p.tiles = (const uint32_t *)e.tiles.p;
                p.tile_off = (const int64_t *)e.toff.p;
            }
            // launched below, side by side once every bucket's table is on its way
            if (n_win > 0) cross.push_back({b, p, bucket_pack_mode(b, h.len, sc)});
        } else {
            tw.clear(); to.clear(); wa.clear();
            for (int k = 0; k < nb; ++k) {
                const std::vector<int32_t> &ts = per_adp[h.id[k]];
                for (size_t s = 0; s < ts.size(); s += 64) {
                    wa.push_back(k);
                    for (size_t q = 0; q < 64; ++q) {
                        if (s + q < ts.size()) { tw.push_back(task_win[ts[s + q]]); to.push_back(ts[s + q]); }
                        else { tw.push_back(-1); to.push_back(0); }
                    }
                }
            }
            if (wa.empty()) continue;
            // the per-bucket task arrays must stay alive until the kernel has read them
            if (int rc = e.tasks_win.ensure(sizeof(int32_t) * tw.size())) return rc;
            if (int rc = e.tasks_out.ensure(sizeof(int32_t) * to.size())) return rc;
            if (int rc = e.wave_adp.ensure(sizeof(int32_t) * wa.size())) return rc;
            HIP_TRY(hipMemcpyAsync(e.tasks_win.p, tw.data(), sizeof(int32_t) * tw.size(), hipMemcpyHostToDevice, e.stream));
            HIP_TRY(hipMemcpyAsync(e.tasks_out.p, to.data(), sizeof(int32_t) * to.size(), hipMemcpyHostToDevice, e.stream));
            HIP_TRY(hipMemcpyAsync(e.wave_adp.p, wa.data(), sizeof(int32_t) * wa.size(), hipMemcpyHostToDevice, e.stream));
            p.task_win = (const int32_t *)e.tasks_win.p;
            p.task_out = (const int32_t *)e.tasks_out.p;
            p.wave_adp = (const int32_t *)e.wave_adp.p;
            p.n_waves = (int64_t)wa.size();
            if (int rc = dispatch(b, p, affine, e.stream, bucket_pack_mode(b, h.len, sc))) return rc;
            // host vectors are reused by the next bucket: drain before overwriting
            HIP_TRY(hipStreamSynchronize(e.stream));
        }
        HIP_TRY(hipGetLastError());
        // bucket buffers are reused across calls only; keep them distinct per bucket
    }
    if (!cross.empty()) {
        // the host bucket tables (bk) outlive these launches: they are read by the copies queued
        // on e.stream before the fork
        std::stable_sort(cross.begin(), cross.end(), [&](const CrossLaunch &x, const CrossLaunch &y) {
            return (int64_t)x.p.n_adp * kBuckets[x.b].rpl > (int64_t)y.p.n_adp * kBuckets[y.b].rpl;
        });
        ForkJoin fj;
        if (int rc = fj.begin(e.stream, cross.size())) return rc;
        for (size_t k = 0; k < cross.size(); ++k)
            if (int rc = dispatch(cross[k].b, cross[k].p, affine, fj.at(k), cross[k].packed)) {
                (void)fj.end();
                return rc;
            }
        if (int rc = fj.end()) return rc;
        HIP_TRY(hipGetLastError());
    }
    if (first_thr) {
        if (int rc = e.hits.ensure(sizeof(int32_t) * 5 * (size_t)n_win)) return rc;
        hipLaunchKernelGGL(k_first_hit, dim3((unsigned)((n_win + 255) / 256)), dim3(256), 0, e.stream,
                           (const int32_t *)e.out.p, n_res, n_win, n_adp, *first_thr, nullptr,
                           (int32_t *)e.hits.p, n_win);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(out, e.hits.p, sizeof(int32_t) * 5 * (size_t)n_win, hipMemcpyDeviceToHost,
                               e.stream));
    } else if (best) {     // adapter-set search: per-adapter max of the full identity, on the device
        double *d_best = best;
        if (!best_dev) {
            if (int rc = e.hits.ensure(sizeof(double) * (size_t)n_adp)) return rc;
            d_best = (double *)e.hits.p;
            HIP_TRY(hipMemcpyAsync(d_best, best, sizeof(double) * (size_t)n_adp, hipMemcpyHostToDevice, e.stream));
        }
        hipLaunchKernelGGL(k_best_full_id, dim3((unsigned)n_adp), dim3(256), 0, e.stream, (const int32_t *)e.out.p,
                           n_res, n_win, d_best);
        HIP_TRY(hipGetLastError());
        if (!best_dev)
            HIP_TRY(hipMemcpyAsync(best, d_best, sizeof(double) * (size_t)n_adp, hipMemcpyDeviceToHost, e.stream));
    } else if (orient) {   // compat all-vs-all: n_win == n_adp == n, the matrix comes back
        if (int rc = e.hits.ensure(sizeof(int32_t) * (size_t)n_res)) return rc;
        const unsigned tb = (unsigned)((n_win + 31) / 32);
        hipLaunchKernelGGL(k_orient, dim3(tb, tb), dim3(256), 0, e.stream, (const int32_t *)e.out.p,
                           (const int32_t *)e.wlen.p, n_win, (int32_t *)e.hits.p);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(out, e.hits.p, sizeof(int32_t) * (size_t)n_res, hipMemcpyDeviceToHost, e.stream));
    } else {
        HIP_TRY(hipMemcpyAsync(out, e.out.p, sizeof(int32_t) * (compat ? 1 : PCABI_NFIELDS) * (size_t)n_res,
                               hipMemcpyDeviceToHost, e.stream));
    }
    HIP_TRY(hipStreamSynchronize(e.stream));
    return 0;
}

}  // namespace

namespace {
int64_t middle_scan_resident(Engine &e, const int64_t *win_off, const int32_t *win_len, int64_t n_win,
                             const uint8_t *adp_codes, const int32_t *adp_off, const int32_t *adp_len, int32_t n_adp,
                             int match, int mismatch, int gap_open, int gap_extend, double threshold, int32_t *hits,
                             int64_t cap);
int stage_seqs(Engine &e, uint8_t *dst, const char *const *seqs, const int32_t *len, const int64_t *off, int64_t n,
               int64_t total);
}  // namespace

extern "C" {

int pcabi_align_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *win_off,
                     const int32_t *win_len, int64_t n_win, const uint8_t *adp_codes,
                     const int32_t *adp_off, const int32_t *adp_len, int32_t n_adp,
                     const int32_t *task_win, const int32_t *task_adp, int64_t n_task, int match,
                     int mismatch, int gap_open, int gap_extend, int32_t *out) {
    return align_host_impl(device, codes, codes_len, win_off, win_len, n_win, adp_codes, adp_off, adp_len,
                           n_adp, task_win, task_adp, n_task, match, mismatch, gap_open, gap_extend, nullptr,
                           out);
}

int pcabi_best_full_identity_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *win_off,
                                  const int32_t *win_len, int64_t n_win, const uint8_t *adp_codes,
                                  const int32_t *adp_off, const int32_t *adp_len, int32_t n_adp, int match,
                                  int mismatch, int gap_open, int gap_extend, double *best, int best_on_device) {
    if (!best && n_adp > 0) return fail(PCABI_E_ARG, "best is NULL");
    if (n_win == 0 || n_adp == 0) return 0;     // no window: every maximum stays as given
    return align_host_impl(device, codes, codes_len, win_off, win_len, n_win, adp_codes, adp_off, adp_len, n_adp,
                           nullptr, nullptr, 0, match, mismatch, gap_open, gap_extend, nullptr, nullptr, false, false,
                           best, best_on_device != 0);
}

int pcabi_first_hits_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *win_off,
                          const int32_t *win_len, int64_t n_win, const uint8_t *adp_codes,
                          const int32_t *adp_off, const int32_t *adp_len, int32_t n_adp, int match,
                          int mismatch, int gap_open, int gap_extend, double threshold, int32_t *hits) {
    if (n_win > 0 && n_adp == 0) {
        for (int64_t w = 0; w < n_win; ++w) {
            hits[w] = -1; hits[n_win + w] = -1; hits[2 * n_win + w] = 0; hits[3 * n_win + w] = 0;
            hits[4 * n_win + w] = 0;
        }
        return 0;
    }
    return align_host_impl(device, codes, codes_len, win_off, win_len, n_win, adp_codes, adp_off, adp_len,
                           n_adp, nullptr, nullptr, 0, match, mismatch, gap_open, gap_extend, &threshold, hits);
}

int64_t pcabi_middle_scan_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *win_off,
                               const int32_t *win_len, int64_t n_win, const uint8_t *adp_codes,
                               const int32_t *adp_off, const int32_t *adp_len, int32_t n_adp, int match,
                               int mismatch, int gap_open, int gap_extend, double threshold, int32_t *hits,
                               int64_t cap) {
    if (device < 0 || device >= 16) return fail(PCABI_E_ARG, "bad device index");
    if (n_win < 0 || n_adp < 0 || cap < 0) return fail(PCABI_E_ARG, "negative count");
    if (int rc = check_common(adp_len, n_adp)) return rc;
    for (int64_t w = 0; w < n_win; ++w) {
        if (win_len[w] < 0 || win_len[w] > pcabi::MAX_WINDOW_LEN)
            return fail(PCABI_E_ARG, "window length out of range");
        if (win_len[w] > 0 && (win_off[w] < 0 || win_off[w] + win_len[w] + 16 > codes_len))
            return fail(PCABI_E_ARG, "window outside the buffer or buffer not padded by 16 bytes");
    }
    if (n_win == 0 || n_adp == 0) return 0;
    Engine &e = g_engines[device];
    std::lock_guard<std::mutex> lock(e.mu);
    if (int rc = engine_init(e, device)) return rc;
    HIP_TRY(hipSetDevice(device));
    if (int rc = e.codes.ensure((size_t)codes_len)) return rc;
    HIP_TRY(hipMemcpyAsync(e.codes.p, codes, (size_t)codes_len, hipMemcpyHostToDevice, e.stream));
    return middle_scan_resident(e, win_off, win_len, n_win, adp_codes, adp_off, adp_len, n_adp, match, mismatch,
                                gap_open, gap_extend, threshold, hits, cap);
}

int pcabi_stage_seqs_host(int device, const char *const *seqs, const int32_t *seq_len, int64_t n, uint8_t *out,
                          int64_t out_len) {
    if (device < 0 || device >= 16) return fail(PCABI_E_ARG, "bad device index");
    if (n < 0) return fail(PCABI_E_ARG, "negative count");
    int64_t total = 0;
    std::vector<int64_t> off((size_t)n);
    for (int64_t w = 0; w < n; ++w) {
        if (seq_len[w] < 0 || seq_len[w] > pcabi::MAX_WINDOW_LEN) return fail(PCABI_E_ARG, "window length out of range");
        if (seq_len[w] > 0 && !seqs[w]) return fail(PCABI_E_ARG, "NULL sequence");
        off[(size_t)w] = total;
        total += ((int64_t)seq_len[w] + 3) & ~(int64_t)3;
    }
    total += 16;
    if (out_len < total) return fail(PCABI_E_ARG, "output buffer smaller than the layout");
    Engine &e = g_engines[device];
    std::lock_guard<std::mutex> lock(e.mu);
    if (int rc = engine_init(e, device)) return rc;
    HIP_TRY(hipSetDevice(device));
    if (int rc = e.codes.ensure((size_t)total)) return rc;
    if (int rc = stage_seqs(e, (uint8_t *)e.codes.p, seqs, seq_len, off.data(), n, total)) return rc;
    HIP_TRY(hipMemcpyAsync(out, e.codes.p, (size_t)total, hipMemcpyDeviceToHost, e.stream));
    HIP_TRY(hipStreamSynchronize(e.stream));
    return 0;
}

int64_t pcabi_middle_scan_seqs(int device, const char *const *seqs, const int32_t *seq_len, int64_t n,
                               const uint8_t *adp_codes, const int32_t *adp_off, const int32_t *adp_len,
                               int32_t n_adp, int match, int mismatch, int gap_open, int gap_extend,
                               double threshold, int32_t *hits, int64_t cap) {
    if (device < 0 || device >= 16) return fail(PCABI_E_ARG, "bad device index");
    if (n < 0 || n_adp < 0 || cap < 0) return fail(PCABI_E_ARG, "negative count");
    if (int rc = check_common(adp_len, n_adp)) return rc;
    // the layout of pcabi_middle_scan_host's buffer (and of the Python SeqPack): windows back to
    // back from 4-aligned offsets, N between them and 16 N bytes after the last
    std::vector<int64_t> off((size_t)n);
    int64_t total = 0;
    for (int64_t w = 0; w < n; ++w) {
        if (seq_len[w] < 0 || seq_len[w] > pcabi::MAX_WINDOW_LEN) return fail(PCABI_E_ARG, "window length out of range");
        if (seq_len[w] > 0 && !seqs[w]) return fail(PCABI_E_ARG, "NULL sequence");
        off[(size_t)w] = total;
        total += ((int64_t)seq_len[w] + 3) & ~(int64_t)3;
    }
    total += 16;
    if (n == 0 || n_adp == 0) return 0;
    Engine &e = g_engines[device];
    std::lock_guard<std::mutex> lock(e.mu);
    if (int rc = engine_init(e, device)) return rc;
    HIP_TRY(hipSetDevice(device));
    if (int rc = e.codes.ensure((size_t)total)) return rc;
    if (int rc = stage_seqs(e, (uint8_t *)e.codes.p, seqs, seq_len, off.data(), n, total)) return rc;
    return middle_scan_resident(e, off.data(), seq_len, n, adp_codes, adp_off, adp_len, n_adp, match, mismatch,
                                gap_open, gap_extend, threshold, hits, cap);
}

}  // extern "C"

namespace {

// The middle scan over windows whose codes are in e.codes (being copied there on e.stream).
int64_t middle_scan_resident(Engine &e, const int64_t *win_off, const int32_t *win_len, int64_t n_win,
                             const uint8_t *adp_codes, const int32_t *adp_off, const int32_t *adp_len, int32_t n_adp,
                             int match, int mismatch, int gap_open, int gap_extend, double threshold, int32_t *hits,
                             int64_t cap) {
    if (int rc = e.woff.ensure(sizeof(int64_t) * (size_t)n_win)) return rc;
    if (int rc = e.wlen.ensure(sizeof(int32_t) * (size_t)n_win)) return rc;
    HIP_TRY(hipMemcpyAsync(e.woff.p, win_off, sizeof(int64_t) * (size_t)n_win, hipMemcpyHostToDevice, e.stream));
    HIP_TRY(hipMemcpyAsync(e.wlen.p, win_len, sizeof(int32_t) * (size_t)n_win, hipMemcpyHostToDevice, e.stream));
    pcabi_adapters *tab = nullptr;
    if (int rc = pcabi_adapters_create_scored(adp_codes, adp_off, adp_len, n_adp, match, mismatch, gap_open,
                                              gap_extend, &tab))
        return rc;
    if (!e.scan) e.scan = new pcabi_scan();
    e.scan->adps = tab;
    const int64_t r = pcabi_middle_scan_dev(e.scan, (uint8_t *)e.codes.p, (const int64_t *)e.woff.p,
                                            (const int32_t *)e.wlen.p, win_len, n_win, match, mismatch, gap_open,
                                            gap_extend, threshold, hits, cap, e.stream);
    (void)hipStreamSynchronize(e.stream);
    e.scan->adps = nullptr;
    pcabi_adapters_destroy(tab);
    return r;
}

// Host strings -> Dna5 codes at dst (device): the layout's bytes [0, total) in chunks of kStageBytes.
// r05: what crosses PCIe is 3 bits a base, not 8 -- each chunk travels as 2-bit codes (base j of
// a 32-base block at bits 2j of its 8 bytes) plus a 1-bit "not A/C/G/T/U" mask (bit j of the
// block's 32-bit word), k_unpack_codes writes the Dna5 bytes (S/basic/alphabet_residue_tabs.h's
// table, as pcabi_encode_dna5: A/a 0, C/c 1, G/g 2, T/t/U/u 3, anything else N = 4) into dst.
// The worker threads gather their share of a chunk's characters (the windows' own bytes, N
// between them) into a thread-local block and encode it with AVX2 (a scalar loop without it) into
// one of four pinned slots; this thread queues each chunk's two copies and its unpack on e.stream
// and waits for a slot only when a worker needs it again. Nothing is written to pageable memory.
constexpr int64_t kStageBytes = 32 << 20;
constexpr int64_t kStageCodes = kStageBytes / 4, kStageMask = kStageBytes / 8, kStageSlot = kStageCodes + kStageMask;

__global__ __launch_bounds__(256) void k_unpack_codes(const uint32_t *__restrict__ codes, const uint32_t *__restrict__ mask,
                                                      uint8_t *__restrict__ dst, int64_t n) {
    // 16 bases a thread: one dword of codes, half a mask word, one 16-byte store
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t b = 16 * q;
    if (b >= n) return;
    const uint32_t c = codes[q];
    const uint32_t m = (mask[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = 4 * k + j;
            const uint32_t v = (m >> i) & 1u ? 4u : (c >> (2 * i)) & 3u;
            x |= v << (8 * j);
        }
        w[k] = x;
    }
    if (b + 16 <= n) {
        *reinterpret_cast<uint4 *>(dst + b) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
        for (int64_t i = b; i < n; ++i) dst[i] = (uint8_t)(w[(i - b) >> 2] >> (8 * ((i - b) & 3)));
    }
}

// 32 characters -> 8 bytes of 2-bit codes + the 32-bit N mask (the scalar and AVX2 forms agree)
inline void pack32_scalar(const uint8_t *s, uint8_t *codes, uint32_t *mask) {
    uint64_t c = 0;
    uint32_t m = 0;
    for (int j = 0; j < 32; ++j) {
        const uint8_t u = s[j] & 0xDF;
        uint32_t v = 4;
        if (u == 'A') v = 0;
        else if (u == 'C') v = 1;
        else if (u == 'G') v = 2;
        else if (u == 'T' || u == 'U') v = 3;
        if (v == 4) m |= 1u << j;
        else c |= (uint64_t)v << (2 * j);
    }
    std::memcpy(codes, &c, 8);
    *mask = m;
}
__attribute__((target("avx2"))) void pack_avx2(const uint8_t *s, int64_t nblk, uint8_t *codes, uint32_t *mask) {
    const __m256i df = _mm256_set1_epi8((char)0xDF);
    const __m256i kA = _mm256_set1_epi8('A'), kC = _mm256_set1_epi8('C'), kG = _mm256_set1_epi8('G');
    const __m256i kT = _mm256_set1_epi8('T'), kU = _mm256_set1_epi8('U');
    const __m256i one = _mm256_set1_epi8(1), two = _mm256_set1_epi8(2), three = _mm256_set1_epi8(3);
    const __m256i m14 = _mm256_set1_epi16(0x0401);             // bytes (1, 4): c0 + 4 c1
    const __m256i m116 = _mm256_set1_epi32(0x00100001);        // words (1, 16)
    const __m256i sh = _mm256_setr_epi8(0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
                                        0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1);
    const __m256i perm = _mm256_setr_epi32(0, 4, 1, 1, 1, 1, 1, 1);
    for (int64_t b = 0; b < nblk; ++b) {
        const __m256i u = _mm256_and_si256(_mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + 32 * b)), df);
        const __m256i eA = _mm256_cmpeq_epi8(u, kA), eC = _mm256_cmpeq_epi8(u, kC), eG = _mm256_cmpeq_epi8(u, kG);
        const __m256i eT = _mm256_or_si256(_mm256_cmpeq_epi8(u, kT), _mm256_cmpeq_epi8(u, kU));
        const __m256i code = _mm256_or_si256(_mm256_or_si256(_mm256_and_si256(eC, one), _mm256_and_si256(eG, two)),
                                             _mm256_and_si256(eT, three));
        const __m256i ok = _mm256_or_si256(_mm256_or_si256(eA, eC), _mm256_or_si256(eG, eT));
        mask[b] = ~(uint32_t)_mm256_movemask_epi8(ok);
        const __m256i p2 = _mm256_maddubs_epi16(code, m14);      // per 16 bits: c0 | c1 << 2
        const __m256i p4 = _mm256_madd_epi16(p2, m116);          // per 32 bits: c0 .. c3 in the low byte
        const __m256i g = _mm256_permutevar8x32_epi32(_mm256_shuffle_epi8(p4, sh), perm);
        _mm_storel_epi64(reinterpret_cast<__m128i *>(codes + 8 * b), _mm256_castsi256_si128(g));
    }
}

int stage_seqs(Engine &e, uint8_t *dst, const char *const *seqs, const int32_t *len, const int64_t *off, int64_t n,
               int64_t total) {
    constexpr int kSlots = 4;
    for (int k = 0; k < kSlots; ++k) {
        if (!e.stage[k]) {
            HIP_TRY(hipHostMalloc((void **)&e.stage[k], (size_t)kStageSlot, hipHostMallocDefault));
            HIP_TRY(hipEventCreateWithFlags(&e.stage_ev[k], hipEventDisableTiming));
        }
        // a call that failed after staging may have left copies out of a slot in flight
        HIP_TRY(hipEventSynchronize(e.stage_ev[k]));
    }
    if (int rc = e.stage_dev.ensure((size_t)(kSlots * kStageSlot))) return rc;
    // PCABI_STAGE_SCALAR=1: the scalar encoder (the form used without AVX2), for its test
    const char *sc_env = std::getenv("PCABI_STAGE_SCALAR");
    const bool avx2 = __builtin_cpu_supports("avx2") && !(sc_env && sc_env[0] == '1');
    // characters [b0, b1) of the layout into raw (windows' bytes, 'N' between them)
    auto gather = [&](int64_t b0, int64_t b1, uint8_t *raw) {
        int64_t w = std::upper_bound(off, off + n, b0) - off - 1;
        int64_t b = b0;
        while (b < b1) {
            if (w >= n) {
                std::memset(raw + (b - b0), 'N', (size_t)(b1 - b));
                break;
            }
            const int64_t s = off[w], t = s + len[w], nx = w + 1 < n ? off[w + 1] : total;
            if (b < t) {
                const int64_t hi = std::min(t, b1);
                std::memcpy(raw + (b - b0), seqs[w] + (b - s), (size_t)(hi - b));
                b = hi;
            }
            const int64_t hi = std::min(nx, b1);
            if (b < hi) {
                std::memset(raw + (b - b0), 'N', (size_t)(hi - b));
                b = hi;
            }
            ++w;
        }
    };
    const int64_t n_chunk = (total + kStageBytes - 1) / kStageBytes;
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>({16, (int64_t)std::thread::hardware_concurrency(),
                                                                 total / (1 << 20)}));
    std::unique_ptr<std::atomic<int>[]> left(new std::atomic<int>[(size_t)n_chunk]);
    for (int64_t c = 0; c < n_chunk; ++c) left[c].store(nt);
    std::atomic<int64_t> free_upto{std::min<int64_t>(kSlots, n_chunk)};   // chunks below it may be encoded
    std::atomic<bool> stop{false};
    auto work = [&](int t) {
        constexpr int64_t kBlk = 256 << 10;                    // characters gathered at a time (L2-resident)
        std::unique_ptr<uint8_t[]> raw(new uint8_t[kBlk + 32]);
        for (int64_t c = 0; c < n_chunk; ++c) {
            while (free_upto.load(std::memory_order_acquire) <= c && !stop.load(std::memory_order_relaxed))
                std::this_thread::yield();
            if (stop.load(std::memory_order_relaxed)) return;
            const int64_t c0 = c * kStageBytes, c1 = std::min(total, c0 + kStageBytes);
            // the thread's share: 32-base blocks of the chunk (the last one may run past c1: 'N')
            const int64_t nb = (c1 - c0 + 31) / 32;
            const int64_t k0 = nb * t / nt, k1 = nb * (t + 1) / nt;
            uint8_t *slot = e.stage[c % kSlots];
            for (int64_t k = k0; k < k1; k += kBlk / 32) {
                const int64_t ke = std::min(k1, k + kBlk / 32);
                const int64_t b0 = c0 + 32 * k, b1 = std::min(c1, c0 + 32 * ke);
                gather(b0, b1, raw.get());
                if (b1 - b0 < 32 * (ke - k)) std::memset(raw.get() + (b1 - b0), 'N', (size_t)(32 * (ke - k) - (b1 - b0)));
                uint8_t *codes = slot + 8 * k;
                uint32_t *mask = reinterpret_cast<uint32_t *>(slot + kStageCodes) + k;
                if (avx2) pack_avx2(raw.get(), ke - k, codes, mask);
                else
                    for (int64_t q = 0; q < ke - k; ++q) pack32_scalar(raw.get() + 32 * q, codes + 8 * q, mask + q);
            }
            left[c].fetch_sub(1, std::memory_order_release);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
    int rc = 0;
    std::string err;
    int64_t freed = std::min<int64_t>(kSlots, n_chunk);   // chunks [0, freed) have a slot
    for (int64_t c = 0; c < n_chunk && !rc; ++c) {
        while (left[c].load(std::memory_order_acquire) > 0) std::this_thread::yield();
        const int64_t c0 = c * kStageBytes, c1 = std::min(total, c0 + kStageBytes);
        const int64_t nb = (c1 - c0 + 31) / 32;
        const int s = (int)(c % kSlots);
        uint8_t *dslot = (uint8_t *)e.stage_dev.p + s * kStageSlot;
        hipError_t he = hipMemcpyAsync(dslot, e.stage[s], (size_t)(8 * nb), hipMemcpyHostToDevice, e.stream);
        if (he == hipSuccess)
            he = hipMemcpyAsync(dslot + kStageCodes, e.stage[s] + kStageCodes, (size_t)(4 * nb), hipMemcpyHostToDevice,
                                e.stream);
        if (he == hipSuccess) he = hipEventRecord(e.stage_ev[s], e.stream);
        if (he == hipSuccess) {
            const int64_t nq = (c1 - c0 + 15) / 16;
            hipLaunchKernelGGL(k_unpack_codes, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, e.stream,
                               (const uint32_t *)dslot, (const uint32_t *)(dslot + kStageCodes), dst + c0, c1 - c0);
            he = hipGetLastError();
        }
        // hand the workers the slot of the oldest copy still queued once it has landed, keeping
        // kSlots - 1 chunks queued or being encoded behind it (the device slot is reused in stream
        // order: its next copy follows this chunk's unpack)
        const int64_t oldest = c - (kSlots - 2);
        if (he == hipSuccess && oldest >= 0 && freed < n_chunk) {
            he = hipEventSynchronize(e.stage_ev[oldest % kSlots]);
            if (he == hipSuccess) {
                freed = std::min<int64_t>(n_chunk, oldest + kSlots);
                free_upto.store(freed, std::memory_order_release);
            }
        }
        if (he != hipSuccess) {
            rc = PCABI_E_DEVICE;
            err = std::string("staging copy: ") + hipGetErrorString(he);
            break;
        }
    }
    stop.store(true);
    for (auto &t : th) t.join();
    if (rc) return fail(rc, err);
    return 0;
}

}  // namespace

extern "C" {

int pcabi_first_hit_dev(const int32_t *res, int64_t stride, int64_t n_win, int32_t n_adp, double threshold,
                        int32_t *hits, int64_t hit_stride, void *stream) {
    if (n_win <= 0) return 0;
    hipLaunchKernelGGL(k_first_hit, dim3((unsigned)((n_win + 255) / 256)), dim3(256), 0, (hipStream_t)stream, res,
                       stride, n_win, n_adp, threshold, nullptr, hits, hit_stride);
    HIP_TRY(hipGetLastError());
    return 0;
}

// ---- legacy drop-in --------------------------------------------------------------------------

static int fmt_pid(char *buf, size_t cap, int m, int l) {
    if (l == 0) return std::snprintf(buf, cap, "-nan");
    return std::snprintf(buf, cap, "%f", 100.0 * m / l);
}

char *adapterAlignment(char *readSeq, char *adapterSeq, int matchScore, int mismatchScore,
                       int gapOpenScore, int gapExtensionScore) {
    const int64_t n = (int64_t)std::strlen(readSeq);
    const int32_t L = (int32_t)std::strlen(adapterSeq);
    char *s = (char *)std::malloc(256);
    if (!s) return nullptr;
    if (n == 0 || L == 0) {
        std::snprintf(s, 256, "-1,0,-1,0,%d,0.000000,0.000000", (int)0x80000000);
        return s;
    }
    std::vector<uint8_t> codes((size_t)((n + 3) & ~3LL) + 16, 4);
    pcabi_encode_dna5(readSeq, codes.data(), n);
    std::vector<uint8_t> ac((size_t)L);
    pcabi_encode_dna5(adapterSeq, ac.data(), L);
    const int64_t woff = 0;
    const int32_t wlen = (int32_t)n;
    const int32_t aoff = 0;
    int32_t out[PCABI_NFIELDS];
    int device = 0;
    (void)hipGetDevice(&device);
    int rc = pcabi_align_host(device, codes.data(), (int64_t)codes.size(), &woff, &wlen, 1, ac.data(), &aoff,
                              &L, 1, nullptr, nullptr, 0, matchScore, mismatchScore, gapOpenScore,
                              gapExtensionScore, out);
    if (rc != 0) {
        // The reference has no error channel and answers every non-empty input: a "-1" sentinel
        // here would read as "no alignment" and silently change trimming decisions, so stop.
        std::fprintf(stderr, "libpcabi: adapterAlignment failed: %s\n", pcabi_last_error());
        std::free(s);
        std::abort();
    }
    char p1[64], p2[64];
    fmt_pid(p1, sizeof p1, out[PCABI_F_M], out[PCABI_F_L1]);
    fmt_pid(p2, sizeof p2, out[PCABI_F_M], out[PCABI_F_L2]);
    std::snprintf(s, 256, "%d,%d,%d,%d,%d,%s,%s", out[0], out[1], out[2], out[3], out[4], p1, p2);
    return s;
}

void freeCString(char *p) { std::free(p); }

// ---- device-resident interface ----------------------------------------------------------------

int pcabi_dev_set(int device) { HIP_TRY(hipSetDevice(device)); return 0; }
int pcabi_dev_malloc(void **ptr, int64_t bytes) { HIP_TRY(hipMalloc(ptr, (size_t)bytes)); return 0; }
int pcabi_dev_free(void *ptr) { HIP_TRY(hipFree(ptr)); return 0; }
int pcabi_dev_h2d(void *dst, const void *src, int64_t bytes) {
    HIP_TRY(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyHostToDevice)); return 0;
}
int pcabi_dev_d2h(void *dst, const void *src, int64_t bytes) {
    HIP_TRY(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDeviceToHost)); return 0;
}
int pcabi_dev_memset(void *dst, int value, int64_t bytes) { HIP_TRY(hipMemset(dst, value, (size_t)bytes)); return 0; }
int pcabi_dev_sync(void) { HIP_TRY(hipDeviceSynchronize()); return 0; }
int pcabi_dev_copy_async(void *dst, const void *src, int64_t bytes, int kind, void *stream) {
    const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : (kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice);
    if (kind < 0 || kind > 2) return fail(PCABI_E_ARG, "copy kind must be 0 (h2d), 1 (d2h) or 2 (d2d)");
    HIP_TRY(hipMemcpyAsync(dst, src, (size_t)bytes, k, (hipStream_t)stream));
    return 0;
}
int pcabi_stream_create(void **stream) {
    hipStream_t s;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = (void *)s;
    return 0;
}
int pcabi_stream_destroy(void *stream) { HIP_TRY(hipStreamDestroy((hipStream_t)stream)); return 0; }
int pcabi_stream_sync(void *stream) { HIP_TRY(hipStreamSynchronize((hipStream_t)stream)); return 0; }
int pcabi_event_create(void **ev) {
    hipEvent_t e;
    HIP_TRY(hipEventCreate(&e));
    *ev = (void *)e;
    return 0;
}
int pcabi_event_destroy(void *ev) { HIP_TRY(hipEventDestroy((hipEvent_t)ev)); return 0; }
int pcabi_event_record(void *ev, void *stream) { HIP_TRY(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream)); return 0; }
int pcabi_stream_wait_event(void *stream, void *ev) {
    HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0));
    return 0;
}
int pcabi_event_elapsed_ms(float *ms, void *start, void *stop) {
    HIP_TRY(hipEventSynchronize((hipEvent_t)stop));
    HIP_TRY(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
    return 0;
}

}  // extern "C"

namespace {
// Device adapter table. sc == nullptr: laid out for the fast buckets (any scoring with negative
// gap costs; pcabi_align_cross_dev rejects scorings the layout cannot serve); otherwise small
// buckets are merged for that scoring (assign_buckets).
int adapters_create_impl(const uint8_t *adp_codes, const int32_t *adp_off, const int32_t *adp_len,
                         int32_t n_adp, const pcabi::Scoring *sc, pcabi_adapters **out, bool all_striped = false) {
    if (int rc = check_common(adp_len, n_adp)) return rc;
    BucketHost bk[kNumBuckets];
    build_buckets(adp_codes, adp_off, adp_len, n_adp, sc ? *sc : pcabi::Scoring{1, -1, -1, -1}, bk, sc != nullptr,
                  sc != nullptr, all_striped);
    pcabi_adapters *a = new pcabi_adapters();
    a->n_adp = n_adp;
    a->hoff.resize((size_t)n_adp);
    a->hlen.assign(adp_len, adp_len + n_adp);
    for (int k = 0; k < n_adp; ++k) {
        a->hoff[k] = (int32_t)a->hcodes.size();
        for (int i = 0; i < adp_len[k]; ++i) {
            if (adp_codes[adp_off[k] + i] > 3) a->has_n = true;
            a->hcodes.push_back(adp_codes[adp_off[k] + i]);
        }
    }
    for (int b = 0; b < kNumBuckets; ++b) {
        const int nb = (int)bk[b].len.size();
        a->count[b] = nb;
        if (!nb) continue;
        a->lens[b] = bk[b].len;
        a->ids[b] = bk[b].id;
        a->rt[b] = bk[b].rt;
        for (int k = 0; k < nb; ++k) {
            if (bk[b].len[k] != kBuckets[b].rpl) a->padded[b] = true;
            a->max_off[b] = std::max(a->max_off[b], kBuckets[b].rpl - bk[b].len[k]);
        }
        if (hipMalloc((void **)&a->pad[b], bk[b].pad.size()) != hipSuccess ||
            hipMalloc((void **)&a->len[b], sizeof(int32_t) * nb) != hipSuccess ||
            hipMalloc((void **)&a->id[b], sizeof(int32_t) * nb) != hipSuccess) {
            pcabi_adapters_destroy(a);
            return fail(PCABI_E_NOMEM, "hipMalloc failed for adapter table");
        }
        (void)hipMemcpy(a->pad[b], bk[b].pad.data(), bk[b].pad.size(), hipMemcpyHostToDevice);
        (void)hipMemcpy(a->len[b], bk[b].len.data(), sizeof(int32_t) * nb, hipMemcpyHostToDevice);
        (void)hipMemcpy(a->id[b], bk[b].id.data(), sizeof(int32_t) * nb, hipMemcpyHostToDevice);
    }
    *out = a;
    return 0;
}
}  // namespace

// Whether a table's register layout serves a scoring on windows up to max_win long: padded FAST
// buckets need gap costs < 0 (the fast core's pass-through padding rows), merged buckets (more
// than 3 padding rows) and the wide / long buckets the packed core's range conditions, and long
// windows a bounded path span (needs_striped).
bool layout_serves(const pcabi_adapters *adps, const pcabi::Scoring &sc, int64_t max_win) {
    int max_L = 0;
    bool regs = false;
    for (int b = 0; b < kNumBuckets; ++b) {
        if (!adps->count[b] || kBuckets[b].kind == STRIPED) continue;
        regs = true;
        for (int32_t L : adps->lens[b]) max_L = std::max<int>(max_L, L);
        if (kBuckets[b].kind == FAST && adps->padded[b] && !pcabi::fast_ok(kBuckets[b].rpl - 1, kBuckets[b].rpl, sc))
            return false;
        if (kBuckets[b].kind == FAST && adps->max_off[b] > 3 && !bucket_packed_ok(b, adps->lens[b], sc)) return false;
        if (kBuckets[b].kind == WIDE || kBuckets[b].kind == LONG)
            for (int32_t L : adps->lens[b])
                if (kBuckets[b].kind == WIDE ? !pcabi::packed_ok(L, kBuckets[b].rpl, sc)
                                             : !pcabi::long_ok(L, kBuckets[b].rpl, sc))
                    return false;
    }
    return !regs || !needs_striped(sc, max_L, max_win);
}

// The layout of `adps` to run a scoring on windows up to max_win long: the table itself when it
// serves them, else a layout of the same adapters built for them on first use and cached in the
// table -- every adapter on the striped core when the windows need it, else register buckets for
// this scoring. The reference accepts any scoring for any read (arg_parser.py:229-236,
// adapter_align.cpp:11-31), so the device ABI does too.
int adapters_for(const pcabi_adapters *adps, const pcabi::Scoring &sc, int64_t max_win, const pcabi_adapters **use) {
    if (layout_serves(adps, sc, max_win)) {
        *use = adps;
        return 0;
    }
    pcabi_adapters *a = const_cast<pcabi_adapters *>(adps);   // the cache is the only mutable part
    std::lock_guard<std::mutex> g(a->alt_mu);
    std::vector<int32_t> off((size_t)a->n_adp);
    for (int32_t k = 0; k < a->n_adp; ++k) off[k] = a->hoff[k];
    // register buckets laid out (and merged) for this scoring, if they serve these windows
    pcabi_adapters *t = nullptr;
    for (auto &e : a->alt_scored)
        if (e.first.ma == sc.ma && e.first.mi == sc.mi && e.first.go == sc.go && e.first.ge == sc.ge) t = e.second;
    if (!t) {
        if (int rc = adapters_create_impl(a->hcodes.data(), off.data(), a->hlen.data(), a->n_adp, &sc, &t)) return rc;
        a->alt_scored.emplace_back(sc, t);
    }
    if (layout_serves(t, sc, max_win)) {
        *use = t;
        return 0;
    }
    if (!a->alt_striped) {
        t = nullptr;
        if (int rc = adapters_create_impl(a->hcodes.data(), off.data(), a->hlen.data(), a->n_adp, &sc, &t, true))
            return rc;
        a->alt_striped = t;
    }
    *use = a->alt_striped;
    return 0;
}

extern "C" {

int pcabi_adapters_create(const uint8_t *adp_codes, const int32_t *adp_off, const int32_t *adp_len,
                          int32_t n_adp, pcabi_adapters **out) {
    return adapters_create_impl(adp_codes, adp_off, adp_len, n_adp, nullptr, out);
}

int pcabi_adapters_create_scored(const uint8_t *adp_codes, const int32_t *adp_off, const int32_t *adp_len,
                                 int32_t n_adp, int match, int mismatch, int gap_open, int gap_extend,
                                 pcabi_adapters **out) {
    const pcabi::Scoring sc{match, mismatch, gap_open, gap_extend};
    return adapters_create_impl(adp_codes, adp_off, adp_len, n_adp, &sc, out);
}

void pcabi_adapters_destroy(pcabi_adapters *a) {
    if (!a) return;
    for (auto &e : a->alt_scored) pcabi_adapters_destroy(e.second);
    pcabi_adapters_destroy(a->alt_striped);
    for (int b = 0; b < kNumBuckets; ++b) {
        if (a->pad[b]) (void)hipFree(a->pad[b]);
        if (a->len[b]) (void)hipFree(a->len[b]);
        if (a->id[b]) (void)hipFree(a->id[b]);
    }
    delete a;
}

int64_t pcabi_tile_layout(const int32_t *win_len, int64_t n_win, int64_t *tile_off) {
    if (n_win < 0 || !win_len || !tile_off) return fail(PCABI_E_ARG, "bad arguments");
    return tile_layout(win_len, n_win, tile_off, nullptr);
}

int pcabi_tile_windows_dev(const uint8_t *codes, const int64_t *win_off, const int32_t *win_len,
                           int64_t n_win, const int64_t *tile_off, int64_t max_chunks, uint32_t *tiles,
                           void *stream) {
    if (n_win < 0) return fail(PCABI_E_ARG, "bad arguments");
    launch_tiles(codes, win_off, win_len, n_win, tile_off, max_chunks, tiles, (hipStream_t)stream);
    HIP_TRY(hipGetLastError());
    return 0;
}

int pcabi_align_cross_dev(const uint32_t *tiles, const int64_t *tile_off, const int32_t *win_len,
                          int64_t n_win, int32_t max_win_len, const pcabi_adapters *adps, int match,
                          int mismatch, int gap_open, int gap_extend, int32_t *out, int64_t out_stride,
                          void *stream) {
    return pcabi_align_cross_dev_marked(tiles, tile_off, win_len, n_win, max_win_len, adps, match, mismatch,
                                        gap_open, gap_extend, out, out_stride, stream, nullptr, nullptr);
}

int pcabi_align_cross_dev_marked(const uint32_t *tiles, const int64_t *tile_off, const int32_t *win_len,
                                 int64_t n_win, int32_t max_win_len, const pcabi_adapters *adps, int match,
                                 int mismatch, int gap_open, int gap_extend, int32_t *out, int64_t out_stride,
                                 void *stream, void *ev_begin, void *ev_end) {
    if (!adps || n_win < 0 || (n_win > 0 && (!tiles || !tile_off))) return fail(PCABI_E_ARG, "bad arguments");
    if (n_win == 0) return 0;
    // a layout of the table that serves this scoring on these windows (the table's own when it can)
    if (int rc = adapters_for(adps, pcabi::Scoring{match, mismatch, gap_open, gap_extend}, max_win_len, &adps))
        return rc;
    KParams p{};
    p.tiles = tiles;
    p.tile_off = tile_off;
    p.win_len = win_len;
    p.n_win = n_win;
    p.out = out;
    p.out_stride = out_stride;
    p.sc = pcabi::Scoring{match, mismatch, gap_open, gap_extend};
    p.max_cols = max_win_len;
    const bool affine = gap_open != gap_extend;
    std::vector<int> order;
    for (int b = 0; b < kNumBuckets; ++b)
        if (adps->count[b]) order.push_back(b);
    // Largest bucket (adapters x rows) on the caller's stream, the others spread over the
    // device's side streams (fork / join with events): a bucket holding one or two adapters is
    // too small a grid to fill 256 CUs on its own, side by side they do.
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
        return (int64_t)adps->count[x] * kBuckets[x].rpl > (int64_t)adps->count[y] * kBuckets[y].rpl;
    });
    ForkJoin fj;
    if (int rc = fj.begin((hipStream_t)stream, order.size())) return rc;
    for (size_t k = 0; k < order.size(); ++k) {
        const int b = order[k];
        p.adp_pad = adps->pad[b];
        p.adp_len = adps->len[b];
        p.adp_id = adps->id[b];
        p.n_adp = adps->count[b];
        p.rt = adps->rt[b];
        const hipStream_t st = fj.at(k);
        // the largest bucket runs on the caller's stream (k == 0): the optional events bracket it
        if (k == 0 && ev_begin) HIP_TRY(hipEventRecord((hipEvent_t)ev_begin, st));
        if (int rc = dispatch(b, p, affine, st, bucket_pack_mode(b, adps->lens[b], p.sc))) {
            (void)fj.end();
            return rc;
        }
        if (k == 0 && ev_end) HIP_TRY(hipEventRecord((hipEvent_t)ev_end, st));
    }
    if (int rc = fj.end()) return rc;
    HIP_TRY(hipGetLastError());
    return 0;
}

int pcabi_align_cross_multi_dev(const pcabi_cross_region *regions, int32_t n_regions, int match, int mismatch,
                                int gap_open, int gap_extend, void *stream, void *ev_begin, void *ev_end) {
    if (n_regions < 0 || (n_regions > 0 && !regions)) return fail(PCABI_E_ARG, "bad arguments");
    const pcabi::Scoring sc{match, mismatch, gap_open, gap_extend};
    const bool affine = gap_open != gap_extend;
    // the units: (region, bucket) with its launch class (-1: a launch of its own)
    struct Unit {
        int cls, b, pack;
        KParams p;
        int64_t blocks, cost;
    };
    std::vector<Unit> units;
    for (int32_t r = 0; r < n_regions; ++r) {
        const pcabi_cross_region &g = regions[r];
        if (!g.adps || g.n_win < 0 || (g.n_win > 0 && (!g.tiles || !g.tile_off || !g.win_len || !g.out)))
            return fail(PCABI_E_ARG, "bad region " + std::to_string(r));
        if (g.n_win == 0) continue;
        const pcabi_adapters *adps = nullptr;
        if (int rc = adapters_for(g.adps, sc, g.max_win_len, &adps)) return rc;
        for (int b = 0; b < kNumBuckets; ++b) {
            if (!adps->count[b]) continue;
            Unit u{};
            u.b = b;
            u.pack = bucket_pack_mode(b, adps->lens[b], sc);
            u.cls = kBuckets[b].kind == FAST ? group_class(kBuckets[b].rpl, u.pack, affine) : -1;
            KParams &p = u.p;
            p.tiles = g.tiles;
            p.tile_off = g.tile_off;
            p.win_len = g.win_len;
            p.n_win = g.n_win;
            p.out = g.out;
            p.out_stride = g.out_stride;
            p.sc = sc;
            p.max_cols = g.max_win_len;
            p.adp_pad = adps->pad[b];
            p.adp_len = adps->len[b];
            p.adp_id = adps->id[b];
            p.n_adp = adps->count[b];
            p.rt = adps->rt[b];
            u.blocks = (g.n_win + 8 * 256 - 1) / (8 * 256) * 8 * (int64_t)p.n_adp;
            u.cost = (g.n_win + 255) / 256 * (int64_t)p.n_adp * kBuckets[b].rpl;
            units.push_back(u);
        }
    }
    if (units.empty()) return 0;
    // the launches: per class, its units longest rows first in segments of at most kMaxGroupSegs;
    // a class of one unit launches it on its own (k_align, the row split where that applies)
    struct Launch {
        int cls;                 // -1: units[unit] alone
        size_t unit;
        GroupParams gp;
        int64_t blocks, cost;
    };
    std::vector<Launch> launches;
    for (int c = 0; c < kGroupClasses; ++c) {
        std::vector<size_t> mine;
        for (size_t k = 0; k < units.size(); ++k)
            if (units[k].cls == c) mine.push_back(k);
        if (mine.size() == 1) units[mine[0]].cls = -1;
        if (mine.size() <= 1) continue;
        std::stable_sort(mine.begin(), mine.end(),
                         [&](size_t x, size_t y) { return kBuckets[units[x].b].rpl > kBuckets[units[y].b].rpl; });
        for (size_t k0 = 0; k0 < mine.size(); k0 += kMaxGroupSegs) {
            Launch l{};
            l.cls = c;
            l.gp.sc = sc;
            for (size_t k = k0; k < std::min(mine.size(), k0 + kMaxGroupSegs); ++k) {
                const Unit &u = units[mine[k]];
                GroupSeg &s = l.gp.seg[l.gp.n_seg++];
                s.tiles = u.p.tiles;
                s.tile_off = u.p.tile_off;
                s.win_len = u.p.win_len;
                s.n_win = u.p.n_win;
                s.adp_pad = u.p.adp_pad;
                s.adp_len = u.p.adp_len;
                s.adp_id = u.p.adp_id;
                s.n_adp = u.p.n_adp;
                s.out = u.p.out;
                s.out_stride = u.p.out_stride;
                s.rpl = kBuckets[u.b].rpl;
                s.block0 = l.blocks;
                l.blocks += u.blocks;
                l.cost += u.cost;
            }
            launches.push_back(l);
        }
    }
    for (size_t k = 0; k < units.size(); ++k)
        if (units[k].cls < 0) {
            Launch l{};
            l.cls = -1;
            l.unit = k;
            l.cost = units[k].cost;
            launches.push_back(l);
        }
    std::stable_sort(launches.begin(), launches.end(), [](const Launch &x, const Launch &y) { return x.cost > y.cost; });
    ForkJoin fj;
    if (int rc = fj.begin((hipStream_t)stream, launches.size())) return rc;
    for (size_t k = 0; k < launches.size(); ++k) {
        const Launch &l = launches[k];
        const hipStream_t st = fj.at(k);
        if (k == 0 && ev_begin) HIP_TRY(hipEventRecord((hipEvent_t)ev_begin, st));
        if (l.cls >= 0) {
            dispatch_group(l.cls, l.gp, l.blocks, st);
        } else {
            const Unit &u = units[l.unit];
            if (int rc = dispatch(u.b, u.p, affine, st, u.pack)) {
                (void)fj.end();
                return rc;
            }
        }
        if (k == 0 && ev_end) HIP_TRY(hipEventRecord((hipEvent_t)ev_end, st));
    }
    if (int rc = fj.end()) return rc;
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // extern "C"


extern "C" {

int pcabi_scan_create(const pcabi_adapters *adps, pcabi_scan **out) {
    if (!adps || !out) return fail(PCABI_E_ARG, "bad arguments");
    pcabi_scan *s = new pcabi_scan();
    s->adps = adps;
    *out = s;
    return 0;
}

void pcabi_scan_destroy(pcabi_scan *s) {
    if (!s) return;
    for (DeviceBuf *b : {&s->tiles, &s->toff, &s->res, &s->hits, &s->idx, &s->start, &s->soff, &s->slen,
                         &s->mwin, &s->eoff, &s->shadow, &s->shadow_zero, &s->s16, &s->tw, &s->to, &s->wa, &s->pres, &s->tck,
                         &s->pspan, &s->ptasks, &s->pfill, &s->pwoff, &s->pcidx, &s->pcand, &s->pbest, &s->phit, &s->phb,
                         &s->plist, &s->pcnt, &s->q_cur, &s->q_start, &s->q_list, &s->q_n, &s->q_flags,
                         &s->q_bk, &s->q_wave, &s->q_misc, &s->pcbase, &s->plen, &s->tw2, &s->to2, &s->tck2,
                         &s->pcand2, &s->wa2, &s->pres2, &s->pcert, &s->pucert, &s->q_bk2, &s->q_misc2, &s->pprof, &s->pcount})
        if (b->p) (void)hipFree(b->p);
    if (s->h_stage) (void)hipHostFree(s->h_stage);
    if (s->h_ctl) (void)hipHostFree(s->h_ctl);
    for (auto &g : s->graphs)
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
    if (s->seed) pcabi_seed::destroy(s->seed);
    delete s;
}

}  // extern "C"

namespace {

// Round 1 of the middle scan through the score filter: best scores of every (read, adapter) in
// packed 16-bit lanes (k_score_filter), then the attribute DP only for the pairs that can reach
// the threshold (pairs mode), and per read the first of those (adapter order) that does.
// Fills hb (5 x n, the k_first_hit layout). Returns 1 if it ran, 0 if the filter does not apply
// to this scoring (caller falls back to the full cross product), < 0 on error.
// Later rounds (h_start != nullptr) reuse round 1's scores as bounds: masking turns read bases
// into N, which never matches an adapter base, so no alignment of the masked read scores above
// the same alignment of the unmasked one -- a pair below the threshold in round 1 stays below.
// h16 / pos1: round 1's scores (adapter-major, round-1 positions) and each read's position.
// Seeds (pcabi_seed.hip) replace the filter when they apply; they are cheap enough to run again
// in every later round on the masked reads (seeded: in, round 1 used them; out, this call did),
// where the hits just masked no longer seed their adapter. make_tiles() lays out this round's
// tiles, which only the filter reads.
// Seeded round with the candidates on the device (dcand: nc unordered keys a << 32 | window):
// plans, runs and merges the candidate DP on the device (kernels above) and fills hb (5 x n, the
// k_first_hit layout) from the windows that hit, the only data that comes back. d_start: this
// round's first adapter per window (device), nullptr in round 1. max_len: longest window.
int device_plan_hits(pcabi_scan *sc, const uint8_t *codes, const int64_t *v_off, const int32_t *v_len, int64_t n,
                     int32_t max_len, const int32_t *d_start, const int64_t *dcand, int64_t nc,
                     const pcabi::Scoring &scr, double threshold, std::vector<int32_t> &hb, hipStream_t st) {
    const pcabi_adapters *adps = sc->adps;
    const int32_t n_adp = adps->n_adp;
    hb.assign((size_t)(5 * n), 0);
    for (int64_t k = 0; k < n; ++k) hb[k] = -1;
    if (nc == 0) return 1;
    // per adapter: the chunk lead-in D of its bucket's plan (-1: whole windows), as the host plan
    std::vector<int32_t> span((size_t)n_adp, -1);
    std::vector<char> bchunk(kNumBuckets, 0);
    std::vector<int32_t> bspan(kNumBuckets, 0);       // largest D of a chunked bucket
    for (int b = 0; b < kNumBuckets; ++b) {
        const int nb = adps->count[b];
        if (!nb) continue;
        bool chunk = chunkable(b, bucket_packed_ok(b, adps->lens[b], scr));
        std::vector<int> sp((size_t)nb, -1);
        for (int kk = 0; chunk && kk < nb; ++kk) {
            const int L = adps->lens[b][kk];
            sp[kk] = pcabi::sf::chunk_span(L, pcabi::sf::filter_threshold(L, threshold, scr), scr);
            if (sp[kk] < 0) chunk = false;
        }
        bchunk[b] = chunk;
        if (chunk)
            for (int kk = 0; kk < nb; ++kk) {
                span[adps->ids[b][kk]] = sp[kk];
                bspan[b] = std::max(bspan[b], sp[kk]);
            }
    }
    if (int rc = sc->pspan.ensure(sizeof(int32_t) * n_adp)) return rc;
    if (int rc = sc->ptasks.ensure(sizeof(int32_t) * n_adp * kPlanC)) return rc;
    if (int rc = sc->pfill.ensure(sizeof(int32_t) * n_adp)) return rc;
    if (int rc = sc->pwoff.ensure(sizeof(int64_t) * n_adp)) return rc;
    if (int rc = sc->pcidx.ensure(sizeof(int32_t) * n_adp)) return rc;
    HIP_TRY(hipMemcpyAsync(sc->pspan.p, span.data(), sizeof(int32_t) * n_adp, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(sc->ptasks.p, 0, sizeof(int32_t) * n_adp * kPlanC, st));
    const unsigned gc = (unsigned)((nc + 255) / 256);
    hipLaunchKernelGGL(k_plan_count, dim3(gc), dim3(256), 0, st, dcand, nc, nullptr, v_len, d_start,
                       (const int32_t *)sc->pspan.p, (int32_t *)sc->ptasks.p, nullptr);
    HIP_TRY(hipGetLastError());
    std::vector<int32_t> tasks((size_t)n_adp * kPlanC);
    HIP_TRY(hipMemcpyAsync(tasks.data(), sc->ptasks.p, sizeof(int32_t) * tasks.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    // chunk length per bucket (the buckets run side by side): the longest whose waves reach the
    // target -- a launch of few waves runs as long as its longest chunk -- else the shortest
    const int64_t target = middle_plan_waves();
    std::vector<int32_t> cidx((size_t)n_adp, 0);
    std::vector<int> bc(kNumBuckets, 0);
    for (int b = 0; b < kNumBuckets; ++b) {
        if (!adps->count[b] || !bchunk[b]) continue;
        for (int cc = kPlanC - 1; cc > 0; --cc) {
            int64_t w = 0;
            for (int32_t a : adps->ids[b]) w += (tasks[(size_t)a * kPlanC + cc] + 63) / 64;
            if (w >= target) {
                bc[b] = cc;
                break;
            }
        }
        for (int32_t a : adps->ids[b]) cidx[a] = bc[b];
    }
    // wave layout: buckets in order, a bucket's adapters in order, one adapter per wave
    std::vector<int64_t> woff((size_t)n_adp, 0);
    std::vector<int32_t> wa;
    std::vector<int> nb_used;
    std::vector<int32_t> nb_maxcols;
    std::vector<int64_t> wave0;
    for (int b = 0; b < kNumBuckets; ++b) {
        const int nb = adps->count[b];
        if (!nb) continue;
        const size_t w_before = wa.size();
        for (int kk = 0; kk < nb; ++kk) {
            const int32_t a = adps->ids[b][kk];
            woff[a] = (int64_t)wa.size();
            const int64_t nw = (tasks[(size_t)a * kPlanC + bc[b]] + 63) / 64;
            for (int64_t w = 0; w < nw; ++w) wa.push_back(kk);
        }
        if (wa.size() == w_before) continue;
        nb_used.push_back(b);
        nb_maxcols.push_back(bchunk[b] ? std::min<int32_t>(max_len, (kPlanMin << bc[b]) + bspan[b] + 1) : max_len);
        wave0.push_back((int64_t)w_before);
    }
    wave0.push_back((int64_t)wa.size());
    const int64_t slots = (int64_t)wa.size() * 64;
    if (g_debug) {
        std::string d;
        for (size_t k = 0; k < nb_used.size(); ++k)
            d += " rpl" + std::to_string(kBuckets[nb_used[k]].rpl) + ":" + std::to_string(wave0[k + 1] - wave0[k]) +
                 "w/c" + std::to_string(kPlanMin << bc[nb_used[k]]);
        std::fprintf(stderr, "[pcabi] middle device plan: %lld candidates, waves per bucket:%s\n", (long long)nc,
                     d.c_str());
    }
    if (slots == 0) return 1;
    if (int rc = sc->tw.ensure(sizeof(int32_t) * slots)) return rc;
    if (int rc = sc->to.ensure(sizeof(int32_t) * slots)) return rc;
    if (int rc = sc->tck.ensure(sizeof(int4) * slots)) return rc;
    if (int rc = sc->pcand.ensure(sizeof(int32_t) * slots)) return rc;
    if (int rc = sc->wa.ensure(sizeof(int32_t) * wa.size())) return rc;
    if (int rc = sc->pres.ensure(sizeof(int32_t) * PCABI_NFIELDS * (size_t)slots)) return rc;
    if (int rc = sc->pbest.ensure(sizeof(unsigned long long) * nc)) return rc;
    if (int rc = sc->phit.ensure(sizeof(int32_t) * n)) return rc;
    if (int rc = sc->phb.ensure(sizeof(int32_t) * 5 * n)) return rc;
    if (int rc = sc->plist.ensure(sizeof(int32_t) * 6 * n)) return rc;
    if (int rc = sc->pcnt.ensure(sizeof(unsigned int))) return rc;
    HIP_TRY(hipMemcpyAsync(sc->pwoff.p, woff.data(), sizeof(int64_t) * n_adp, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(sc->pcidx.p, cidx.data(), sizeof(int32_t) * n_adp, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(sc->wa.p, wa.data(), sizeof(int32_t) * wa.size(), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)sc->tw.p, -1, (size_t)slots, st));
    HIP_TRY(hipMemsetAsync(sc->pfill.p, 0, sizeof(int32_t) * n_adp, st));
    hipLaunchKernelGGL(k_plan_place, dim3(gc), dim3(256), 0, st, dcand, nc, nullptr, v_len, d_start,
                       (const int32_t *)sc->pspan.p, (const int32_t *)sc->pcidx.p, (const int64_t *)sc->pwoff.p,
                       (int32_t *)sc->pfill.p,
                       (int32_t *)sc->tw.p, (int32_t *)sc->to.p, (int4 *)sc->tck.p, (int32_t *)sc->pcand.p, nullptr,
                       nullptr, nullptr);
    HIP_TRY(hipGetLastError());
    KParams p{};
    p.codes = codes;
    p.win_off = v_off;
    p.win_len = v_len;
    p.n_win = n;
    p.out = (int32_t *)sc->pres.p;
    p.out_stride = slots;
    p.sc = scr;
    {
        ForkJoin fj;
        if (int rc = fj.begin(st, nb_used.size())) return rc;
        for (size_t k = 0; k < nb_used.size(); ++k) {
            const int b = nb_used[k];
            p.adp_pad = adps->pad[b];
            p.adp_len = adps->len[b];
            p.adp_id = adps->id[b];
            p.n_adp = adps->count[b];
            p.task_win = (const int32_t *)sc->tw.p + wave0[k] * 64;
            p.task_out = (const int32_t *)sc->to.p + wave0[k] * 64;
            p.wave_adp = (const int32_t *)sc->wa.p + wave0[k];
            p.task_chunk = (const int4 *)sc->tck.p + wave0[k] * 64;
            p.n_waves = wave0[k + 1] - wave0[k];
            p.rt = adps->rt[b];
            p.max_cols = nb_maxcols[k];
            int rc;
            if (bchunk[b]) {
                rc = dispatch_chunk(b, p, scr.go != scr.ge, fj.at(k), bucket_pack_mode(b, adps->lens[b], scr) == 2);
            } else {
                p.task_chunk = nullptr;   // whole windows
                rc = dispatch(b, p, scr.go != scr.ge, fj.at(k), bucket_pack_mode(b, adps->lens[b], scr));
            }
            if (rc) {
                (void)fj.end();
                return rc;
            }
        }
        if (int rc = fj.end()) return rc;
    }
    HIP_TRY(hipGetLastError());
    const unsigned gs = (unsigned)((slots + 255) / 256), gn = (unsigned)((n + 255) / 256);
    HIP_TRY(hipMemsetAsync(sc->pbest.p, 0, sizeof(unsigned long long) * nc, st));
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)sc->phit.p, INT32_MAX, (size_t)n, st));
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)sc->phb.p, -1, (size_t)n, st));
    HIP_TRY(hipMemsetAsync(sc->pcnt.p, 0, sizeof(unsigned int), st));
    const int32_t *tw = (const int32_t *)sc->tw.p, *tcand = (const int32_t *)sc->pcand.p;
    const int4 *tck = (const int4 *)sc->tck.p;
    const int32_t *res = (const int32_t *)sc->pres.p;
    hipLaunchKernelGGL(k_merge_best, dim3(gs), dim3(256), 0, st, tw, tck, tcand, res, slots, nullptr,
                       (unsigned long long *)sc->pbest.p);
    for (int pass = 0; pass < 2; ++pass)
        hipLaunchKernelGGL(k_merge_hit, dim3(gs), dim3(256), 0, st, dcand, tw, tck, tcand, res, slots, nullptr,
                           (const unsigned long long *)sc->pbest.p, threshold, pass, (int32_t *)sc->phit.p,
                           (int32_t *)sc->phb.p, n, nullptr, 0);
    hipLaunchKernelGGL(k_hits_compact, dim3(gn), dim3(256), 0, st, (const int32_t *)sc->phb.p, n,
                       (int32_t *)sc->plist.p, (unsigned int *)sc->pcnt.p);
    HIP_TRY(hipGetLastError());
    unsigned int nh = 0;
    HIP_TRY(hipMemcpyAsync(&nh, sc->pcnt.p, sizeof(nh), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if ((int64_t)nh > n) return fail(PCABI_E_DEVICE, "middle scan: hit count overflow");
    std::vector<int32_t> list((size_t)6 * nh);
    if (nh) {
        HIP_TRY(hipMemcpyAsync(list.data(), sc->plist.p, sizeof(int32_t) * list.size(), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    for (unsigned int j = 0; j < nh; ++j) {
        const int32_t *o = list.data() + 6 * (size_t)j;
        const int64_t k = o[0];
        for (int f = 0; f < 5; ++f) hb[(size_t)f * n + k] = o[1 + f];
    }
    return 1;
}

template <typename MakeTiles>
int filtered_first_hits(pcabi_scan *sc, const uint8_t *codes, const int64_t *v_off, const int32_t *v_len,
                        const int32_t *h_len, int64_t n, const int32_t *h_start, const int32_t *d_start,
                        int32_t max_len, const int32_t *reads,
                        std::vector<int16_t> &h16, int64_t n1, const std::vector<int32_t> &pos1,
                        const pcabi::Scoring &scr, double threshold, std::vector<int32_t> &hb, bool &seeded,
                        const MakeTiles &make_tiles, hipStream_t st) {
    const pcabi_adapters *adps = sc->adps;
    const int32_t n_adp = adps->n_adp;
    std::vector<int> fb;   // buckets the score filter serves, largest first
    for (int b = 0; b < kNumBuckets; ++b)
        if (adps->count[b] && (kBuckets[b].kind == FAST || kBuckets[b].kind == WIDE) &&
            pcabi::sf::filter_ok(kBuckets[b].rpl, scr))
            fb.push_back(b);
    const int seed_mode = middle_seed_mode();
    if (fb.empty() && !seed_mode) return 0;
    std::stable_sort(fb.begin(), fb.end(), [&](int x, int y) {
        return (int64_t)adps->count[x] * kBuckets[x].rpl > (int64_t)adps->count[y] * kBuckets[y].rpl;
    });
    std::vector<char> filtered((size_t)n_adp, 0);
    std::vector<int32_t> lenof((size_t)n_adp, 0);
    for (int b = 0; b < kNumBuckets; ++b)
        for (size_t k = 0; k < adps->ids[b].size(); ++k) lenof[adps->ids[b][k]] = adps->lens[b][k];
    for (int b : fb)
        for (int32_t id : adps->ids[b]) filtered[id] = 1;
    // 1. bounds of every (adapter, read): seeds (any round, when round 1 used them) or the score
    //    filter (round 1 only), buckets side by side
    bool local = !h_start;   // h16 holds this round's bounds (a * n + k), not round 1's
    std::vector<int64_t> seed_cands;   // seeded: the filtered candidates, sorted (a << 32 | k)
    if (!h_start || seeded) {
        if (int rc = sc->s16.ensure(sizeof(int16_t) * (size_t)n * n_adp)) return rc;
        int got = 0;
        const int mode = seed_mode;
        if (mode && (!h_start || seeded)) {
            if (!sc->seed) sc->seed = pcabi_seed::create();
            // seeds cover every adapter the plan accepts, long (generic-core) ones included
            // (striped adapters stay outside: every read is their candidate)
            std::vector<int> rows((size_t)n_adp, 0);
            for (int b = 0; b < kNumBuckets; ++b)
                if (kBuckets[b].kind != STRIPED)
                    for (int32_t id : adps->ids[b]) rows[id] = kBuckets[b].rpl;
            // every adapter seeded (no striped one): the candidates stay on the device
            const bool devplan = middle_devplan_on() && adps->count[kStripedBucket] == 0;
            const int64_t *dcand = nullptr;
            int64_t ndc = 0;
            got = pcabi_seed::bounds(sc->seed, adps, adps->hcodes.data(), adps->hoff.data(), adps->hlen.data(),
                                     n_adp, rows, codes, v_off, v_len, n, scr, threshold, h_start ? 2 : mode,
                                     (int16_t *)sc->s16.p, devplan ? nullptr : &seed_cands,
                                     devplan ? &dcand : nullptr, &ndc, st);
            if (got < 0) return got;
            if (got > 0 && devplan) {
                seeded = true;
                return device_plan_hits(sc, codes, v_off, v_len, n, max_len, h_start ? d_start : nullptr, dcand, ndc,
                                        scr, threshold, hb, st);
            }
        }
        if (h_start && !got) return fail(PCABI_E_DEVICE, "middle scan: seeds stopped applying after round 1");
        seeded = got > 0;
        if (seeded) {
            for (int b = 0; b < kNumBuckets; ++b)
                if (kBuckets[b].kind != STRIPED)
                    for (int32_t id : adps->ids[b]) filtered[id] = 1;
        } else if (fb.empty()) {
            return 0;
        } else {
            if (int rc = make_tiles()) return rc;
            ForkJoin fj;
            if (int rc = fj.begin(st, fb.size())) return rc;
            for (size_t k = 0; k < fb.size(); ++k) {
                const int b = fb[k];
                FParams f{};
                f.tiles = (const uint32_t *)sc->tiles.p;
                f.tile_off = (const int64_t *)sc->toff.p;
                f.win_len = v_len;
                f.n_win = n;
                f.adp_pad = adps->pad[b];
                f.adp_len = adps->len[b];
                f.adp_id = adps->id[b];
                f.n_adp = adps->count[b];
                f.s16 = (int16_t *)sc->s16.p;
                f.sc = scr;
                dispatch_filter(kBuckets[b].rpl, f, scr.go != scr.ge, fj.at(k));
            }
            if (int rc = fj.end()) return rc;
            HIP_TRY(hipGetLastError());
            h16.resize((size_t)n * n_adp);
            HIP_TRY(hipMemcpyAsync(h16.data(), sc->s16.p, sizeof(int16_t) * h16.size(), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
        }
        local = true;
    }
    // 2. candidates (adapter-major): pairs that can reach the threshold, from each read's start
    //    adapter on
    std::vector<int32_t> cand_w, cand_a;
    size_t sc_i = 0;
    for (int32_t a = 0; a < n_adp; ++a) {
        if (seeded && filtered[a]) {                   // from the device's list
            for (; sc_i < seed_cands.size() && (int32_t)(seed_cands[sc_i] >> 32) == a; ++sc_i) {
                const int32_t k = (int32_t)(seed_cands[sc_i] & 0xFFFFFFFF);
                if (h_len[k] <= 0 || (h_start && a < h_start[k])) continue;
                cand_w.push_back(k);
                cand_a.push_back(a);
            }
            continue;
        }
        const int T = pcabi::sf::filter_threshold(lenof[a], threshold, scr);
        const int16_t *row = filtered[a] ? h16.data() + (size_t)a * (local ? n : n1) : nullptr;
        for (int64_t k = 0; k < n; ++k) {
            if (h_len[k] <= 0 || (h_start && a < h_start[k])) continue;
            if (!row || row[local ? k : pos1[reads[k]]] >= T) { cand_w.push_back((int32_t)k); cand_a.push_back(a); }
        }
    }
    const int64_t n_task = (int64_t)cand_w.size();
    hb.assign((size_t)(5 * n), 0);
    for (int64_t k = 0; k < n; ++k) { hb[k] = -1; hb[n + k] = -1; }
    if (g_debug) {
        std::vector<int64_t> per((size_t)n_adp, 0);
        for (int32_t a : cand_a) ++per[a];
        std::string s;
        for (int32_t a = 0; a < n_adp; ++a) s += std::to_string(per[a]) + (a + 1 < n_adp ? "," : "");
        std::fprintf(stderr, "[pcabi] middle round %s: %lld reads, %lld candidate pairs; per adapter: %s\n",
                     h_start ? "2+" : "1", (long long)n, (long long)n_task, s.c_str());
    }
    if (n_task == 0) return 1;
    // attribute DP of the candidates: one task list per bucket (waves of 64 lanes, one adapter
    // per wave), all buckets in one upload, launched side by side. Packed-core buckets split
    // long reads into chunks (sf::chunk_plan), so no lane walks a whole long read alone: a task
    // is one chunk, and a candidate's chunks are merged below.
    std::vector<int64_t> first((size_t)n_adp + 1, 0);
    for (int64_t t = 0; t < n_task; ++t) ++first[cand_a[t] + 1];
    for (int32_t a = 0; a < n_adp; ++a) first[a + 1] += first[a];
    std::vector<int32_t> tw, to, wa;
    std::vector<int4> tck;
    std::vector<int64_t> task_cand;                 // task -> candidate
    std::vector<int32_t> task_start;                // task -> read offset of its chunk
    std::vector<int> nb_used;
    std::vector<char> nb_chunked;
    std::vector<int32_t> nb_maxcols;                // longest window / chunk per bucket (striped scratch)
    std::vector<int64_t> wave0;
    // chunk length: the shortest (power of two >= kChunkColsMin) whose task count stays within
    // kChunkTasks (the count over all candidates, chunked or not -- a bound)
    int chunk_cols = kChunkCols;
    for (int c = kChunkColsMin; c < kChunkCols; c *= 2) {
        int64_t tasks = 0;
        for (int64_t t = 0; t < n_task && tasks <= kChunkTasks; ++t) tasks += (h_len[cand_w[t]] + c - 1) / c;
        if (tasks <= kChunkTasks) {
            chunk_cols = c;
            break;
        }
    }
    for (int b = 0; b < kNumBuckets; ++b) {
        const int nb = adps->count[b];
        if (!nb) continue;
        const size_t w_before = wa.size();
        bool chunk = chunkable(b, bucket_packed_ok(b, adps->lens[b], scr));
        std::vector<int> span((size_t)nb, -1);
        for (int kk = 0; chunk && kk < nb; ++kk) {
            const int L = adps->lens[b][kk];
            span[kk] = pcabi::sf::chunk_span(L, pcabi::sf::filter_threshold(L, threshold, scr), scr);
            if (span[kk] < 0) chunk = false;
        }
        int32_t maxcols = 0;
        for (int kk = 0; kk < nb; ++kk) {
            const int32_t a = adps->ids[b][kk];
            int lane = 64;
            auto add = [&](int64_t t, int32_t w, int4 ck) {
                maxcols = std::max(maxcols, chunk ? ck.y : h_len[w]);
                if (lane == 64) {
                    wa.push_back(kk);
                    lane = 0;
                }
                tw.push_back(w);
                to.push_back((int32_t)task_cand.size());
                tck.push_back(ck);
                task_cand.push_back(t);
                task_start.push_back(ck.x);
                ++lane;
            };
            for (int64_t t = first[a]; t < first[a + 1]; ++t) {
                const int32_t k = cand_w[t];
                if (chunk)
                    pcabi::sf::chunk_plan(h_len[k], span[kk], chunk_cols, [&](const pcabi::sf::Chunk &c) {
                        add(t, k, make_int4(c.start, c.len, c.own_lo, c.own_hi));
                    });
                else
                    add(t, k, make_int4(0, 0, 0, 0));
            }
            for (; lane < 64; ++lane) {                // idle lanes of the adapter's last wave
                tw.push_back(-1);
                to.push_back(0);
                tck.push_back(make_int4(0, 0, 0, 0));
            }
        }
        if (wa.size() == w_before) continue;
        nb_used.push_back(b);
        nb_chunked.push_back(chunk ? 1 : 0);
        nb_maxcols.push_back(maxcols);
        wave0.push_back((int64_t)w_before);
    }
    wave0.push_back((int64_t)wa.size());
    const int64_t n_run = (int64_t)task_cand.size();
    if (g_debug) {
        std::string s;
        for (size_t k = 0; k < nb_used.size(); ++k)
            s += " rpl" + std::to_string(kBuckets[nb_used[k]].rpl) + ":" + std::to_string(wave0[k + 1] - wave0[k]) +
                 "w/" + std::to_string(nb_maxcols[k]) + "c";
        std::fprintf(stderr, "[pcabi] middle tasks %lld (chunks of %d), waves per bucket:%s\n", (long long)n_run,
                     chunk_cols, s.c_str());
    }
    if (int rc = sc->pres.ensure(sizeof(int32_t) * PCABI_NFIELDS * (size_t)n_run)) return rc;
    if (int rc = sc->tw.ensure(sizeof(int32_t) * tw.size())) return rc;
    if (int rc = sc->to.ensure(sizeof(int32_t) * to.size())) return rc;
    if (int rc = sc->wa.ensure(sizeof(int32_t) * wa.size())) return rc;
    if (int rc = sc->tck.ensure(sizeof(int4) * tck.size())) return rc;
    HIP_TRY(hipMemcpyAsync(sc->tw.p, tw.data(), sizeof(int32_t) * tw.size(), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(sc->to.p, to.data(), sizeof(int32_t) * to.size(), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(sc->wa.p, wa.data(), sizeof(int32_t) * wa.size(), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(sc->tck.p, tck.data(), sizeof(int4) * tck.size(), hipMemcpyHostToDevice, st));
    KParams p{};
    p.codes = codes;
    p.win_off = v_off;
    p.win_len = v_len;
    p.n_win = n;
    p.out = (int32_t *)sc->pres.p;
    p.out_stride = n_run;
    p.sc = scr;
    {
        ForkJoin fj;
        if (int rc = fj.begin(st, nb_used.size())) return rc;
        for (size_t k = 0; k < nb_used.size(); ++k) {
            const int b = nb_used[k];
            p.adp_pad = adps->pad[b];
            p.adp_len = adps->len[b];
            p.adp_id = adps->id[b];
            p.n_adp = adps->count[b];
            p.task_win = (const int32_t *)sc->tw.p + wave0[k] * 64;
            p.task_out = (const int32_t *)sc->to.p + wave0[k] * 64;
            p.wave_adp = (const int32_t *)sc->wa.p + wave0[k];
            p.task_chunk = (const int4 *)sc->tck.p + wave0[k] * 64;
            p.n_waves = wave0[k + 1] - wave0[k];
            p.rt = adps->rt[b];
            p.max_cols = nb_maxcols[k];
            int rc;
            if (nb_chunked[k]) {
                rc = dispatch_chunk(b, p, scr.go != scr.ge, fj.at(k), bucket_pack_mode(b, adps->lens[b], scr) == 2);
            } else {
                p.task_chunk = nullptr;   // whole windows
                rc = dispatch(b, p, scr.go != scr.ge, fj.at(k), bucket_pack_mode(b, adps->lens[b], scr));
            }
            if (rc) {
                (void)fj.end();
                return rc;
            }
        }
        if (int rc = fj.end()) return rc;
    }
    HIP_TRY(hipGetLastError());
    std::vector<int32_t> res((size_t)PCABI_NFIELDS * n_run);
    HIP_TRY(hipMemcpyAsync(res.data(), sc->pres.p, sizeof(int32_t) * res.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    // merge each candidate's chunks: the first (read order) with the largest score; read offsets
    // back to the whole read
    std::vector<int64_t> best((size_t)n_task, -1);
    for (int64_t u = 0; u < n_run; ++u) {
        const int64_t t = task_cand[u];
        if (best[t] < 0 || res[4 * n_run + u] > res[4 * n_run + best[t]]) best[t] = u;
    }
    // 3. per read, the first candidate (adapter order) over the threshold
    for (int64_t t = 0; t < n_task; ++t) {
        const int64_t k = cand_w[t];
        const int32_t a = cand_a[t];
        if (hb[k] >= 0 && hb[k] <= a) continue;
        const int64_t u = best[t];
        const int rs = res[0 * n_run + u];
        const int m = res[5 * n_run + u], l2 = res[7 * n_run + u];
        const double full = rs == -1 ? 0.0 : pcabi::pid6(m, l2);
        if (full < threshold) continue;
        hb[k] = a;
        hb[n + k] = rs + task_start[u];
        hb[2 * n + k] = res[1 * n_run + u] + task_start[u];
        hb[3 * n + k] = m;
        hb[4 * n + k] = l2;
    }
    return 1;
}


// PCABI_MIDDLE_DEVROUNDS=0: the seeded scan keeps the host-driven round loop (A/B runs).
bool middle_devrounds_on() {
    const char *e = std::getenv("PCABI_MIDDLE_DEVROUNDS");
    return !(e && e[0] == '0');
}

// ---- the shadow arena of the input-preserving masking (k_round_hits, k_mask_list) ----------------
// eoff values are offsets from the caller's `codes`, so a copy in the arena is addressed as
// codes + eoff like any window (a flat device address space).
int64_t shadow_rel(const pcabi_scan *sc, const uint8_t *codes) {
    return (int64_t)((intptr_t)sc->shadow.p - (intptr_t)codes);
}
constexpr int64_t kShadowMax = (int64_t)INT32_MAX * 16;   // k_round_hits' 16-byte unit index is an int32
constexpr int64_t kShadowLead = 256;                      // arena bytes before the first copy

// The arena's first size: 1/8 of the batch's bases (about 3x the ~4.5 % of reads a round 1 hits at
// the default threshold), at least 16 MB; tests set it with the 4th PCABI_MIDDLE_INIT_CAPS value.
int shadow_reserve(pcabi_scan *sc, const int32_t *h_win_len, int64_t n) {
    if (sc->shadow_cap > 0) return 0;
    int64_t want = 16ll << 20;
    if (h_win_len) {
        int64_t bases = 0;
        for (int64_t k = 0; k < n; ++k) bases += std::max(h_win_len[k], 0);
        want = std::max(want, bases / 8);
    }
    long long raw = 0, task = 0, slots = 0, arena = 0;
    if (const char *e = std::getenv("PCABI_MIDDLE_INIT_CAPS"))
        if (std::sscanf(e, "%lld,%lld,%lld,%lld", &raw, &task, &slots, &arena) == 4 && arena > 0) want = arena;
    want = std::min(std::max(want, kShadowLead), kShadowMax);
    if (int rc = sc->shadow.ensure((size_t)want)) return rc;
    sc->shadow_cap = want;
    return 0;
}

// A larger arena (the round that ran out flagged itself and is queued again): the copies move with
// it (eoff rebased), and the bump goes on from the old end. taken: the bytes the rounds asked for.
int shadow_grow(pcabi_scan *sc, const uint8_t *codes, const int64_t *win_off, int64_t *eoff, int64_t n, int64_t taken,
                unsigned long long *d_bump, hipStream_t st) {
    (void)codes;
    const int64_t old_cap = sc->shadow_cap;
    const int64_t want = std::min<int64_t>(std::max<int64_t>(2 * std::max(old_cap, taken), 1ll << 20), kShadowMax);
    if (want <= old_cap || want < taken - old_cap) return fail(PCABI_E_NOMEM, "middle scan: shadow arena past its limit");
    void *np = nullptr;
    if (hipMalloc(&np, (size_t)want) != hipSuccess) return fail(PCABI_E_NOMEM, "hipMalloc failed (shadow arena)");
    pcabi_poison(np, (size_t)want);
    if (sc->shadow.p && old_cap > 0) HIP_TRY(hipMemcpyAsync(np, sc->shadow.p, (size_t)old_cap, hipMemcpyDeviceToDevice, st));
    const int64_t delta = (int64_t)((intptr_t)np - (intptr_t)sc->shadow.p);
    if (sc->shadow.p && n > 0)
        hipLaunchKernelGGL(k_shadow_rebase, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 2048)), dim3(256), 0, st,
                           win_off, eoff, n, delta);
    HIP_TRY(hipGetLastError());
    const unsigned long long at = (unsigned long long)old_cap;
    if (d_bump) HIP_TRY(hipMemcpyAsync(d_bump, &at, sizeof(at), hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (sc->shadow.p) HIP_TRY(hipFree(sc->shadow.p));
    sc->shadow.p = np;
    sc->shadow.cap = (size_t)want;
    sc->shadow_cap = want;
    return 0;
}

// Overflow recovery of the queued rounds, counted for the tests (pcabi_middle_requeues).
std::atomic<int64_t> g_requeues{0};
std::atomic<int32_t> g_requeue_flags{0};

// Tests: PCABI_MIDDLE_FAULT="round:bits[,round:bits...]" makes the first run of that round (0 =
// round 1 of a call) overflow for real -- its raw-hit slabs (1), inside-task regions (2) and / or
// candidate-DP task slots (4) shrunk to nothing -- so its kernels flag it, nothing of it is kept and
// it is queued again (without growing: the real capacities were enough).
std::vector<std::pair<int64_t, int>> middle_faults() {
    std::vector<std::pair<int64_t, int>> f;
    const char *e = std::getenv("PCABI_MIDDLE_FAULT");
    while (e && *e) {
        long long r = 0;
        int bits = 0, used = 0;
        if (std::sscanf(e, "%lld:%d%n", &r, &bits, &used) < 2 || used <= 0) break;
        f.emplace_back((int64_t)r, bits & 15);
        e += used;
        if (*e == ',') ++e;
    }
    return f;
}

// The whole seeded middle scan as QUEUED rounds: no host synchronisation between the end trim and
// the scan's result. Every round runs the seeded plan's steps with its counts on the device -- the
// reads of the round (round 1: all windows, longest first by a device radix sort; later: those
// that just hit, from the adapter that hit), the seeds (pcabi_seed::bounds_dev), the plan's counts,
// layout and task slots (k_plan_count, k_plan_layout, k_plan_place), the chunked candidate DP (the
// launches stride over the device's wave counts), the merges, the round's hit list and the
// masking. The host queues kBatch rounds, reads the round counts once, and queues more while
// reads still hit. A buffer that overflowed in a round flags it before anything of it is kept or
// masked; the host grows the buffers and queues that round again. The hits come back once, sorted
// by (round, read): per read the reference's discovery order.
// Returns the hit count (> 0, <= 0 on error as pcabi_middle_scan_dev); applied = false when the
// seeded plan does not cover this table and scoring (the caller runs the host-driven loop).
int64_t middle_device_rounds(pcabi_scan *sc, const uint8_t *codes, const int64_t *win_off, const int32_t *win_len,
                             const int32_t *h_win_len, int64_t n_win, const pcabi::Scoring &scr, double threshold,
                             int32_t *hits, int64_t cap, hipStream_t st, bool &applied) {
    applied = false;
    const pcabi_adapters *adps = sc->adps;
    const int32_t n_adp = adps->n_adp;
    if (!middle_devrounds_on() || !middle_devplan_on() || adps->count[kStripedBucket] || n_win >= (1ll << 31) ||
        (int64_t)n_win * n_adp >= (1ll << 40))
        return 0;
    // every bucket chunked (the device plan's launches are k_align_chunk), with its span
    std::vector<int32_t> span((size_t)n_adp, -1);
    std::vector<int> used;
    std::vector<int32_t> bk_first(1, 0), bk_adp, bk_local;
    for (int b = 0; b < kNumBuckets; ++b) {
        const int nb = adps->count[b];
        if (!nb) continue;
        if (!chunkable(b, bucket_packed_ok(b, adps->lens[b], scr))) return 0;
        for (int kk = 0; kk < nb; ++kk) {
            const int L = adps->lens[b][kk];
            const int D = pcabi::sf::chunk_span(L, pcabi::sf::filter_threshold(L, threshold, scr), scr);
            if (D < 0) return 0;
            span[adps->ids[b][kk]] = D;
            bk_adp.push_back(adps->ids[b][kk]);
            bk_local.push_back(kk);
        }
        used.push_back(b);
        bk_first.push_back((int32_t)bk_adp.size());
    }
    std::vector<int> rows((size_t)n_adp, 0);
    for (int b = 0; b < kNumBuckets; ++b)
        for (int32_t id : adps->ids[b]) rows[id] = kBuckets[b].rpl;
    if (!sc->seed) sc->seed = pcabi_seed::create();
    {
        hmark("setup");
        const int rc = pcabi_seed::plan_ready(sc->seed, adps->hcodes.data(), adps->hoff.data(), adps->hlen.data(), n_adp,
                                              rows, scr, threshold, middle_seed_mode(), st);
        hmark("plan");
        if (rc < 0) return rc;
        if (rc == 0) return 0;
    }
    applied = true;
    const int n_bk = (int)used.size();
    const int64_t n = n_win;
    constexpr int kSlots = 16;                      // round slots held on the device (wrapped past)
    constexpr int kBatch = 3;                       // rounds queued per host check (later batches)
    // the first batch's rounds: as many as the previous call needed (its rounds up to the first one
    // that found nothing), 2 to 3. Data where round 2 finds nothing then skips a third round of ~35
    // empty launches, data with a third round pays no extra host round trip for it (r05y, in-process
    // A/B: the 20 kb scan 2.86 ms with 3 against 2.72 with 2, the 8 kb one 2.01 with 3 against 2.19
    // with 2).
    const int batch1 = std::min(kBatch, std::max(2, sc->rounds_hint));
    constexpr unsigned kGrid = 2048;                // blocks of the device-counted launches
    // ---- device buffers ----
    if (int rc = sc->q_cur.ensure(4 * (size_t)n * (kSlots + 1))) return rc;
    if (int rc = sc->q_start.ensure(4 * (size_t)n * (kSlots + 1))) return rc;
    if (int rc = sc->q_list.ensure(4 * 8 * (size_t)n * kSlots)) return rc;
    // the control block, laid out as its pinned host copy (one D2H per batch of rounds): round
    // counts [kSlots + 2], round flags [kSlots + 2], then int64 [slots, need, plan flag, need2,
    // shadow-arena bytes taken]
    constexpr size_t kCtlBytes = 4 * 2 * (kSlots + 2) + 8 * 5;
    if (int rc = sc->q_n.ensure(kCtlBytes)) return rc;
    if (int rc = sc->eoff.ensure(sizeof(int64_t) * n)) return rc;
    if (int rc = shadow_reserve(sc, h_win_len, n)) return rc;
    if (int rc = sc->soff.ensure(sizeof(int64_t) * n)) return rc;
    if (int rc = sc->slen.ensure(sizeof(int32_t) * n)) return rc;
    if (int rc = sc->pspan.ensure(sizeof(int32_t) * n_adp)) return rc;
    if (int rc = sc->plen.ensure(sizeof(int32_t) * n_adp)) return rc;
    if (int rc = sc->ptasks.ensure(sizeof(int32_t) * n_adp * kPlanC)) return rc;
    if (int rc = sc->pfill.ensure(sizeof(int32_t) * n_adp)) return rc;
    if (int rc = sc->pwoff.ensure(sizeof(int64_t) * n_adp)) return rc;
    if (int rc = sc->pcidx.ensure(sizeof(int32_t) * n_adp)) return rc;
    if (int rc = sc->phit.ensure(sizeof(int32_t) * n)) return rc;
    if (int rc = sc->phb.ensure(sizeof(int32_t) * 5 * n)) return rc;
    if (int rc = sc->pbest.ensure(sizeof(unsigned long long) * n * n_adp)) return rc;
    if (int rc = sc->pcbase.ensure(sizeof(int32_t) * n * n_adp)) return rc;
    if (int rc = sc->pcount.ensure(sizeof(int32_t) * ((size_t)n / 256 + 2))) return rc;
    if (int rc = sc->q_bk.ensure(4 * (bk_first.size() + 2 * bk_adp.size() + 2 * (size_t)n_bk + 16))) return rc;
    if (int rc = sc->q_misc2.ensure(64)) return rc;  // the second plan's slots and need
    if (int rc = sc->q_bk2.ensure(4 * (2 * (size_t)n_bk + 16))) return rc;
    if (int rc = sc->pcert.ensure(sizeof(int32_t) * n * n_adp)) return rc;
    if (sc->pucert.cap < sizeof(int32_t) * (size_t)n_adp) sc->h_ucert.clear();   // (re)allocated below
    if (int rc = sc->pucert.ensure(sizeof(int32_t) * n_adp)) return rc;
    int32_t *d_bk_first = (int32_t *)sc->q_bk.p, *d_bk_adp = d_bk_first + bk_first.size();
    int32_t *d_bk_local = d_bk_adp + bk_adp.size(), *d_bk_waves = d_bk_local + bk_adp.size();
    std::vector<int32_t> bk_host(bk_first);
    bk_host.insert(bk_host.end(), bk_adp.begin(), bk_adp.end());
    bk_host.insert(bk_host.end(), bk_local.begin(), bk_local.end());
    {   // the bucket tables, spans and lengths depend on the table and scoring only: up once per
        // change (three pageable copies cost ~20 us of every call otherwise)
        std::vector<int32_t> key(bk_host);
        key.insert(key.end(), span.begin(), span.end());
        key.insert(key.end(), adps->hlen.begin(), adps->hlen.end());
        const void *where[3] = {sc->q_bk.p, sc->pspan.p, sc->plen.p};
        if (key != sc->h_up || std::memcmp(where, sc->up_at, sizeof(where)) != 0) {
            HIP_TRY(hipMemcpyAsync(sc->q_bk.p, bk_host.data(), 4 * bk_host.size(), hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemcpyAsync(sc->pspan.p, span.data(), 4 * (size_t)n_adp, hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemcpyAsync(sc->plen.p, adps->hlen.data(), 4 * (size_t)n_adp, hipMemcpyHostToDevice, st));
            sc->h_up.swap(key);
            std::memcpy(sc->up_at, where, sizeof(where));
        }
    }
    double mean_len = sc->last_mean;
    if (h_win_len) {
        double tot = 0.0;
        for (int64_t k = 0; k < n; ++k) tot += h_win_len[k];
        mean_len = n ? tot / (double)n : 0.0;
    }
    hmark("bufs");
    const bool windows = middle_windows_on(mean_len);
    if (windows) {
        std::vector<int32_t> U;
        pcabi_seed::cert_bounds(sc->seed, U);
        if (U != sc->h_ucert) {                       // a new plan: its bounds up once (pageable: staged)
            HIP_TRY(hipMemcpyAsync(sc->pucert.p, U.data(), 4 * (size_t)n_adp, hipMemcpyHostToDevice, st));
            sc->h_ucert = U;
        }
    }
    int32_t *d_bk_waves2 = (int32_t *)sc->q_bk2.p;
    // q_misc: [0] slots, [1] need, [2] plan flag (int32), [3] the second plan's need (read with need)
    int64_t *d_slots2 = (int64_t *)sc->q_misc2.p;
    int64_t *d_slots = (int64_t *)((int32_t *)sc->q_n.p + 2 * (kSlots + 2)), *d_need = d_slots + 1, *d_need2 = d_slots + 3;
    unsigned long long *d_bump = (unsigned long long *)(d_slots + 4);
    int32_t *d_pflag = (int32_t *)(d_slots + 2);
    int32_t *d_n = (int32_t *)sc->q_n.p, *d_rflag = d_n + (kSlots + 2);
    // the plans' slot counts and needs start at 0 (q_n is uninitialised device memory: a round that
    // overflowed read a need its plan never wrote -- r05aa, a 10^18-byte growth request)
    HIP_TRY(hipMemsetAsync(d_slots, 0, 4 * sizeof(int64_t), st));
    // the reads' effective offsets start as the caller's; no shadow taken yet
    int64_t *eoff = (int64_t *)sc->eoff.p;
    HIP_TRY(hipMemcpyAsync(eoff, win_off, sizeof(int64_t) * n, hipMemcpyDeviceToDevice, st));
    // the bump starts past the arena's lead-in (kShadowLead bytes no copy uses: band loads that
    // reach a little before a read's start stay inside the allocation)
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)d_bump, (int)kShadowLead, 1, st));
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)((int32_t *)d_bump + 1), 0, 1, st));
    auto cur_of = [&](int slot) { return (int32_t *)sc->q_cur.p + (int64_t)slot * n; };
    auto start_of = [&](int slot) { return (int32_t *)sc->q_start.p + (int64_t)slot * n; };
    auto list_of = [&](int slot) { return (int32_t *)sc->q_list.p + (int64_t)slot * 8 * n; };
    // round 1: every window (in window order: a round's results do not depend on its order); its
    // read count d_n[0] = n is written by its k_round_views
    if (sc->q_slots_cap == 0) {
        sc->q_slots_cap = std::max<int64_t>(1 << 20, 4 * n);
        long long raw = 0, task = 0, slots = 0;     // tests: PCABI_MIDDLE_INIT_CAPS="raw,task,slots"
        if (const char *e = std::getenv("PCABI_MIDDLE_INIT_CAPS"))
            if (std::sscanf(e, "%lld,%lld,%lld", &raw, &task, &slots) == 3 && slots > 0) sc->q_slots_cap = slots;
    }
    const std::vector<std::pair<int64_t, int>> faults = middle_faults();
    const int serial_from = kMiddleSerialFrom;
    // the candidate-DP buckets' own threshold: in the window rounds (long reads) round 1's buckets
    // run serial too (r05aw in-process A/B, 20 kb: 2.512 -> 2.491 ms; 8 kb whole-read rounds keep
    // them side by side: 1.933 against 1.999 serial)
    const int dp_serial_from = windows ? 0 : serial_from;
    std::vector<char> fired(faults.size(), 0);
    int injected[kSlots + 1] = {};                  // per slot: the faults its last queueing injected
    const int64_t target = middle_plan_waves();
    const unsigned gn = (unsigned)std::min<int64_t>((n + 255) / 256, kGrid);
    std::vector<int32_t> out;                       // (round, 8 ints) of finished slots
    std::vector<int64_t> out_round;
    int64_t round_base = 0;                         // global round number of slot 0
    int slot = 0;                                   // next round to queue (slot index)
    int queued_to = 0;                              // rounds [0, queued_to) are queued
    auto queue_round = [&](int r) -> int {
        int fault = 0;
        for (size_t k = 0; k < faults.size(); ++k)
            if (!fired[k] && faults[k].first == round_base + r) {
                fault |= faults[k].second;
                fired[k] = 1;
            }
        injected[r] = fault;
        if (fault & 3) pcabi_seed::shrink_next(sc->seed, fault & 3);
        const bool serial = round_base + r >= serial_from;
        if (serial) pcabi_seed::serial_next(sc->seed);
        const int64_t slots_cap = (fault & 4) ? 64 : sc->q_slots_cap;
        if (int rc = sc->tw.ensure(sizeof(int32_t) * slots_cap)) return rc;
        if (int rc = sc->to.ensure(sizeof(int32_t) * slots_cap)) return rc;
        if (int rc = sc->tck.ensure(sizeof(int4) * slots_cap)) return rc;
        if (int rc = sc->pcand.ensure(sizeof(int32_t) * slots_cap)) return rc;
        if (int rc = sc->wa.ensure(sizeof(int32_t) * (slots_cap / 64 + 1))) return rc;
        if (int rc = sc->pres.ensure(sizeof(int32_t) * PCABI_NFIELDS * (size_t)slots_cap)) return rc;
        const int32_t *nr = d_n + r;
        const bool first = r == 0 && round_base == 0;  // round 1: the windows themselves
        const int32_t *start = first ? nullptr : start_of(r);
        const int32_t *cur = first ? nullptr : cur_of(r);
        MidProf &pf_ = sc->prof;                       // pcabi_scan_profile: marks of this round
        hipEvent_t pr_begin = nullptr, pr_seed[4] = {};
        if (pf_.on) {
            pf_.used = 0;
            pf_.spans.clear();
            if (int rc = sc->pprof.ensure(64)) return rc;
            HIP_TRY(hipMemsetAsync(sc->pprof.p, 0, 32, st));
            pr_begin = pf_.get();
            for (auto &e : pr_seed) e = pf_.get();
            if (!pr_begin || !pr_seed[3]) return fail(PCABI_E_DEVICE, "profile events");
            HIP_TRY(hipEventRecord(pr_begin, st));
            pcabi_seed::profile_events(sc->seed, pr_seed);
            if (int rc = pcabi_seed::profile_band_stats(sc->seed, true)) return rc;
        }
        struct SeedMarksOff {                          // the seed state never keeps this frame's events
            pcabi_seed::State *s;
            ~SeedMarksOff() {
                pcabi_seed::profile_events(s, nullptr);
                (void)pcabi_seed::profile_band_stats(s, false);
            }
        } seed_marks_off{sc->seed};
        auto pmark = [&](int phase, hipEvent_t from) -> hipEvent_t {   // a span from `from` to now
            if (!pf_.on) return nullptr;
            hipEvent_t e = pf_.get();
            if (!e || hipEventRecord(e, st) != hipSuccess) return nullptr;
            if (phase >= 0 && from) pf_.spans.emplace_back(phase, from, e);
            return e;
        };
        hipLaunchKernelGGL(k_round_views, dim3(first ? 1 : gn), dim3(256), 0, st, eoff, win_len, cur, nr,
                           (int64_t *)sc->soff.p, (int32_t *)sc->slen.p, d_n + r + 1, d_pflag, (int32_t *)sc->ptasks.p,
                           (int32_t *)sc->pfill.p, n_adp, first ? d_n : nullptr, (int32_t)n);
        const int64_t *dcand = nullptr;
        const unsigned long long *dcount = nullptr;
        const int32_t *sflags = nullptr;
        const int64_t *v_off = first ? eoff : (const int64_t *)sc->soff.p;
        const int32_t *v_len = first ? win_len : (const int32_t *)sc->slen.p;
        const int4 *vlist = nullptr;
        const int32_t *vcount = nullptr, *pmap = nullptr;
        int64_t vcap = 0;
        if (int rc = pcabi_seed::bounds_dev(sc->seed, codes, v_off, v_len, n, nr, n_adp, scr, &dcand, &dcount, &sflags,
                                            windows ? &vlist : nullptr, &vcount, &pmap, &vcap, st))
            return rc;
        if (pf_.on) {
            pf_.spans.emplace_back(kPhScan, pr_seed[0], pr_seed[1]);
            pf_.spans.emplace_back(kPhExpand, pr_seed[1], pr_seed[2]);
            pf_.spans.emplace_back(kPhBands, pr_seed[2], pr_seed[3]);
            (void)pmark(kPhCands, pr_seed[3]);
            hipLaunchKernelGGL(k_prof_round, dim3(64), dim3(256), 0, st, v_len, nr,
                               (unsigned long long *)sc->pprof.p);
        }
        const int64_t ncap = n * (int64_t)n_adp;
        // one candidate-DP plan into a set of task slots: WIN = the verified seeds' windows, else the
        // candidates' whole-read chunks (cmask != nullptr: only the candidates it flags)
        struct Plan {
            DeviceBuf *tw, *to, *tck, *cand, *wa, *res;
            int32_t *bk_waves;
            int64_t *slots, *need;
        };
        auto run_plan = [&](const Plan &pl, bool win, const int32_t *cmask) -> int {
            if (int rc = pl.tw->ensure(sizeof(int32_t) * slots_cap)) return rc;
            if (int rc = pl.to->ensure(sizeof(int32_t) * slots_cap)) return rc;
            if (int rc = pl.tck->ensure(sizeof(int4) * slots_cap)) return rc;
            if (int rc = pl.cand->ensure(sizeof(int32_t) * slots_cap)) return rc;
            if (int rc = pl.wa->ensure(sizeof(int32_t) * (slots_cap / 64 + 1))) return rc;
            if (int rc = pl.res->ensure(sizeof(int32_t) * PCABI_NFIELDS * (size_t)slots_cap)) return rc;
            const hipEvent_t pr_plan = pmark(-1, nullptr);
            if (win)
                hipLaunchKernelGGL(k_wplan_count, dim3(kGrid), dim3(256), 0, st, vlist, vcount, vcap, v_len, start,
                                   (int32_t *)sc->ptasks.p);
            else
                hipLaunchKernelGGL(k_plan_count, dim3(kGrid), dim3(256), 0, st, dcand, ncap, dcount, v_len, start,
                                   (const int32_t *)sc->pspan.p, (int32_t *)sc->ptasks.p, cmask);
            // the flagged candidates' whole reads (cmask): half the wave target, so their chunks are
            // 64 columns rather than 32 at a few hundred reads -- the lead-in (the adapter's span) is
            // recomputed per chunk (r05q: 20 kb 3.21-3.27 -> 3.13-3.22 ms; 8 kb keeps 4096)
            hipLaunchKernelGGL(k_plan_layout, dim3(1), dim3(256), 0, st, (const int32_t *)sc->ptasks.p, n_bk, d_bk_first,
                               d_bk_adp, d_bk_local, cmask ? std::max<int64_t>(1, target / 2) : target, slots_cap,
                               (int32_t *)sc->pcidx.p, (int64_t *)sc->pwoff.p,
                               (int32_t *)pl.wa->p, (int32_t *)pl.tw->p, pl.bk_waves, pl.slots, d_pflag, pl.need);
            if (win) {
                hipLaunchKernelGGL(k_wplan_place, dim3(kGrid), dim3(256), 0, st, vlist, vcount, vcap, v_off, v_len, start,
                                   (const int32_t *)sc->plen.p, (const int32_t *)sc->pspan.p, pmap, n,
                                   (const int64_t *)sc->pwoff.p, (int32_t *)sc->pfill.p, (int32_t *)pl.tw->p,
                                   (int32_t *)pl.to->p, (int4 *)pl.tck->p, (int32_t *)pl.cand->p, (const int64_t *)pl.slots);
            } else {
                hipLaunchKernelGGL(k_plan_place, dim3(kGrid), dim3(256), 0, st, dcand, ncap, dcount, v_len, start,
                                   (const int32_t *)sc->pspan.p, (const int32_t *)sc->pcidx.p,
                                   (const int64_t *)sc->pwoff.p, (int32_t *)sc->pfill.p, (int32_t *)pl.tw->p,
                                   (int32_t *)pl.to->p, (int4 *)pl.tck->p, (int32_t *)pl.cand->p,
                                   (const int64_t *)pl.slots, (int32_t *)sc->pcbase.p, cmask);
                hipLaunchKernelGGL(k_plan_fill, dim3(kGrid), dim3(256), 0, st, dcand, ncap, dcount, v_len,
                                   (const int32_t *)sc->pspan.p, (const int32_t *)sc->pcidx.p,
                                   (const int32_t *)sc->pcbase.p, (int32_t *)pl.tw->p, (int32_t *)pl.to->p,
                                   (int4 *)pl.tck->p, (int32_t *)pl.cand->p, (const int64_t *)pl.slots);
            }
            HIP_TRY(hipGetLastError());
            const hipEvent_t pr_dp = pmark(kPhPlan, pr_plan);
            KParams p{};
            p.codes = codes;
            p.win_off = v_off;
            p.win_len = v_len;
            p.n_win = n;
            p.out = (int32_t *)pl.res->p;
            p.out_stride = slots_cap;
            p.sc = scr;
            p.task_win = (const int32_t *)pl.tw->p;
            p.task_out = (const int32_t *)pl.to->p;
            p.wave_adp = (const int32_t *)pl.wa->p;
            p.task_chunk = (const int4 *)pl.tck->p;
            p.n_waves = kGrid;
            // two lanes per chunk task in the candidate-window rounds (long reads: the windows and the
            // certified-out candidates' whole reads), one lane in the whole-read rounds of shorter reads
            // (r05y / r05z in-process A/B: two lanes everywhere made the 20 kb scan 0.13 ms faster --
            // most of it the whole reads' 32-column chunks -- and the 8 kb one 0.08-0.09 ms slower)
            p.chunk_split = windows ? 2 : 0;
            // the run-tagged buckets (<= 28 rows) as one grouped launch (k_align_chunk_group), longest
            // rows first; the other buckets (and a lone run-tagged one) launch on their own
            const bool affine_dp = scr.go != scr.ge;
            ChunkGroupParams cg{};
            std::vector<int> singles;
            for (int k = n_bk - 1; k >= 0; --k) {
                const int b = used[k];
                const bool tg = bucket_pack_mode(b, adps->lens[b], scr) == 2;
                if (p.chunk_split == 0 && affine_dp && tg && kBuckets[b].kind == FAST &&
                    kBuckets[b].rpl <= kChunkGroupRpl && cg.n_seg < kMaxChunkSegs) {
                    ChunkSeg &sg = cg.seg[cg.n_seg++];
                    sg.adp_pad = adps->pad[b];
                    sg.adp_len = adps->len[b];
                    sg.adp_id = adps->id[b];
                    sg.dev_waves = pl.bk_waves + 2 * k;
                    sg.n_adp = adps->count[b];
                    sg.rpl = kBuckets[b].rpl;
                } else {
                    singles.push_back(k);
                }
            }
            if (cg.n_seg == 1) {                         // a lone bucket: its own launch, as before
                for (int k = 0; k < n_bk; ++k)
                    if (pl.bk_waves + 2 * k == cg.seg[0].dev_waves) singles.push_back(k);
                cg.n_seg = 0;
            }
            std::sort(singles.begin(), singles.end());
            const size_t n_launch = singles.size() + (cg.n_seg ? 1 : 0);
            ForkJoin fj;
            if (int rc = fj.begin(st, round_base + r >= dp_serial_from ? 1 : n_launch)) return rc;
            size_t li = 0;
            if (cg.n_seg) {
                cg.p = p;
                dispatch_chunk_group(cg, 4 * (unsigned)p.n_waves, fj.at(li++));
            }
            for (int k : singles) {
                const int b = used[k];
                p.adp_pad = adps->pad[b];
                p.adp_len = adps->len[b];
                p.adp_id = adps->id[b];
                p.n_adp = adps->count[b];
                p.rt = adps->rt[b];
                p.dev_waves = pl.bk_waves + 2 * k;
                // the packed buckets (36+ rows) of the whole-read rounds on the row-split core, two
                // lanes per chunk task (r06: 8 kb middle scan 1.74-1.86 -> 1.71-1.75 ms; their
                // one-lane waves hold 109-132 VGPRs, 3-4 waves per SIMD)
                const int split_keep = p.chunk_split;
                if (p.chunk_split == 0 && bucket_pack_mode(b, adps->lens[b], scr) != 2 && kBuckets[b].kind == FAST &&
                    kBuckets[b].rpl >= 36)
                    p.chunk_split = 2;
                const int rc_d = dispatch_chunk(b, p, affine_dp, fj.at(li++), bucket_pack_mode(b, adps->lens[b], scr) == 2);
                p.chunk_split = split_keep;
                if (rc_d) {
                    (void)fj.end();
                    return rc_d;
                }
            }
            if (int rc = fj.end()) return rc;
            HIP_TRY(hipGetLastError());
            if (pf_.on) {
                (void)pmark(kPhDp, pr_dp);
                hipLaunchKernelGGL(k_prof_cells, dim3(256), dim3(256), 0, st, (const int32_t *)pl.tw->p,
                                   (const int4 *)pl.tck->p, (const int32_t *)pl.cand->p, dcand, v_len,
                                   (const int32_t *)sc->plen.p, (const int64_t *)pl.slots,
                                   (unsigned long long *)sc->pprof.p);
                HIP_TRY(hipGetLastError());
            }
            return 0;
        };
        const Plan pw{&sc->tw, &sc->to, &sc->tck, &sc->pcand, &sc->wa, &sc->pres, d_bk_waves, d_slots, d_need};
        const Plan pf{&sc->tw2, &sc->to2, &sc->tck2, &sc->pcand2, &sc->wa2, &sc->pres2, d_bk_waves2, d_slots2, d_need2};
        auto merge_best = [&](const Plan &pl) {
            hipLaunchKernelGGL(k_merge_best, dim3(kGrid), dim3(256), 0, st, (const int32_t *)pl.tw->p,
                               (const int4 *)pl.tck->p, (const int32_t *)pl.cand->p, (const int32_t *)pl.res->p,
                               slots_cap, (const int64_t *)pl.slots, (unsigned long long *)sc->pbest.p);
        };
        auto merge_hit = [&](const Plan &pl, int pass, const int32_t *cmask, int want) {
            hipLaunchKernelGGL(k_merge_hit, dim3(kGrid), dim3(256), 0, st, dcand, (const int32_t *)pl.tw->p,
                               (const int4 *)pl.tck->p, (const int32_t *)pl.cand->p, (const int32_t *)pl.res->p,
                               slots_cap, (const int64_t *)pl.slots, (const unsigned long long *)sc->pbest.p,
                               threshold, pass, (int32_t *)sc->phit.p, (int32_t *)sc->phb.p, n, cmask, want);
        };
        if (!windows) {
            if (int rc = run_plan(pw, false, nullptr)) return rc;
            hipLaunchKernelGGL(k_merge_reset, dim3(kGrid), dim3(256), 0, st, (unsigned long long *)sc->pbest.p, dcount,
                               ncap, (int32_t *)sc->phit.p, (int32_t *)sc->phb.p, nr, nullptr);
            merge_best(pw);
            for (int pass = 0; pass < 2; ++pass) merge_hit(pw, pass, nullptr, 0);
        } else {
            // the windows; then per candidate the certificate (k_certify): its best window score is the
            // whole read's when it lies above every score an alignment without an exact piece, or
            // with more gap columns than the band, can reach; the other candidates (flagged) run
            // their whole reads in chunks, into the same merge
            if (int rc = run_plan(pw, true, nullptr)) return rc;
            hipLaunchKernelGGL(k_merge_reset, dim3(kGrid), dim3(256), 0, st, (unsigned long long *)sc->pbest.p, dcount,
                               ncap, (int32_t *)sc->phit.p, (int32_t *)sc->phb.p, nr, (int32_t *)sc->pcert.p);
            merge_best(pw);
            hipLaunchKernelGGL(k_certify, dim3(kGrid), dim3(256), 0, st, dcand, (const int32_t *)pw.tw->p,
                               (const int4 *)pw.tck->p, (const int32_t *)pw.cand->p, (const int32_t *)pw.res->p,
                               slots_cap, (const int64_t *)pw.slots, threshold, (const int32_t *)sc->pucert.p,
                               (unsigned long long *)sc->pbest.p, (int32_t *)sc->pcert.p, (int32_t *)sc->ptasks.p,
                               (int32_t *)sc->pfill.p, n_adp);
            const int32_t *flagged = (const int32_t *)sc->pcert.p;
            if (int rc = run_plan(pf, false, flagged)) return rc;
            merge_best(pf);
            for (int pass = 0; pass < 2; ++pass) {
                merge_hit(pw, pass, flagged, 0);      // certified candidates: their windows
                merge_hit(pf, pass, nullptr, 0);      // flagged candidates: their whole reads
            }
        }
        hipLaunchKernelGGL(k_round_count, dim3(gn), dim3(256), 0, st, (const int32_t *)sc->phb.p, nr, sflags, d_pflag,
                           (int32_t *)sc->pcount.p);
        hipLaunchKernelGGL(k_round_hits, dim3(gn), dim3(256), 0, st, (const int32_t *)sc->phb.p, n, nr, cur,
                           (const int32_t *)sc->pcount.p, list_of(r), d_n + r + 1, cur_of(r + 1), start_of(r + 1),
                           sflags, d_pflag, d_rflag + r, win_off, (const int64_t *)eoff, win_len, d_bump);
        hipLaunchKernelGGL(k_mask_list, dim3(4096), dim3(256), 0, st, codes, win_off, eoff, win_len, list_of(r),
                           d_n + r + 1, (uint8_t *)sc->shadow.p, shadow_rel(sc, codes), (fault & 8) ? (int64_t)-1 : sc->shadow_cap,
                           (const unsigned long long *)d_bump, d_rflag + r);
        HIP_TRY(hipGetLastError());
        if (g_debug) {                               // debugging only: a synchronisation per round
            int64_t c[5];
            if (int rc = pcabi_seed::debug_counts(sc->seed, c, st)) return rc;
            int32_t rn[2];
            int64_t sl = 0;
            HIP_TRY(hipMemcpy(rn, d_n + r, 8, hipMemcpyDeviceToHost));
            HIP_TRY(hipMemcpy(&sl, d_slots, 8, hipMemcpyDeviceToHost));
            std::fprintf(stderr, "[pcabi] middle round %lld: %d reads, band tasks %lld + %lld edge, %lld + %lld edge, "
                         "%lld candidates, %lld task slots, %d hits\n", (long long)(round_base + r), rn[0],
                         (long long)c[0], (long long)c[1], (long long)c[2], (long long)c[3], (long long)c[4],
                         (long long)sl, rn[1]);
            if (windows) {                           // the certificate's flagged candidates, their plan
                std::vector<int32_t> fl((size_t)std::max<int64_t>(1, std::min<int64_t>(c[4], ncap)));
                HIP_TRY(hipMemcpy(fl.data(), sc->pcert.p, 4 * fl.size(), hipMemcpyDeviceToHost));
                int64_t nf = 0, sl2 = 0;
                for (int32_t x : fl) nf += x != 0;
                HIP_TRY(hipMemcpy(&sl2, d_slots2, 8, hipMemcpyDeviceToHost));
                std::vector<int32_t> bw(2 * (size_t)n_bk), bw2(2 * (size_t)n_bk);
                HIP_TRY(hipMemcpy(bw.data(), d_bk_waves, 4 * bw.size(), hipMemcpyDeviceToHost));
                HIP_TRY(hipMemcpy(bw2.data(), d_bk_waves2, 4 * bw2.size(), hipMemcpyDeviceToHost));
                std::string w1, w2;
                for (int b = 0; b < n_bk; ++b) {
                    w1 += " " + std::to_string(bw[2 * b + 1]);
                    w2 += " " + std::to_string(bw2[2 * b + 1]);
                }
                std::fprintf(stderr, "[pcabi]   windows plan waves per bucket:%s; %lld flagged, whole-read plan %lld slots, "
                             "waves per bucket:%s\n", w1.c_str(), (long long)nf, (long long)sl2, w2.c_str());
            }
        }
        if (pf_.on) {                                // the round on its own: its spans and counters
            const hipEvent_t pr_end = pmark(-1, nullptr);
            int64_t cnt[3] = {};
            if (int rc = pcabi_seed::profile_counts(sc->seed, cnt, st)) return rc;   // (synchronises st)
            unsigned long long bst[8];
            if (int rc = pcabi_seed::band_stats(sc->seed, bst)) return rc;
            for (int i = 0; i < 8; ++i) pf_.band[i] += bst[i];
            unsigned long long u[4] = {};
            HIP_TRY(hipMemcpy(u, sc->pprof.p, sizeof(u), hipMemcpyDeviceToHost));
            float tot = 0.f;
            HIP_TRY(hipEventElapsedTime(&tot, pr_begin, pr_end));
            double named = 0.0;
            for (const auto &sp : pf_.spans) {
                float ms = 0.f;
                HIP_TRY(hipEventElapsedTime(&ms, std::get<1>(sp), std::get<2>(sp)));
                pf_.ms[std::get<0>(sp)] += ms;
                named += ms;
            }
            pf_.ms[kPhOther] += std::max(0.0, (double)tot - named);
            if (first) pf_.round1_ms += tot;
            pf_.rounds += 1;
            pf_.reads += (int64_t)u[0];
            pf_.bases += (int64_t)u[1];
            pf_.dp_tasks += (int64_t)u[2];
            pf_.dp_cells += (int64_t)u[3];
            pf_.raw += cnt[0];
            pf_.band_in += cnt[1];
            pf_.band_edge += cnt[2];
        }
        return 0;
    };
    // A round other than a call's first one is ~40 small launches and fork / join events whose
    // arguments depend only on the slot, the call's inputs and the scratch addresses: it is captured
    // once into a graph and replayed (r05: one host call instead of ~40 launches and ~10 event
    // operations, and the graph's ~1.6 us per kernel instead of ~2.7 back to back, tools/
    // launch_bench.hip; r05au: serial rounds too, the fork setting in the key). Not for rounds that
    // inject faults (tests), profile, debug or the legacy stream, and only rounds that run serial
    // (a capture would record another caller's launches on the shared side streams).
    const bool graphs_on = st != nullptr && faults.empty() && !g_debug && !sc->prof.on && sc->last_table == adps->serial;
    // (a table new to this scan -- e.g. the host API's per-call tables -- runs its rounds directly:
    // a capture pays only for a table the next call uses again)
    sc->last_table = adps->serial;
    auto run_round = [&](int r) -> int {
        const bool first = r == 0 && round_base == 0;
        const bool serial = round_base + r >= serial_from && round_base + r >= dp_serial_from;
        if (!graphs_on || first || !serial) return queue_round(r);
        std::vector<int64_t> key = {(int64_t)round_base, (int64_t)(intptr_t)codes, (int64_t)(intptr_t)win_off,
                                    (int64_t)(intptr_t)win_len, n, windows ? 1 : 0, (int64_t)(threshold * 1e6),
                                    scr.ma, scr.mi, scr.go, scr.ge, (int64_t)adps->serial, sc->q_slots_cap,
                                    sc->shadow_cap, (int64_t)(intptr_t)sc->shadow.p, target,
                                    (int64_t)g_buf_gen.load()};
        auto &g = sc->graphs[r & 31];
        if (g.exec && g.key == key) {
            HIP_TRY(hipGraphLaunch(g.exec, st));
            return 0;
        }
        if (g.exec) {
            (void)hipGraphExecDestroy(g.exec);
            g.exec = nullptr;
        }
        // captured on the second sight of a key: a caller alternating inputs (or switches) keeps
        // queueing directly instead of paying a capture per call
        if (g.seen != key) {
            g.seen = key;
            return queue_round(r);
        }
        // the round's buffers exist after round 1 of this call; a reallocation while capturing would
        // change the generation: the graph is then dropped and the round queued directly
        if (hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed) != hipSuccess) {
            (void)hipGetLastError();
            return queue_round(r);
        }
        const uint64_t gen0 = g_buf_gen.load();
        const int rc = queue_round(r);
        hipGraph_t graph = nullptr;
        const hipError_t ec = hipStreamEndCapture(st, &graph);
        if (rc) {
            if (graph) (void)hipGraphDestroy(graph);
            return rc;
        }
        hipGraphExec_t exec = nullptr;
        const bool ok = ec == hipSuccess && graph && g_buf_gen.load() == gen0 &&
                        hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) == hipSuccess;
        if (graph) (void)hipGraphDestroy(graph);
        if (!ok) {                                   // nothing of the round ran: queue it directly
            (void)hipGetLastError();
            if (exec) (void)hipGraphExecDestroy(exec);
            return queue_round(r);
        }
        g.exec = exec;
        g.key = key;
        key[16] = (int64_t)g_buf_gen.load();
        g.key = key;
        HIP_TRY(hipGraphLaunch(g.exec, st));
        return 0;
    };
    // pinned control block: round counts [kSlots + 2], flags [kSlots + 2], need / flag word / need2
    if (!sc->h_ctl) HIP_TRY(hipHostMalloc((void **)&sc->h_ctl, kCtlBytes + 8, hipHostMallocDefault));
    int32_t *h_n = sc->h_ctl, *h_flag = sc->h_ctl + (kSlots + 2);
    int64_t *h_nd = (int64_t *)(sc->h_ctl + 2 * (kSlots + 2));   // [0..4] as the device's; [5] round 1's segments
    h_nd[5] = -1;
    // every queued round's first spec entries come back with the counts (one synchronisation per
    // batch of rounds instead of two); a round with more hits fetches the rest after
    const int64_t spec = std::min<int64_t>(sc->spec_hits, n);
    {
        const size_t want = 8 * (size_t)spec * kBatch;
        if (want > sc->h_stage_cap) {
            if (sc->h_stage) HIP_TRY(hipHostFree(sc->h_stage));
            sc->h_stage = nullptr;
            sc->h_stage_cap = 0;
            HIP_TRY(hipHostMalloc((void **)&sc->h_stage, 4 * want, hipHostMallocDefault));
            sc->h_stage_cap = want;
        }
    }
    int64_t need = 0, need2 = 0, most_hits = 0;
    hmark("pre");
    for (int guard = 0;; ++guard) {
        if (guard > 10000) return fail(PCABI_E_DEVICE, "middle scan: rounds did not settle");
        // queue up to kBatch rounds from `slot`
        const int upto = std::min(slot + (round_base == 0 && slot == 0 ? batch1 : kBatch), kSlots);
        for (int r = slot; r < upto; ++r) {
            if (int rc = run_round(r)) return rc;
            hmark("round");
            if (r == 0 && round_base == 0)        // round 1's segment total (the next call's mean length)
                HIP_TRY(hipMemcpyAsync(h_nd + 5, pcabi_seed::seg_cum_dev(sc->seed) + n, sizeof(int64_t),
                                       hipMemcpyDeviceToHost, st));
        }
        queued_to = upto;
        hmark("queue");
        HIP_TRY(hipMemcpyAsync(sc->h_ctl, d_n, kCtlBytes, hipMemcpyDeviceToHost, st));   // counts, flags, needs
        for (int r = slot; r < queued_to; ++r)
            HIP_TRY(hipMemcpyAsync(sc->h_stage + 8 * (size_t)spec * (r - slot), list_of(r), 32 * (size_t)spec,
                                   hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        hmark("sync");
        need = h_nd[1];
        need2 = h_nd[3];
        // the first flagged round (nothing of it or after it was kept): grow, queue it again
        int bad = -1;
        for (int r = slot; r < queued_to && bad < 0; ++r)
            if (h_flag[r]) bad = r;
        int done_to = bad >= 0 ? bad : queued_to;    // rounds [slot, done_to) are final
        // the finished rounds' lists: the staged part, then (rarely) the rest
        for (int r = slot; r < done_to; ++r) {
            const int64_t nh = h_n[r + 1];
            if (!nh) continue;
            most_hits = std::max(most_hits, nh);
            const int32_t *st_r = sc->h_stage + 8 * (size_t)spec * (r - slot);
            out.insert(out.end(), st_r, st_r + 8 * (size_t)std::min(nh, spec));
            if (nh > spec) {
                const size_t old = out.size();
                out.resize(old + 8 * (size_t)(nh - spec));
                HIP_TRY(hipMemcpy(out.data() + old, list_of(r) + 8 * spec, 32 * (size_t)(nh - spec),
                                  hipMemcpyDeviceToHost));
            }
            out_round.insert(out_round.end(), (size_t)nh, round_base + r);
        }
        if (g_debug)
            for (int r = slot; r < queued_to; ++r)
                std::fprintf(stderr, "[pcabi] middle queued round %lld: %d reads, %d hits, flag %d\n",
                             (long long)(round_base + r), h_n[r], h_n[r + 1], h_flag[r]);
        if (bad >= 0) {
            g_requeues.fetch_add(1);
            g_requeue_flags.fetch_or(h_flag[bad] & 15);
            // the rounds queued behind it ran on no reads: their injected faults fire again
            for (size_t k = 0; k < faults.size(); ++k)
                if (faults[k].first > round_base + bad) fired[k] = 0;
            if (injected[bad]) {
                // an injected overflow (tests): the real buffers were large enough, queue it again
            } else if ((h_flag[bad] & 3) &&
                       !pcabi_seed::grow_after_overflow(sc->seed, h_flag[bad] & 1, (h_flag[bad] >> 1) & 1)) {
                return fail(PCABI_E_DEVICE, "middle scan: seed buffers past their limits");
            }
            if ((h_flag[bad] & 4) && !injected[bad]) {
                // need2: the whole-read plan's slots, written only by the window rounds' second plan
                const int64_t most = std::max(need, windows ? need2 : (int64_t)0);
                sc->q_slots_cap = std::max<int64_t>(2 * sc->q_slots_cap, most + most / 4);
            }
            // the shadow arena was too small for the round's first hits: a larger one (the copies
            // made so far move with it), allocations go on past the old end
            if ((h_flag[bad] & 8) && h_nd[4] > sc->shadow_cap)
                if (int rc = shadow_grow(sc, codes, win_off, eoff, n, h_nd[4], d_bump, st)) return rc;
            HIP_TRY(hipStreamSynchronize(st));
            slot = bad;
            continue;
        }
        if (h_n[queued_to] == 0) {                   // the last queued round found no hit
            // the rounds this call needed: up to the first that found nothing (the next call's first batch)
            int need_r = queued_to;
            for (int r = slot; r < queued_to; ++r)
                if (h_n[r + 1] == 0) {
                    need_r = r + 1;
                    break;
                }
            sc->rounds_hint = (int)std::min<int64_t>(round_base + need_r, 64);
            break;
        }
        slot = queued_to;
        if (slot == kSlots) {                        // wrap: the next round's reads to slot 0
            HIP_TRY(hipMemcpyAsync(cur_of(0), cur_of(kSlots), 4 * (size_t)h_n[kSlots], hipMemcpyDeviceToDevice, st));
            HIP_TRY(hipMemcpyAsync(start_of(0), start_of(kSlots), 4 * (size_t)h_n[kSlots], hipMemcpyDeviceToDevice, st));
            HIP_TRY(hipMemcpyAsync(d_n, d_n + kSlots, 4, hipMemcpyDeviceToDevice, st));
            round_base += kSlots;
            slot = 0;
        }
    }
    HIP_TRY(hipStreamSynchronize(st));
    // the next call stages as many hits per round as this one's busiest round had (+ 25 %), and
    // takes its mean read length from this call's round-1 segments
    hmark("end");
    sc->spec_hits = std::max<int64_t>(4096, most_hits + most_hits / 4);
    if (h_nd[5] >= 0 && n > 0) sc->last_mean = (double)h_nd[5] * pcabi_seed::seg_positions() / (double)n;
    // (round, read) order: per read the reference's discovery order. The rounds come in order and
    // each round's list in read order (k_round_hits' ordered compaction): only checked here
    const int64_t total = (int64_t)out_round.size();
    for (int64_t j = 1; j < total; ++j)
        if (out_round[j] == out_round[j - 1] && out[8 * j] <= out[8 * (j - 1)])
            return fail(PCABI_E_DEVICE, "middle scan: a round's hit list is out of read order");
    for (int64_t q = 0; q < total && q < cap; ++q) {
        const int32_t *o = out.data() + 8 * q;
        hits[0 * cap + q] = o[0];
        hits[1 * cap + q] = o[1];
        hits[2 * cap + q] = o[2];
        hits[3 * cap + q] = o[2] == -1 ? 0 : o[3] + 1;
        hits[4 * cap + q] = o[4];
        hits[5 * cap + q] = o[5];
    }
    return total;
}

}  // namespace

extern "C" {

int pcabi_set_side_streams(int on) {
    const int prev = side_streams_on() ? 1 : 0;
    if (on >= 0) g_side_on.store(on ? 1 : 0);
    return prev;
}

int pcabi_stream_side_streams(void *stream, int on) {
    const hipStream_t st = (hipStream_t)stream;
    std::lock_guard<std::mutex> g(g_stream_side_mu);
    for (size_t k = 0; k < g_stream_side.size(); ++k)
        if (g_stream_side[k].first == st) {
            const int prev = g_stream_side[k].second;
            if (on < 0) g_stream_side.erase(g_stream_side.begin() + (long)k);
            else g_stream_side[k].second = on ? 1 : 0;
            return prev;
        }
    if (on >= 0) g_stream_side.emplace_back(st, on ? 1 : 0);
    return -1;
}

int32_t pcabi_scan_profile(pcabi_scan *s, int32_t mode, double *out, int32_t n_out) {
    if (!s || mode < 0 || mode > 2 || n_out < 0 || (n_out && !out)) return fail(PCABI_E_ARG, "bad arguments");
    MidProf &p = s->prof;
    if (mode == 1) {
        std::fill(p.ms, p.ms + kPhases, 0.0);
        p.rounds = p.reads = p.bases = p.raw = p.band_in = p.band_edge = p.dp_tasks = p.dp_cells = 0;
        p.round1_ms = 0.0;
        std::fill(p.band, p.band + 8, 0ull);
    }
    if (mode != 2) p.on = mode == 1;
    const int32_t nv = kPhases + 9 + 8 + 2;
    const double v[nv] = {p.ms[0], p.ms[1], p.ms[2], p.ms[3], p.ms[4], p.ms[5], p.ms[6],
                          (double)p.rounds, (double)p.reads, (double)p.bases, (double)p.raw,
                          (double)p.band_in, (double)p.band_edge, (double)p.dp_tasks, (double)p.dp_cells,
                          p.round1_ms,
                          (double)p.band[0], (double)p.band[1], (double)p.band[2], (double)p.band[3],
                          (double)p.band[4], (double)p.band[5], (double)p.band[6], (double)p.band[7],
                          (double)(s->seed ? pcabi_seed::band_e(s->seed, 0) : 0),
                          (double)(s->seed ? pcabi_seed::band_e(s->seed, 1) : 0)};
    const int32_t k = std::min<int32_t>(n_out, nv);
    for (int32_t i = 0; i < k; ++i) out[i] = v[i];
    return nv;
}

int64_t pcabi_middle_requeues(int32_t *flags_seen) {
    if (flags_seen) *flags_seen = g_requeue_flags.load();
    return g_requeues.load();
}

int64_t pcabi_middle_scan_dev(pcabi_scan *sc, const uint8_t *codes, const int64_t *win_off, const int32_t *win_len,
                              const int32_t *h_win_len, int64_t n_win, int match, int mismatch, int gap_open,
                              int gap_extend, double threshold, int32_t *hits, int64_t cap, void *stream) {
    if (!sc || n_win < 0 || cap < 0) return fail(PCABI_E_ARG, "bad arguments");
    if (!(threshold > 0.0))
        return fail(PCABI_E_ARG, "middle threshold must be > 0 (the reference's loop never ends otherwise)");
    const hipStream_t st = (hipStream_t)stream;
    const int32_t n_adp = sc->adps->n_adp;
    if (n_win == 0 || n_adp == 0) return 0;
    HostMarks hm;
    struct MarksOff {
        ~MarksOff() { g_hm = nullptr; }
    } marks_off;
    g_hm = hm.on ? &hm : nullptr;
    hmark("entry");
    // the layout of the scan's table that serves this scoring on these reads (adapters_for: any
    // scoring the reference accepts, any read length), for the duration of the call
    struct TableSwap {
        pcabi_scan *s;
        const pcabi_adapters *own;
        ~TableSwap() { s->adps = own; }
    } swap_back{sc, sc->adps};
    std::vector<int32_t> h_len_copy;
    auto host_lengths = [&]() -> int {              // lengths only on the device: one small copy
        if (h_win_len) return 0;
        h_len_copy.resize((size_t)n_win);
        HIP_TRY(hipMemcpyAsync(h_len_copy.data(), win_len, 4 * (size_t)n_win, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        h_win_len = h_len_copy.data();
        return 0;
    };
    const pcabi::Scoring scoring{match, mismatch, gap_open, gap_extend};
    {
        // the longest window decides the layout only when the table may not serve every length
        // (a scoring without a span bound): otherwise no length needs to come to the host
        int32_t longest = INT32_MAX / 2;
        if (!layout_serves(sc->adps, scoring, longest)) {
            if (int rc = host_lengths()) return rc;
            longest = 0;
            for (int64_t k = 0; k < n_win; ++k) longest = std::max(longest, h_win_len[k]);
        }
        const pcabi_adapters *use = nullptr;
        if (int rc = adapters_for(sc->adps, scoring, longest, &use)) return rc;
        sc->adps = use;
    }
    {
        bool applied = false;
        const int64_t r = middle_device_rounds(sc, codes, win_off, win_len, h_win_len, n_win, scoring, threshold, hits,
                                               cap, st, applied);
        if (applied || r < 0) return r;
    }
    if (int rc = host_lengths()) return rc;
    // input-preserving masking (k_mask_list): effective offsets, shadows allocated on the host here
    if (int rc = sc->eoff.ensure(sizeof(int64_t) * n_win)) return rc;
    if (int rc = sc->shadow_zero.ensure(sizeof(unsigned long long))) return rc;
    if (int rc = shadow_reserve(sc, h_win_len, n_win)) return rc;
    int64_t *eoff = (int64_t *)sc->eoff.p;
    HIP_TRY(hipMemcpyAsync(eoff, win_off, sizeof(int64_t) * n_win, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemsetAsync(sc->shadow_zero.p, 0, sizeof(unsigned long long), st));
    std::vector<char> shadowed((size_t)n_win, 0);
    int64_t sh_bump = kShadowLead;                  // arena bytes taken (the lead-in first)
    int64_t n_hits = 0;
    std::vector<int32_t> cur, nxt, nxt_start, hm_list, lens;
    std::vector<int32_t> hb;
    std::vector<int64_t> toff;
    std::vector<int16_t> h16;                       // round-1 filter scores (bounds for later rounds)
    std::vector<int32_t> pos1((size_t)n_win, 0);    // read -> round-1 position
    bool filt_round1 = false;
    bool seeded = false;                            // round 1 took its bounds from seeds
    // Round 1 visits the reads longest first: lanes of a wave (and tiles) then run near-equal
    // column counts (read lengths are log-normal; unsorted, a wave would idle ~2/3 of its lanes).
    cur.resize((size_t)n_win);
    for (int64_t k = 0; k < n_win; ++k) cur[k] = (int32_t)k;
    {
        // longest first, ties in read order: a stable LSD radix sort on (longest - length), 11-bit
        // digits over the bits the longest length needs (two passes up to 4 M bases)
        int32_t longest = 0;
        for (int64_t k = 0; k < n_win; ++k) longest = std::max(longest, h_win_len[k]);
        int bits = 1;
        while (bits < 31 && (1u << bits) <= (uint32_t)longest) ++bits;
        std::vector<int32_t> tmp((size_t)n_win);
        std::vector<uint32_t> key((size_t)n_win), ktmp((size_t)n_win);
        for (int64_t k = 0; k < n_win; ++k) key[k] = (uint32_t)(longest - std::max(h_win_len[k], 0));
        constexpr int kDig = 11;
        std::vector<int64_t> cnt((size_t)1 << kDig);
        for (int sh = 0; sh < bits; sh += kDig) {
            std::fill(cnt.begin(), cnt.end(), 0);
            for (int64_t k = 0; k < n_win; ++k) ++cnt[(key[k] >> sh) & ((1u << kDig) - 1)];
            int64_t run = 0;
            for (int64_t &c : cnt) { const int64_t x = c; c = run; run += x; }
            for (int64_t k = 0; k < n_win; ++k) {
                const int64_t d = cnt[(key[k] >> sh) & ((1u << kDig) - 1)]++;
                tmp[d] = cur[k];
                ktmp[d] = key[k];
            }
            cur.swap(tmp);
            key.swap(ktmp);
        }
    }
    for (int round = 0;; ++round) {
        const int64_t n = (int64_t)cur.size();
        const int64_t *v_off = eoff;
        const int32_t *v_len = win_len;
        lens.resize((size_t)n);
        {
            for (int64_t k = 0; k < n; ++k) lens[k] = h_win_len[cur[k]];
            if (int rc = sc->idx.ensure(sizeof(int32_t) * n)) return rc;
            if (int rc = sc->start.ensure(sizeof(int32_t) * n)) return rc;
            if (int rc = sc->soff.ensure(sizeof(int64_t) * n)) return rc;
            if (int rc = sc->slen.ensure(sizeof(int32_t) * n)) return rc;
            HIP_TRY(hipMemcpyAsync(sc->idx.p, cur.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
            if (round > 0)
                HIP_TRY(hipMemcpyAsync(sc->start.p, nxt_start.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_gather_views, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, eoff, win_len,
                               (const int32_t *)sc->idx.p, n, (int64_t *)sc->soff.p, (int32_t *)sc->slen.p);
            v_off = (const int64_t *)sc->soff.p;
            v_len = (const int32_t *)sc->slen.p;
        }
        // tiles of this round's windows (the score filter and the full cross product read them)
        int32_t max_len = 0;
        for (int32_t l : lens) max_len = std::max(max_len, l);
        if (int rc = sc->hits.ensure(sizeof(int32_t) * 5 * (size_t)n)) return rc;
        bool tiled = false;
        auto make_tiles = [&]() -> int {
            if (tiled) return 0;
            toff.assign((size_t)((n + 255) / 256 + 1), 0);
            int64_t max_nq = 0;
            const int64_t nd = tile_layout(lens.data(), n, toff.data(), &max_nq);
            if (int rc = sc->toff.ensure(sizeof(int64_t) * toff.size())) return rc;
            if (int rc = sc->tiles.ensure(sizeof(uint32_t) * (size_t)nd)) return rc;
            HIP_TRY(hipMemcpyAsync(sc->toff.p, toff.data(), sizeof(int64_t) * toff.size(), hipMemcpyHostToDevice, st));
            launch_tiles(codes, v_off, v_len, n, (const int64_t *)sc->toff.p, max_nq, (uint32_t *)sc->tiles.p, st);
            tiled = true;
            return 0;
        };
        int filt = 0;
        if (middle_filter_on() && (round == 0 || filt_round1)) {
            filt = filtered_first_hits(sc, codes, v_off, v_len, lens.data(), n, round == 0 ? nullptr : nxt_start.data(),
                                       round == 0 ? nullptr : (const int32_t *)sc->start.p, max_len,
                                       cur.data(), h16, n_win, pos1,
                                       pcabi::Scoring{match, mismatch, gap_open, gap_extend}, threshold, hb, seeded,
                                       make_tiles, st);
            if (round == 0) {
                // the bound needs masked bases (N) to never match an adapter base
                filt_round1 = filt > 0 && !sc->adps->has_n;
                for (int64_t k = 0; k < n; ++k) pos1[cur[k]] = (int32_t)k;
            }
            if (filt < 0) return filt;
        }
        if (!filt) {
            const auto t0 = std::chrono::steady_clock::now();
            if (int rc = make_tiles()) return rc;
            if (g_debug) HIP_TRY(hipStreamSynchronize(st));
            const auto t1 = std::chrono::steady_clock::now();
            if (int rc = sc->res.ensure(sizeof(int32_t) * PCABI_NFIELDS * (size_t)n * n_adp)) return rc;
            if (int rc = pcabi_align_cross_dev((const uint32_t *)sc->tiles.p, (const int64_t *)sc->toff.p, v_len, n,
                                               max_len, sc->adps, match, mismatch, gap_open, gap_extend,
                                               (int32_t *)sc->res.p, n * n_adp, stream))
                return rc;
            if (g_debug) {
                HIP_TRY(hipStreamSynchronize(st));
                const auto t2 = std::chrono::steady_clock::now();
                std::fprintf(stderr, "[pcabi] middle host round %d: tiles %.3f ms, cross product %.3f ms (%lld x %d, longest %d)\n",
                             round, std::chrono::duration<double, std::milli>(t1 - t0).count(),
                             std::chrono::duration<double, std::milli>(t2 - t1).count(), (long long)n, n_adp, max_len);
            }
            hipLaunchKernelGGL(k_first_hit, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                               (const int32_t *)sc->res.p, n * n_adp, n, n_adp, threshold,
                               round == 0 ? nullptr : (const int32_t *)sc->start.p, (int32_t *)sc->hits.p, n);
            HIP_TRY(hipGetLastError());
            hb.resize((size_t)(5 * n));
            HIP_TRY(hipMemcpyAsync(hb.data(), sc->hits.p, sizeof(int32_t) * 5 * n, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
        }
        nxt.clear(); nxt_start.clear(); hm_list.clear();
        for (int64_t k = 0; k < n; ++k) {
            const int32_t a = hb[k];
            if (a < 0) continue;
            const int32_t r = cur[k];
            const int32_t rs = hb[n + k], re = hb[2 * n + k];
            const int32_t rend = rs == -1 ? 0 : re + 1;
            if (n_hits < cap) {
                hits[0 * cap + n_hits] = r;
                hits[1 * cap + n_hits] = a;
                hits[2 * cap + n_hits] = rs;
                hits[3 * cap + n_hits] = rend;
                hits[4 * cap + n_hits] = hb[3 * n + k];
                hits[5 * cap + n_hits] = hb[4 * n + k];
            }
            ++n_hits;
            nxt.push_back(r);
            nxt_start.push_back(a);
            if (rend > rs) {                       // k_mask_list's entry; a read's first: its shadow
                int32_t unit = 0;
                if (!shadowed[r]) {
                    shadowed[r] = 1;
                    unit = (int32_t)(sh_bump / 16) + 1;
                    sh_bump += (std::max(h_win_len[r], 0) + 16 + 15) & ~(int64_t)15;
                }
                const int32_t e[8] = {r, a, rs, re, 0, 0, 0, unit};
                hm_list.insert(hm_list.end(), e, e + 8);
            }
        }
        if (g_debug)
            std::fprintf(stderr, "[pcabi] middle host round %d: %lld reads, %zu hits (%s)\n", round, (long long)n,
                         nxt.size(), filt ? "filtered" : "cross product");
        if (nxt.empty()) break;
        if (!hm_list.empty()) {
            if (sh_bump > sc->shadow_cap) {           // grow first: this round's copies go past the end
                if (sh_bump > kShadowMax) return fail(PCABI_E_NOMEM, "middle scan: shadow arena past its limit");
                if (int rc = shadow_grow(sc, codes, win_off, eoff, n_win, sh_bump, nullptr, st)) return rc;
            }
            const int32_t m = (int32_t)(hm_list.size() / 8);
            if (int rc = sc->mwin.ensure(sizeof(int32_t) * (hm_list.size() + 1))) return rc;
            HIP_TRY(hipMemcpyAsync(sc->mwin.p, hm_list.data(), sizeof(int32_t) * hm_list.size(), hipMemcpyHostToDevice, st));
            int32_t *d_m = (int32_t *)sc->mwin.p + hm_list.size();
            HIP_TRY(hipMemcpyAsync(d_m, &m, sizeof(int32_t), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_mask_list, dim3((unsigned)std::min<int32_t>(m, 1024)), dim3(256), 0, st, codes, win_off,
                               eoff, win_len, (const int32_t *)sc->mwin.p, d_m, (uint8_t *)sc->shadow.p,
                               shadow_rel(sc, codes), sc->shadow_cap, (const unsigned long long *)sc->shadow_zero.p,
                               (int32_t *)nullptr);
            HIP_TRY(hipGetLastError());
        }
        // host vectors uploaded above must stay intact until the copies ran
        HIP_TRY(hipStreamSynchronize(st));
        // next round: the reads that just hit, longest first, each from the adapter that hit
        std::vector<int32_t> perm(nxt.size());
        for (size_t k = 0; k < perm.size(); ++k) perm[k] = (int32_t)k;
        std::stable_sort(perm.begin(), perm.end(),
                         [&](int32_t x, int32_t y) { return h_win_len[nxt[x]] > h_win_len[nxt[y]]; });
        cur.resize(perm.size());
        std::vector<int32_t> st_sorted(perm.size());
        for (size_t k = 0; k < perm.size(); ++k) { cur[k] = nxt[perm[k]]; st_sorted[k] = nxt_start[perm[k]]; }
        nxt_start.swap(st_sorted);
    }
    return n_hits;
}

int pcabi_middle_cuts_host(int device, const int32_t *hits, int64_t hit_stride, int64_t n_hits, int64_t n_reads,
                           const uint8_t *bad_start, const uint8_t *bad_end, int32_t n_adp, int good_side,
                           int bad_side, int64_t *cut_off, int64_t *cuts) {
    if (device < 0 || device >= 16) return fail(PCABI_E_ARG, "bad device index");
    if (n_hits < 0 || n_reads < 0 || n_adp < 0 || hit_stride < n_hits) return fail(PCABI_E_ARG, "bad counts");
    for (int64_t k = 0; k < n_hits; ++k)
        if (hits[k] < 0 || hits[k] >= n_reads || hits[hit_stride + k] < 0 || hits[hit_stride + k] >= n_adp)
            return fail(PCABI_E_ARG, "hit read / adapter index out of range");
    Engine &e = g_engines[device];
    std::lock_guard<std::mutex> lock(e.mu);
    if (int rc = engine_init(e, device)) return rc;
    HIP_TRY(hipSetDevice(device));
    const size_t hb = sizeof(int32_t) * 4 * (size_t)std::max<int64_t>(n_hits, 1);
    const size_t fb = 2 * (size_t)std::max<int32_t>(n_adp, 1);
    const size_t ob = sizeof(int64_t) * ((size_t)n_reads + 1), cb = sizeof(int64_t) * 2 * (size_t)std::max<int64_t>(n_hits, 1);
    if (int rc = e.bc.ensure(hb + fb + ob + cb + 64)) return rc;
    char *p = (char *)e.bc.p;
    int32_t *d_hits = (int32_t *)p;
    uint8_t *d_flags = (uint8_t *)(p + hb);
    int64_t *d_off = (int64_t *)(((uintptr_t)(p + hb + fb) + 7) & ~(uintptr_t)7);
    int64_t *d_cuts = d_off + n_reads + 1;
    // the four used rows (read, adapter, read_start, read_end), packed with stride n_hits
    for (int f = 0; f < 4 && n_hits; ++f)
        HIP_TRY(hipMemcpyAsync(d_hits + f * n_hits, hits + f * hit_stride, sizeof(int32_t) * (size_t)n_hits,
                               hipMemcpyHostToDevice, e.stream));
    if (n_adp) {
        HIP_TRY(hipMemcpyAsync(d_flags, bad_start, (size_t)n_adp, hipMemcpyHostToDevice, e.stream));
        HIP_TRY(hipMemcpyAsync(d_flags + n_adp, bad_end, (size_t)n_adp, hipMemcpyHostToDevice, e.stream));
    }
    if (int rc = pcabi_middle_cuts_dev(d_hits, n_hits, n_hits, n_reads, d_flags, d_flags + n_adp, good_side, bad_side,
                                       d_off, d_cuts, e.stream))
        return rc;
    HIP_TRY(hipMemcpyAsync(cut_off, d_off, sizeof(int64_t) * ((size_t)n_reads + 1), hipMemcpyDeviceToHost, e.stream));
    if (n_hits)
        HIP_TRY(hipMemcpyAsync(cuts, d_cuts, sizeof(int64_t) * 2 * (size_t)n_hits, hipMemcpyDeviceToHost, e.stream));
    HIP_TRY(hipStreamSynchronize(e.stream));
    return 0;
}

int pcabi_end_trim_dev(const int32_t *start_res, int64_t start_stride, int32_t n_sa,
                       const int32_t *end_res, int64_t end_stride, int32_t n_ea, int64_t n_read,
                       int end_size, int extra_trim, double end_threshold, int min_trim_size,
                       int32_t *start_trim, int32_t *end_trim, uint8_t *start_hit, uint8_t *end_hit,
                       void *stream) {
    if (n_read <= 0) return 0;
    const unsigned blocks = (unsigned)((n_read + 63) / 64);
    hipLaunchKernelGGL(k_end_trim, dim3(blocks), dim3(256), 0, (hipStream_t)stream, start_res, start_stride,
                       n_sa, end_res, end_stride, n_ea, n_read, end_size, extra_trim, end_threshold,
                       min_trim_size, start_trim, end_trim, start_hit, end_hit);
    HIP_TRY(hipGetLastError());
    return 0;
}

int pcabi_trim_views_dev(const int64_t *read_off, const int32_t *read_len, const int32_t *start_trim,
                         const int32_t *end_trim, int64_t n_read, int64_t *view_off, int32_t *view_len, void *stream) {
    if (n_read < 0) return fail(PCABI_E_ARG, "bad read count");
    if (n_read == 0) return 0;
    hipLaunchKernelGGL(k_trim_views, dim3((unsigned)std::min<int64_t>((n_read + 255) / 256, 4096)), dim3(256), 0,
                       (hipStream_t)stream, read_off, read_len, start_trim, end_trim, n_read, view_off, view_len);
    HIP_TRY(hipGetLastError());
    return 0;
}

int pcabi_best_full_identity_dev(const int32_t *res, int64_t stride, int64_t n_win, int32_t n_adp,
                                 double *best, void *stream) {
    if (n_adp <= 0 || n_win <= 0) return 0;
    hipLaunchKernelGGL(k_best_full_id, dim3((unsigned)n_adp), dim3(256), 0, (hipStream_t)stream, res, stride,
                       n_win, best);
    HIP_TRY(hipGetLastError());
    return 0;
}

int pcabi_barcode_call_dev(const int32_t *start_res, int64_t start_stride, const int32_t *start_slot_adp,
                           const int32_t *start_slot_name, int32_t n_start_slots, const int32_t *end_res,
                           int64_t end_stride, const int32_t *end_slot_adp, const int32_t *end_slot_name,
                           int32_t n_end_slots, int64_t n_read, double barcode_threshold, double barcode_diff,
                           int require_two, int32_t *call, double *scores, void *stream) {
    if (n_read < 0 || n_start_slots < 0 || n_end_slots < 0) return fail(PCABI_E_ARG, "negative count");
    if (n_read == 0) return 0;
    const BcSide st{start_res, start_stride, start_slot_adp, start_slot_name, n_start_slots};
    const BcSide en{end_res, end_stride, end_slot_adp, end_slot_name, n_end_slots};
    hipLaunchKernelGGL(k_barcode_call, dim3((unsigned)((n_read + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       st, en, n_read, barcode_threshold, barcode_diff, require_two, call, scores);
    HIP_TRY(hipGetLastError());
    return 0;
}

int pcabi_compat_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *seq_off,
                      const int32_t *seq_len, int64_t n_seq, const int32_t *pair_i, const int32_t *pair_j,
                      int64_t n_pairs, int32_t *flags) {
    if (n_seq < 0 || n_pairs < 0) return fail(PCABI_E_ARG, "negative count");
    if (n_seq > INT32_MAX) return fail(PCABI_E_ARG, "too many sequences");
    // row 0 = the longer sequence (make_stringSet, compatibility.cpp:17-28: ties keep seq1 first)
    std::vector<int32_t> tw, ta;
    std::vector<int64_t> at;           // result slot of each task
    tw.reserve((size_t)n_pairs);
    ta.reserve((size_t)n_pairs);
    for (int64_t t = 0; t < n_pairs; ++t) {
        const int32_t i = pair_i[t], j = pair_j[t];
        if (i < 0 || i >= n_seq || j < 0 || j >= n_seq) return fail(PCABI_E_ARG, "pair index out of range");
        const bool swap = seq_len[i] < seq_len[j];
        const int32_t lo = swap ? j : i, sh = swap ? i : j;
        flags[t] = 0;                  // empty sequences: no alignment (the reference is undefined)
        if (seq_len[lo] == 0 || seq_len[sh] == 0) continue;
        if (seq_len[sh] > pcabi::MAX_STRIPED_LEN)
            return fail(PCABI_E_ARG, "check_compatibility: the shorter sequence exceeds " +
                                         std::to_string(pcabi::MAX_STRIPED_LEN) + " bases");
        tw.push_back(lo);
        ta.push_back(sh);
        at.push_back(t);
    }
    if (tw.empty()) return 0;
    std::vector<uint8_t> acodes;
    std::vector<int32_t> aoff((size_t)n_seq), alen((size_t)n_seq);
    for (int64_t k = 0; k < n_seq; ++k) {
        aoff[k] = (int32_t)acodes.size();
        alen[k] = std::max<int32_t>(1, std::min<int32_t>(seq_len[k], pcabi::MAX_STRIPED_LEN));
        for (int32_t q = 0; q < alen[k]; ++q) acodes.push_back(seq_len[k] > 0 ? codes[seq_off[k] + q] : 0);
    }
    std::vector<int32_t> got(tw.size());
    // compatibility.h:5-8: Score<int, Simple>(match 2, mismatch -1, gap -1) -> linear gaps
    if (int rc = align_host_impl(device, codes, codes_len, seq_off, seq_len, n_seq, acodes.data(), aoff.data(),
                                 alen.data(), (int32_t)n_seq, tw.data(), ta.data(), (int64_t)tw.size(), 2, -1, -1, -1,
                                 nullptr, got.data(), true))
        return rc;
    for (size_t k = 0; k < tw.size(); ++k) flags[at[k]] = got[k];
    return 0;
}

int pcabi_compat_all_vs_all_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *seq_off,
                                 const int32_t *seq_len, int64_t n_seq, int32_t *mat) {
    if (n_seq < 0) return fail(PCABI_E_ARG, "negative count");
    if (n_seq > 46340) return fail(PCABI_E_ARG, "too many sequences for one matrix");
    const int64_t n = n_seq;
    for (int64_t k = 0; k < n; ++k) mat[k * n + k] = -1;   // every other entry is written below
    if (n < 2) return 0;
    bool cross_ok = true;
    for (int64_t k = 0; k < n; ++k) cross_ok = cross_ok && seq_len[k] >= 1 && seq_len[k] <= pcabi::MAX_STRIPED_LEN;
    if (!cross_ok) {
        // some sequence cannot be a DP row set: explicit pairs (the longer is never a row set)
        std::vector<int32_t> pi, pj;
        for (int64_t i = 0; i < n; ++i)
            for (int64_t j = i + 1; j < n; ++j) { pi.push_back((int32_t)i); pj.push_back((int32_t)j); }
        std::vector<int32_t> f(pi.size());
        if (int rc = pcabi_compat_host(device, codes, codes_len, seq_off, seq_len, n, pi.data(), pj.data(),
                                       (int64_t)pi.size(), f.data()))
            return rc;
        for (size_t t = 0; t < pi.size(); ++t) mat[(int64_t)pi[t] * n + pj[t]] = mat[(int64_t)pj[t] * n + pi[t]] = f[t];
        return 0;
    }
    // every sequence against every sequence in the tiled cross mode (both orientations, no host
    // task lists), then per pair the orientation the reference uses: row 0 = the longer, ties ->
    // the first argument (consensus.py:90-97 passes seq_i, seq_j with i < j)
    std::vector<uint8_t> acodes;
    std::vector<int32_t> aoff((size_t)n);
    for (int64_t k = 0; k < n; ++k) {
        aoff[k] = (int32_t)acodes.size();
        acodes.insert(acodes.end(), codes + seq_off[k], codes + seq_off[k] + seq_len[k]);
    }
    // the cross product f[a * n + w] stays on the device; k_orient writes the matrix
    return align_host_impl(device, codes, codes_len, seq_off, seq_len, n, acodes.data(), aoff.data(), seq_len,
                           (int32_t)n, nullptr, nullptr, 0, 2, -1, -1, -1, nullptr, mat, true, true);
}

int check_compatibility(char *raw_seq1, char *raw_seq2) {
    // SeqAn String<Dna> (compatibility.h:23): A C G T/U, anything else -> A
    const size_t n1 = raw_seq1 ? std::strlen(raw_seq1) : 0, n2 = raw_seq2 ? std::strlen(raw_seq2) : 0;
    std::vector<uint8_t> codes(((n1 + 3) & ~(size_t)3) + n2 + 16, 0);
    auto enc = [](char c) -> uint8_t {
        switch (c) {
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': case 'U': case 'u': return 3;
        default: return 0;
        }
    };
    for (size_t k = 0; k < n1; ++k) codes[k] = enc(raw_seq1[k]);
    const int64_t o2 = (int64_t)((n1 + 3) & ~(size_t)3);
    for (size_t k = 0; k < n2; ++k) codes[o2 + k] = enc(raw_seq2[k]);
    const int64_t off[2] = {0, o2};
    const int32_t len[2] = {(int32_t)n1, (int32_t)n2};
    const int32_t pi = 0, pj = 1;
    int32_t flag = 0;
    int device = 0;
    (void)hipGetDevice(&device);
    if (pcabi_compat_host(device, codes.data(), (int64_t)codes.size(), off, len, 2, &pi, &pj, 1, &flag) != 0) {
        // the reference has no error channel and never fails here: stop rather than answer wrongly
        std::fprintf(stderr, "libpcabi: check_compatibility failed: %s\n", pcabi_last_error());
        std::abort();
    }
    return flag;
}

int pcabi_barcode_call_host(int device, const int32_t *start_res, int32_t n_sa, const int32_t *start_slot_adp,
                            const int32_t *start_slot_name, int32_t n_start_slots, const int32_t *end_res,
                            int32_t n_ea, const int32_t *end_slot_adp, const int32_t *end_slot_name,
                            int32_t n_end_slots, int64_t n_read, double barcode_threshold, double barcode_diff,
                            int require_two, int32_t *call, double *scores) {
    if (device < 0 || device >= 16) return fail(PCABI_E_ARG, "bad device index");
    if (n_read < 0 || n_sa < 0 || n_ea < 0 || n_start_slots < 0 || n_end_slots < 0)
        return fail(PCABI_E_ARG, "negative count");
    for (int k = 0; k < n_start_slots; ++k)
        if (start_slot_adp[k] < 0 || start_slot_adp[k] >= n_sa) return fail(PCABI_E_ARG, "start slot adapter out of range");
    for (int k = 0; k < n_end_slots; ++k)
        if (end_slot_adp[k] < 0 || end_slot_adp[k] >= n_ea) return fail(PCABI_E_ARG, "end slot adapter out of range");
    if (n_read == 0) return 0;
    Engine &e = g_engines[device];
    std::lock_guard<std::mutex> lock(e.mu);
    if (int rc = engine_init(e, device)) return rc;
    HIP_TRY(hipSetDevice(device));
    const size_t sres = sizeof(int32_t) * PCABI_NFIELDS * (size_t)n_sa * (size_t)n_read;
    const size_t eres = sizeof(int32_t) * PCABI_NFIELDS * (size_t)n_ea * (size_t)n_read;
    const size_t slots = sizeof(int32_t) * 2 * (size_t)(n_start_slots + n_end_slots);
    if (int rc = e.bc.ensure(sres + eres + slots + sizeof(int32_t) * (size_t)n_read + 32 * (size_t)n_read + 64))
        return rc;
    char *p = (char *)e.bc.p;
    int32_t *d_sres = (int32_t *)p; p += sres;
    int32_t *d_eres = (int32_t *)p; p += eres;
    int32_t *d_slots = (int32_t *)p; p += slots;
    int32_t *d_call = (int32_t *)p; p += sizeof(int32_t) * (size_t)n_read;
    p = (char *)(((uintptr_t)p + 7) & ~(uintptr_t)7);
    double *d_scores = (double *)p;
    std::vector<int32_t> h_slots;
    h_slots.insert(h_slots.end(), start_slot_adp, start_slot_adp + n_start_slots);
    h_slots.insert(h_slots.end(), start_slot_name, start_slot_name + n_start_slots);
    h_slots.insert(h_slots.end(), end_slot_adp, end_slot_adp + n_end_slots);
    h_slots.insert(h_slots.end(), end_slot_name, end_slot_name + n_end_slots);
    if (sres) HIP_TRY(hipMemcpyAsync(d_sres, start_res, sres, hipMemcpyHostToDevice, e.stream));
    if (eres) HIP_TRY(hipMemcpyAsync(d_eres, end_res, eres, hipMemcpyHostToDevice, e.stream));
    if (slots) HIP_TRY(hipMemcpyAsync(d_slots, h_slots.data(), slots, hipMemcpyHostToDevice, e.stream));
    const int32_t *ss = d_slots, *en_ = d_slots + 2 * n_start_slots;
    if (int rc = pcabi_barcode_call_dev(d_sres, (int64_t)n_sa * n_read, ss, ss + n_start_slots, n_start_slots, d_eres,
                                        (int64_t)n_ea * n_read, en_, en_ + n_end_slots, n_end_slots, n_read,
                                        barcode_threshold, barcode_diff, require_two, d_call,
                                        scores ? d_scores : nullptr, e.stream))
        return rc;
    HIP_TRY(hipMemcpyAsync(call, d_call, sizeof(int32_t) * (size_t)n_read, hipMemcpyDeviceToHost, e.stream));
    if (scores)
        HIP_TRY(hipMemcpyAsync(scores, d_scores, 32 * (size_t)n_read, hipMemcpyDeviceToHost, e.stream));
    HIP_TRY(hipStreamSynchronize(e.stream));
    return 0;
}

}  // extern "C"

// ---- end-trim decisions of the reference-API driver (find_adapters_at_read_ends) -----------------
extern "C" int pcabi_flag_list_dev(const uint8_t *flag, int32_t n_adp, int64_t n_read, const int32_t *res,
                                   int64_t stride, int32_t *out, int64_t cap, unsigned long long *n_out,
                                   void *stream);

namespace {

// out[j * n_read + r] = the full-adapter identity (pid6(m, l2), 0.0 for no alignment) of adapter
// sel[j] on read r: the barcode dicts of find_start_trim / find_end_trim (nanopore_read.py:193-195).
__global__ __launch_bounds__(256) void k_full_ids(const int32_t *res, int64_t stride, int64_t n_read,
                                                  const int32_t *sel, int32_t n_sel, double *out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)n_sel * n_read) return;
    const int32_t j = (int32_t)(i / n_read);
    const int64_t q = (int64_t)sel[j] * n_read + (i - (int64_t)j * n_read);
    out[i] = res[q] == -1 ? 0.0 : pcabi::pid6(res[5 * stride + q], res[7 * stride + q]);
}

// The compact form of a side's alignment list for the D2H (pcabi_end_decisions_host): per
// alignment six int16 (adapter, rs, re, m, l1, l2), per read its alignment count (uint16, two per
// dword); the read row is rebuilt on the host from the counts (the list is read-major). 12 B per
// alignment + 2 B per read instead of 28 B per alignment.
__global__ __launch_bounds__(256) void k_list_pack(const int32_t *list, int64_t dcap, int64_t cnt, int16_t *out,
                                                   uint32_t *counts) {
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < cnt; k += (int64_t)gridDim.x * 256) {
        const int32_t r = list[k];
#pragma unroll
        for (int f = 0; f < 6; ++f) out[f * cnt + k] = (int16_t)list[(f + 1) * dcap + k];
        atomicAdd(&counts[r >> 1], 1u << (16 * (r & 1)));
    }
}

int side_table(Engine::DTab &c, const uint8_t *codes, const int32_t *off, const int32_t *len, int32_t n,
               const pcabi::Scoring &sc, pcabi_adapters **out) {
    std::vector<uint8_t> key;
    for (int32_t a = 0; a < n; ++a) key.insert(key.end(), codes + off[a], codes + off[a] + len[a]);
    if (c.t && c.sc.ma == sc.ma && c.sc.mi == sc.mi && c.sc.go == sc.go && c.sc.ge == sc.ge && c.codes == key &&
        c.lens == std::vector<int32_t>(len, len + n)) {
        *out = c.t;
        return 0;
    }
    if (c.t) pcabi_adapters_destroy(c.t);   // the previous call synchronised its stream
    c.t = nullptr;
    if (int rc = adapters_create_impl(codes, off, len, n, &sc, &c.t)) return rc;
    c.codes.swap(key);
    c.lens.assign(len, len + n);
    c.sc = sc;
    *out = c.t;
    return 0;
}

}  // namespace

namespace {
// pcabi_end_decisions_host / _seqs: the windows' codes come from `codes` (a host Dna5 buffer) or,
// when `win` is set, from the 2 n_read window strings (start windows, then end windows), encoded
// straight into pinned staging buffers while earlier chunks copy (stage_seqs)
int end_decisions_impl(
    int device, const uint8_t *codes, const char *const *win, const int32_t *win_len, int64_t codes_len,
    const int64_t *s_off, const int32_t *s_len, const int64_t *e_off, const int32_t *e_len, int64_t n_read,
    const uint8_t *sa_codes, const int32_t *sa_off, const int32_t *sa_len, int32_t n_sa, const uint8_t *ea_codes,
    const int32_t *ea_off, const int32_t *ea_len, int32_t n_ea, int match, int mismatch, int gap_open, int gap_extend,
    int end_size, int extra_trim, double end_threshold, int min_trim_size, int32_t *start_trim, int32_t *end_trim,
    int32_t *start_hits, int32_t *end_hits, int64_t cap, int64_t *n_hits, const int32_t *bc_s, int32_t n_bc_s,
    const int32_t *bc_e, int32_t n_bc_e, double *bc_full) {
    if (device < 0 || device >= 16) return fail(PCABI_E_ARG, "bad device index");
    if (n_read < 0 || n_sa < 0 || n_ea < 0 || cap < 0 || n_bc_s < 0 || n_bc_e < 0) return fail(PCABI_E_ARG, "negative count");
    if (int rc = check_common(sa_len, n_sa)) return rc;
    if (int rc = check_common(ea_len, n_ea)) return rc;
    for (int side = 0; side < 2; ++side) {
        const int64_t *off = side ? e_off : s_off;
        const int32_t *len = side ? e_len : s_len;
        for (int64_t w = 0; w < n_read; ++w) {
            if (len[w] < 0 || len[w] > pcabi::MAX_WINDOW_LEN) return fail(PCABI_E_ARG, "window length out of range");
            if (len[w] > 0 && (off[w] < 0 || off[w] + len[w] + 16 > codes_len))
                return fail(PCABI_E_ARG, "window outside the buffer or buffer not padded by 16 bytes");
        }
    }
    for (int32_t j = 0; j < n_bc_s; ++j)
        if (bc_s[j] < 0 || bc_s[j] >= n_sa) return fail(PCABI_E_ARG, "start barcode adapter out of range");
    for (int32_t j = 0; j < n_bc_e; ++j)
        if (bc_e[j] < 0 || bc_e[j] >= n_ea) return fail(PCABI_E_ARG, "end barcode adapter out of range");
    n_hits[0] = n_hits[1] = 0;
    if (n_read == 0) return 0;
    // PCABI_END_PROF=1: the call's host / device phases on stderr
    static const bool prof = [] { const char *v = std::getenv("PCABI_END_PROF"); return v && v[0] == '1'; }();
    const auto t0 = std::chrono::steady_clock::now();
    auto mark = [&](const char *what) {
        if (prof)
            std::fprintf(stderr, "pcabi_end_decisions: %-10s %.3f ms\n", what,
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    };
    Engine &e = g_engines[device];
    std::lock_guard<std::mutex> lock(e.mu);
    if (int rc = engine_init(e, device)) return rc;
    HIP_TRY(hipSetDevice(device));
    const pcabi::Scoring sc{match, mismatch, gap_open, gap_extend};
    const hipStream_t st = e.stream;
    const size_t n = (size_t)n_read;
    const int32_t n_adp[2] = {n_sa, n_ea};
    // buffers: 0 codes; per side (base 1 + 6 side): offsets, lengths, tile offsets, tiles, results, flags;
    // 13 trims (2 x n); 14 lists (2 sides x 7 x n_read x n_adp bound); 15 counts + barcode identities
    if (int rc = e.dec[0].ensure((size_t)codes_len)) return rc;
    if (win) {
        std::vector<int64_t> off(2 * n);
        std::copy(s_off, s_off + n, off.begin());
        std::copy(e_off, e_off + n, off.begin() + (int64_t)n);
        if (int rc = stage_seqs(e, (uint8_t *)e.dec[0].p, win, win_len, off.data(), 2 * n_read, codes_len)) return rc;
    } else {
        HIP_TRY(hipMemcpyAsync(e.dec[0].p, codes, (size_t)codes_len, hipMemcpyHostToDevice, st));
    }
    mark("staged");
    if (int rc = e.dec[13].ensure(8 * n)) return rc;
    int32_t *d_st = (int32_t *)e.dec[13].p, *d_et = d_st + n;
    std::vector<int64_t> toff[2];
    const int32_t *res[2] = {nullptr, nullptr};
    uint8_t *flag[2] = {nullptr, nullptr};
    pcabi_cross_region reg[2];
    int32_t n_reg = 0;
    for (int side = 0; side < 2; ++side) {
        const int64_t *off = side ? e_off : s_off;
        const int32_t *len = side ? e_len : s_len;
        DeviceBuf *b = e.dec + 1 + 6 * side;
        if (int rc = b[0].ensure(8 * n)) return rc;
        if (int rc = b[1].ensure(4 * n)) return rc;
        toff[side].assign((n + 255) / 256 + 1, 0);
        int64_t max_nq = 0;
        const int64_t nd = tile_layout(len, n_read, toff[side].data(), &max_nq);
        if (int rc = b[2].ensure(8 * toff[side].size())) return rc;
        if (int rc = b[3].ensure(4 * (size_t)std::max<int64_t>(nd, 1))) return rc;
        if (int rc = b[4].ensure(4 * PCABI_NFIELDS * n * (size_t)std::max(n_adp[side], 1))) return rc;
        if (int rc = b[5].ensure(n * (size_t)std::max(n_adp[side], 1))) return rc;
        HIP_TRY(hipMemcpyAsync(b[0].p, off, 8 * n, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(b[1].p, len, 4 * n, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(b[2].p, toff[side].data(), 8 * toff[side].size(), hipMemcpyHostToDevice, st));
        res[side] = (const int32_t *)b[4].p;
        flag[side] = (uint8_t *)b[5].p;
        if (!n_adp[side]) continue;
        int32_t max_len = 0;
        for (size_t w = 0; w < n; ++w) max_len = std::max(max_len, len[w]);
        pcabi_adapters *tab = nullptr;
        if (int rc = side_table(e.dtab[side], side ? ea_codes : sa_codes, side ? ea_off : sa_off, side ? ea_len : sa_len,
                                n_adp[side], sc, &tab))
            return rc;
        launch_tiles((const uint8_t *)e.dec[0].p, (const int64_t *)b[0].p, (const int32_t *)b[1].p, n_read,
                     (const int64_t *)b[2].p, max_nq, (uint32_t *)b[3].p, st);
        reg[n_reg++] = pcabi_cross_region{(const uint32_t *)b[3].p, (const int64_t *)b[2].p, (const int32_t *)b[1].p,
                                          n_read, max_len, tab, (int32_t *)b[4].p, (int64_t)n_adp[side] * n_read};
    }
    // both read ends in one call: the register buckets of both sides in grouped launches (r06)
    if (int rc = pcabi_align_cross_multi_dev(reg, n_reg, match, mismatch, gap_open, gap_extend, st, nullptr, nullptr))
        return rc;
    if (int rc = pcabi_end_trim_dev(res[0], (int64_t)n_sa * n_read, n_sa, res[1], (int64_t)n_ea * n_read, n_ea, n_read,
                                    end_size, extra_trim, end_threshold, min_trim_size, d_st, d_et, flag[0], flag[1], st))
        return rc;
    // the alignment lists (device capacity: every pair of the side -- they never overflow there)
    const size_t dcap[2] = {n * (size_t)n_sa, n * (size_t)n_ea};
    if (int rc = e.dec[14].ensure(4 * 7 * (dcap[0] + dcap[1]) + 16)) return rc;
    int32_t *d_list[2] = {(int32_t *)e.dec[14].p, (int32_t *)e.dec[14].p + 7 * dcap[0]};
    const size_t nbc = (size_t)n_bc_s + (size_t)n_bc_e;
    if (int rc = e.dec[15].ensure(64 + ((4 * nbc + 7) & ~(size_t)7) + 8 * nbc * n)) return rc;   // d_full below
    unsigned long long *d_cnt = (unsigned long long *)e.dec[15].p;
    int32_t *d_sel = (int32_t *)((char *)e.dec[15].p + 16);
    double *d_full = (double *)((char *)e.dec[15].p + 64 + ((4 * nbc + 7) & ~(size_t)7));
    for (int side = 0; side < 2; ++side) {
        if (!n_adp[side]) {
            HIP_TRY(hipMemsetAsync(d_cnt + side, 0, 8, st));
            continue;
        }
        if (int rc = pcabi_flag_list_dev(flag[side], n_adp[side], n_read, res[side], (int64_t)n_adp[side] * n_read,
                                         d_list[side], (int64_t)dcap[side], d_cnt + side, st))
            return rc;
    }
    if (nbc && bc_full) {
        std::vector<int32_t> sel(bc_s, bc_s + n_bc_s);
        sel.insert(sel.end(), bc_e, bc_e + n_bc_e);
        HIP_TRY(hipMemcpyAsync(d_sel, sel.data(), 4 * nbc, hipMemcpyHostToDevice, st));
        for (int side = 0; side < 2; ++side) {
            const int32_t ns = side ? n_bc_e : n_bc_s;
            if (!ns) continue;
            const int64_t tot = (int64_t)ns * n_read;
            hipLaunchKernelGGL(k_full_ids, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, res[side],
                               (int64_t)n_adp[side] * n_read, n_read, d_sel + (side ? n_bc_s : 0), ns,
                               d_full + (side ? (size_t)n_bc_s * n : 0));
        }
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(bc_full, d_full, 8 * nbc * n, hipMemcpyDeviceToHost, st));
    }
    unsigned long long cnt[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(start_trim, d_st, 4 * n, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(end_trim, d_et, 4 * n, hipMemcpyDeviceToHost, st));
    mark("queued");
    HIP_TRY(hipMemcpyAsync(cnt, d_cnt, 16, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    mark("device");
    n_hits[0] = (int64_t)cnt[0];
    n_hits[1] = (int64_t)cnt[1];
    // the lists: compact (int16 fields, per-read counts) when every field fits 16 bits -- the
    // alignment lengths l1 / l2 reach the window plus the adapter
    int32_t max_win = 0, max_adp = 0;
    for (size_t w = 0; w < n; ++w) max_win = std::max(max_win, std::max(s_len[w], e_len[w]));
    for (int32_t a = 0; a < n_sa; ++a) max_adp = std::max(max_adp, sa_len[a]);
    for (int32_t a = 0; a < n_ea; ++a) max_adp = std::max(max_adp, ea_len[a]);
    const bool compact = (int64_t)max_win + max_adp < 32768 && n_sa < 32768 && n_ea < 32768;
    const size_t half = (n + 1) / 2;                // count dwords per side
    if (compact) {
        size_t words = 0;
        for (int side = 0; side < 2; ++side)
            if ((int64_t)cnt[side] <= cap) words += 3 * (size_t)cnt[side] + half;   // 6 int16 = 3 dwords
        if (int rc = e.dec[16].ensure(4 * words + 64)) return rc;
        std::vector<uint32_t> h((size_t)words);
        size_t at = 0, at_side[2] = {0, 0};
        for (int side = 0; side < 2; ++side) {
            const int64_t k = (int64_t)cnt[side];
            if (k > cap) continue;
            at_side[side] = at;
            uint32_t *dc = (uint32_t *)e.dec[16].p + at + 3 * (size_t)k;
            HIP_TRY(hipMemsetAsync(dc, 0, 4 * half, st));
            if (k)
                hipLaunchKernelGGL(k_list_pack, dim3((unsigned)std::min<int64_t>((k + 255) / 256, 4096)), dim3(256), 0, st,
                                   d_list[side], (int64_t)dcap[side], k, (int16_t *)((uint32_t *)e.dec[16].p + at), dc);
            at += 3 * (size_t)k + half;
        }
        HIP_TRY(hipGetLastError());
        if (words) HIP_TRY(hipMemcpyAsync(h.data(), e.dec[16].p, 4 * words, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        mark("lists d2h");
        for (int side = 0; side < 2; ++side) {
            int32_t *dst = side ? end_hits : start_hits;
            const int64_t k = (int64_t)cnt[side];
            if (k > cap || !k) continue;            // too many: the caller grows cap and calls again
            const int16_t *f16 = (const int16_t *)(h.data() + at_side[side]);
            const uint16_t *c16 = (const uint16_t *)(h.data() + at_side[side] + 3 * (size_t)k);
            int64_t j = 0;
            for (size_t r = 0; r < n && j < k; ++r)
                for (uint16_t c = c16[r]; c > 0; --c) dst[j++] = (int32_t)r;
            for (int f = 0; f < 6; ++f)
                for (int64_t q = 0; q < k; ++q) dst[(f + 1) * cap + q] = f16[f * k + q];
        }
        mark("unpacked");
        return 0;
    }
    for (int side = 0; side < 2; ++side) {
        int32_t *dst = side ? end_hits : start_hits;
        const int64_t k = (int64_t)cnt[side];
        if (k > cap || !k) continue;                // too many: the caller grows cap and calls again
        for (int f = 0; f < 7; ++f)                 // rows of the device list (stride dcap) -> stride cap
            HIP_TRY(hipMemcpyAsync(dst + f * cap, d_list[side] + f * dcap[side], 4 * (size_t)k, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}
}  // namespace

extern "C" int pcabi_end_decisions_host(
    int device, const uint8_t *codes, int64_t codes_len, const int64_t *s_off, const int32_t *s_len,
    const int64_t *e_off, const int32_t *e_len, int64_t n_read, const uint8_t *sa_codes, const int32_t *sa_off,
    const int32_t *sa_len, int32_t n_sa, const uint8_t *ea_codes, const int32_t *ea_off, const int32_t *ea_len,
    int32_t n_ea, int match, int mismatch, int gap_open, int gap_extend, int end_size, int extra_trim,
    double end_threshold, int min_trim_size, int32_t *start_trim, int32_t *end_trim, int32_t *start_hits,
    int32_t *end_hits, int64_t cap, int64_t *n_hits, const int32_t *bc_s, int32_t n_bc_s, const int32_t *bc_e,
    int32_t n_bc_e, double *bc_full) {
    return end_decisions_impl(device, codes, nullptr, nullptr, codes_len, s_off, s_len, e_off, e_len, n_read, sa_codes,
                              sa_off, sa_len, n_sa, ea_codes, ea_off, ea_len, n_ea, match, mismatch, gap_open,
                              gap_extend, end_size, extra_trim, end_threshold, min_trim_size, start_trim, end_trim,
                              start_hits, end_hits, cap, n_hits, bc_s, n_bc_s, bc_e, n_bc_e, bc_full);
}

// pcabi_end_decisions_host over window strings: win / win_len hold the n_read start windows, then
// the n_read end windows (addresses of their first characters -- ASCII, one byte per base -- and
// lengths); the library lays them out as the host entry's buffer and encodes them itself.
extern "C" int pcabi_end_decisions_seqs(
    int device, const char *const *win, const int32_t *win_len, int64_t n_read, const uint8_t *sa_codes,
    const int32_t *sa_off, const int32_t *sa_len, int32_t n_sa, const uint8_t *ea_codes, const int32_t *ea_off,
    const int32_t *ea_len, int32_t n_ea, int match, int mismatch, int gap_open, int gap_extend, int end_size,
    int extra_trim, double end_threshold, int min_trim_size, int32_t *start_trim, int32_t *end_trim,
    int32_t *start_hits, int32_t *end_hits, int64_t cap, int64_t *n_hits, const int32_t *bc_s, int32_t n_bc_s,
    const int32_t *bc_e, int32_t n_bc_e, double *bc_full) {
    if (n_read < 0) return fail(PCABI_E_ARG, "negative count");
    const int64_t nw = 2 * n_read;
    std::vector<int64_t> off((size_t)nw);
    int64_t total = 0;
    for (int64_t w = 0; w < nw; ++w) {
        if (win_len[w] < 0 || win_len[w] > pcabi::MAX_WINDOW_LEN) return fail(PCABI_E_ARG, "window length out of range");
        if (win_len[w] > 0 && !win[w]) return fail(PCABI_E_ARG, "NULL sequence");
        off[(size_t)w] = total;
        total += ((int64_t)win_len[w] + 3) & ~(int64_t)3;
    }
    total += 16;
    return end_decisions_impl(device, nullptr, win, win_len, total, off.data(), win_len, off.data() + n_read,
                              win_len + n_read, n_read, sa_codes, sa_off, sa_len, n_sa, ea_codes, ea_off, ea_len, n_ea,
                              match, mismatch, gap_open, gap_extend, end_size, extra_trim, end_threshold, min_trim_size,
                              start_trim, end_trim, start_hits, end_hits, cap, n_hits, bc_s, n_bc_s, bc_e, n_bc_e,
                              bc_full);
}
