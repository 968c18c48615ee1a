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
// Kernels (integer work, no MFMA), r03 layout: the streaming part and the irregular part apart.
//   k_seed_scan   the read bytes stream through (every wave an equal range of 32-position segments):
//                 2-bit codes packed once per lane, one LDS byte-map read per two positions (the
//                 merged 8-mer table; positions whose valid run is shorter than 8 flagged for the
//                 short tables). A position that hits is appended as a raw hit (read, position, its
//                 8-mer) to the wave's own slab in global memory (no global atomics, no barriers
//                 inside the loop);
//   k_seed_expand resident blocks over the slabs: the probe entries of every raw hit (rank / entry tables in
//                 LDS) become (read, adapter, diagonal) tasks per band class -- a block scan of the
//                 per-hit counts, one global atomic per class and 256 hits;
//   k_seed_band   grid-stride over a class's tasks: the banded Gotoh score DP (2E+1 cells per
//                 adapter row in registers; the read bytes of the band streamed in dwords, the
//                 adapters in LDS), atomicMax into the pair's bound;
//   k_cands       the pairs whose bound reaches T, compacted (k_bound16: or all bounds as int16).
// Every count the launches need may live on the device (the read count of a round included), so
// the engine can queue whole rounds without a host round trip; capacities that a launch could
// exceed raise a flag the host checks once, and the scan is then rerun with larger buffers.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

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
// pcabi_engine.hip: the scratch generation its captured round graphs are keyed on (a reallocation,
// a new plan or new capacities here change addresses or launch arguments those graphs hold)
extern std::atomic<uint64_t> g_buf_gen;
void pcabi_poison(void *p, size_t bytes);   // pcabi_engine.hip: PCABI_POISON=1 fills fresh scratch
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

#ifndef PCABI_BAND_EXIT
#define PCABI_BAND_EXIT 1   // rows between the banded DP's early-exit checks (1: every row, r02 A/B)
#endif
constexpr int kLdsMax = 64 * 1024; // per block: probe tables
constexpr int kAdpLds = 16 * 1024; // adapters copied to LDS by the band kernels up to this size
constexpr int kNeg = -(1 << 20);
constexpr int kSeg = 32;           // read positions per lane and scan step (a segment; 40 bytes loaded)
constexpr unsigned kSlowBit = 0x80000000u;   // raw hit: the position's valid run is shorter than 8
constexpr int kBandGrid = 4096;    // band / cands launches whose count is on the device: grid-stride
// task counters: [c] inside-band tasks of class c (from the region's start), [kCls + c] edge tasks
// (bands touching a read end, from the region's end), then the two overflow flags
constexpr int kCnt = 2 * kCls + 2;
constexpr int kFlag = 2 * kCls;
constexpr int kVer = kCnt;          // the verified-seed counter, after the task counters and flags
constexpr int kCntAll = kCnt + 1;   // every counter k_bound_reset zeroes
constexpr int kPinMaxE = 8;        // the pinned band is built for E <= kPinMaxE
constexpr int kStatBlocks = 8192;  // profiled band launches: per-wave counter slots for this many blocks

struct ScanArgs {
    const uint8_t *codes;
    const int64_t *v_off;
    const int32_t *v_len;
    int64_t n;                  // reads (host upper bound)
    const int32_t *n_dev;       // != nullptr: the read count on the device (<= n)
    const uint32_t *tabs;       // LDS image: bits | rank16 | estart16 | ent (dwords, copied as is)
    int32_t tab_dw;             // its dwords
    int32_t bits_dw;            // the bitmaps' dwords at its head (all the scan needs)
    int32_t bits_off[kNK];      // dword offset of K's bitmap in the image, -1 when no probe has length K;
                                // K = 8 is the merged table: every 8-mer extending a probe of any K
    int32_t min_k;              // shortest probe
    int32_t rank_off, estart_off, ent_off;   // dword offsets of the other sections
                                             // (entries: adapter << 12 | (K - 4) << 9 | band class << 8 | offset)
    uint4 *raw;                 // per scan block a slab of raw hits (read, position | kSlowBit,
                                // 8-mer code | valid run << 16, 0): the expansion reads no read bytes
    int32_t slab;
    int32_t n_slab;             // slabs (scan blocks); the expansion's blocks stride over them
    int32_t *raw_cnt;           // raw hits per slab
    int32_t *flags;             // [0] a slab overflowed, [1] a task region overflowed
    int4 *task;                 // per class cap inside-band tasks, then ecap edge tasks (bands that touch
                                // a read end): (read, adapter, diagonal, probe offset)
    int64_t cap, ecap;
    int32_t *cnt;               // kCnt counters (inside / edge tasks per class, flags)
    int32_t ent2_off;           // dword offset of the entries' inside limits (lo | hi << 16): a task
                                // is inside when q >= lo and (read length - q) > hi
    int32_t pin_cls[kCls];      // class c's inside tasks run the pinned band: records (read,
                                // adapter << 11 | (K - 4) << 8 | o, the probe's byte offset in codes: lo, hi)
    const int64_t *seg_cum;     // n + 1 entries: segments (kSeg positions) before each read, the total last
};

__device__ __forceinline__ int64_t dev_count(const int32_t *n_dev, int64_t n) {
    return n_dev ? min((int64_t)*n_dev, n) : n;
}

// Verified seeds (the device rounds' candidate windows): every band task whose bound
// reaches its adapter's T is recorded as (read, adapter | E << 24, the diagonal's codes offset
// v_off[read] + d0 as lo / hi): an alignment scoring >= T has an exact piece, so its task is among
// these, and its end cell lies within the band's reach of the diagonal. list == nullptr: off.
struct VerOut {
    int4 *list;
    int32_t *cnt;
    int32_t *flag;              // set when the list overflowed (the round reruns with a larger one)
    int64_t cap;
};
// Every lane of the wave that reaches this call takes part (one atomic per wave).
__device__ __forceinline__ void put_verified(const VerOut &vo, bool want, int32_t read, int32_t a, int E, int64_t dabs) {
    const uint64_t m = __ballot(want);
    if (!m) return;
    const int lane = (int)(threadIdx.x & 63);
    const int leader = __ffsll((unsigned long long)m) - 1;
    int b0 = 0;
    if (lane == leader) b0 = atomicAdd(vo.cnt, __popcll(m));
    b0 = __shfl(b0, leader);
    if (want) {
        const int64_t slot = (int64_t)b0 + __popcll(m & ((1ull << lane) - 1));
        if (slot < vo.cap)
            vo.list[slot] = make_int4(read, a | (E << 24), (int)(uint32_t)(uint64_t)dabs, (int)(uint32_t)((uint64_t)dabs >> 32));
        else
            atomicOr(vo.flag, 1);
    }
}

// Segments (kSeg positions) of read r of a round: 0 past the round's read count.
struct SegCount {
    const int32_t *len;
    const int32_t *n_dev;
    int64_t n;
    __host__ __device__ int64_t operator()(int64_t r) const {
        const int64_t nr = n_dev ? (*n_dev < n ? (int64_t)*n_dev : n) : n;
        return r < nr ? ((int64_t)max(len[r], 0) + kSeg - 1) / kSeg : 0;
    }
};

// A dword of k_seed_scan's LDS by byte address: the kernel declares no static LDS, so its dynamic
// area starts at LDS address 0 and the code's mask is the whole address computation.
__device__ __forceinline__ uint32_t lds_at(uint32_t byte_addr) {
    return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>((size_t)byte_addr);
}

// 64-bit wave-uniform value (readfirstlane per half)
__device__ __forceinline__ int64_t rfl64(int64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// A read's segment end, code offset and length (reads past the round's count: an empty read at
// the end of the segment space).
struct ReadMeta {
    int64_t s1, off;
    int32_t len;
};
__device__ __forceinline__ ReadMeta read_meta(const ScanArgs &a, int64_t r, int64_t nr, int64_t S) {
    ReadMeta m{S, 0, 0};
    if (r < nr) {
        m.s1 = rfl64(a.seg_cum[r + 1]);
        m.off = rfl64(a.v_off[r]);
        m.len = __builtin_amdgcn_readfirstlane(a.v_len[r]);
    }
    return m;
}

// The segment walk (r03): the reads' positions are cut into segments of kSeg = 32 (seg_cum, an
// exclusive scan of ceil(len / 32) over the round's reads), and every WAVE takes an equal,
// contiguous range of segments -- no read-length imbalance between waves, and no idle lanes at
// a read's end beyond its last segment (r02 / early r03: blocks took whole reads in steps of
// 4096 positions, so a 5 kb read cost as much as an 8 kb one and the slowest block set the time).
// Lane l of a step holds segment b + l: 40 bytes (its 32 positions and the 7-base lookahead), in
// three loads issued one step ahead. The wave keeps the metadata of its current read and the next
// one (scalar loads when the wave crosses a read end); a lane past both (reads < 2 kb) looks its
// read up itself.
// Per position: the rolling 8-mer (first base in the top bits), its bitmap word (LDS byte address
// (code >> 3) & 0x1FFC: the merged K = 8 bitmap sits at LDS byte 0) and the bit shifted into the
// step's hit mask (alignbit) -- no validity work. A lane whose 40 bytes hold an N or pass its
// read's end masks the hits afterwards: bit i survives when bytes i .. i + 7 are valid bases of
// the read (doubling ORs of the invalid-byte mask), and the positions whose valid run is shorter
// than 8 but at least the shortest probe are flagged for the short tables. (An N byte = 4 only
// disturbs the codes of windows that contain it, and those are masked.)
// Hits are appended to the block's slab as before: (read, position | kSlowBit, its clean 8-mer |
// valid run << 16, read length - position).
// k_seed_scan (r04): that segment walk, with the per-position work cut from the r03 kernel's 6 VALU
// instructions (an LDS bitmap word per position) to 2:
//   * the merged 8-mer bitmap is expanded into a BYTE map in LDS (64 KiB), so a lookup is one
//     ds_read_u8 at an 8-mer code; r05: a PAIR map -- byte c holds the membership of c and, per next
//     base j, of the 8-mer that follows (c << 2 | j), so one read serves two positions;
//   * a lane's 40 bytes are packed once into 2-bit codes, base 0 in the top bits (P0 = bases 0-15,
//     Q0 = 8-23, P1 = 16-31, Q1 = 24-39): position i's code is one bit-field extract of one of them;
//   * a hit's 8-mer comes from the same packed words (no re-read of the read bytes).
// Two blocks per CU share the CU's LDS between their byte maps.
constexpr int kScanThreads = 1024;
constexpr int kByteMap = 1 << 16;            // bytes: one per 8-mer code

// 4 bytes (base codes in their low 2 bits) -> 8 bits, byte 0's base in the top two: in the low byte
__device__ __forceinline__ uint32_t pack4(uint32_t d) {
    const uint32_t t = d & 0x03030303u;
    const uint32_t v = (t << 2) | (t >> 8);          // byte 0: b0 b1, byte 2: b2 b3
    return (v << 4) | (v >> 16);                     // byte 0: b0 b1 b2 b3
}
// the same byte with one dot product: byte k's code times 64 >> 2k (the N code's bit 2 masked first)
__device__ __forceinline__ uint32_t pack4_dot(uint32_t d) {
    return __builtin_amdgcn_udot4(d & 0x03030303u, 0x01041040u, 0u, false);
}
// four packed bytes (low bytes of x0..x3) -> one word, x0 in the top byte
__device__ __forceinline__ uint32_t pack16(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
    const uint32_t hi = __builtin_amdgcn_perm(x0, x1, 0x0C0C0400u);   // byte 1: x0, byte 0: x1
    const uint32_t lo = __builtin_amdgcn_perm(x2, x3, 0x0C0C0400u);
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// TPB: threads per block (r05: 1024 -- two blocks per CU, each holding the 64 KiB map, run 32 waves
// per CU instead of the r04 blocks' 16; measured neutral, kept)
template <int TPB>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(TPB == 1024 ? 8 : 4))) void k_seed_scan(ScanArgs a) {
    // static LDS (a workgroup may hold more than 64 KiB of it on gfx950): the byte map -- a position's
    // code plus the map's constant LDS address is its read address
    __shared__ __attribute__((aligned(16))) uint32_t bmap[kByteMap / 4];
    {   // the pair map from the bitmap B (2048 words, bit c of the merged table = word c >> 5, bit
        // c & 31): byte c holds, for each next base j, bits 2j = B[c] and 2j + 1 = B[(4c + j) & 0xFFFF]
        // -- the membership of the 8-mers at positions i and i + 1 of a 9-mer c.j. Map dword m (codes
        // 4m .. 4m + 3): the first bits from nibble m & 7 of word m >> 3, the second ones from the
        // 16-bit half m & 1 of word (m >> 1) & 2047 (bits 16m + 4j' .. + 3 for byte j'). Bitmap word w
        // covers map dwords 8w .. 8w + 7; a thread's words loaded together.
        constexpr int kWpt = (kByteMap / 32) / TPB;        // bitmap words per thread
        static_assert(kWpt * TPB == kByteMap / 32, "whole bitmap words per thread");
        uint32_t word[kWpt], half[kWpt][4];
#pragma unroll
        for (int q = 0; q < kWpt; ++q) {
            const int w = threadIdx.x + q * TPB;
            word[q] = a.tabs[w];
#pragma unroll
            for (int h = 0; h < 4; ++h) half[q][h] = a.tabs[(4 * w + h) & 2047];
        }
#pragma unroll
        for (int q = 0; q < kWpt; ++q) {
            const int w = threadIdx.x + q * TPB;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t first = ((((word[q] >> (4 * k)) & 0xFu) * 0x00204081u) & 0x01010101u) * 0x55u;
                const uint32_t hs = (half[q][k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                const uint32_t d = (hs & 0xFu) | ((hs & 0xF0u) << 4) | ((hs & 0xF00u) << 8) | ((hs & 0xF000u) << 12);
                const uint32_t second = ((d & 0x01010101u) << 1) | ((d & 0x02020202u) << 2) | ((d & 0x04040404u) << 3) |
                                        ((d & 0x08080808u) << 4);
                bmap[w * 8 + k] = first | second;
            }
        }
    }
    const uint8_t *bytes = reinterpret_cast<const uint8_t *>(bmap);
    __syncthreads();
    const int64_t nr = dev_count(a.n_dev, a.n);
    const int64_t S = rfl64(a.seg_cum[nr]);
    const int lane = (int)(threadIdx.x & 63);
    constexpr int kW = TPB / 64;
    const int64_t nw = (int64_t)gridDim.x * kW;
    // the wave's index, read as wave-uniform so its bounds and slab live in SGPRs (r05: as a lane
    // value they cost a 64-bit division per lane and, at 64 VGPRs, two spilled registers)
    const int64_t gw = (int64_t)blockIdx.x * kW + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t lo = rfl64(S * gw / nw), hi = rfl64(S * (gw + 1) / nw);
    // one slab per WAVE (its own running count: no LDS atomic), so the expansion has 8x the slabs
    // to spread over its blocks
    uint4 *slab = a.raw + gw * a.slab;
    int wcnt = 0;
    const uint64_t lt_mask = (1ull << lane) - 1;
    if (lo < hi) {
        int64_t ra = 0, rb = nr;
        while (rb - ra > 1) {
            const int64_t step = (rb - ra + 63) / 64;
            const int64_t idx = ra + (int64_t)lane * step;
            const bool le = idx < rb && a.seg_cum[idx] <= lo;
            const int c = __popcll(__ballot(le));
            ra = rfl64(ra + (int64_t)(c - 1) * step);
            rb = rfl64(min(rb, ra + step));
        }
        int64_t rc = ra, s0c = rfl64(a.seg_cum[ra]);
        ReadMeta mc = read_meta(a, rc, nr, S), mn = read_meta(a, rc + 1, nr, S);
        auto advance = [&](int64_t b) {
            while (b >= mc.s1) {
                ++rc;
                s0c = mc.s1;
                mc = mn;
                mn = read_meta(a, rc + 1, nr, S);
            }
        };
        auto map = [&](int64_t b, int32_t &r, int &p, int64_t &off, int &len) -> bool {
            const int64_t sg = b + lane;
            if (sg >= hi) return false;
            if (sg < mc.s1) {
                r = (int32_t)rc; p = (int)(sg - s0c) * kSeg; off = mc.off; len = mc.len;
            } else if (sg < mn.s1) {
                r = (int32_t)rc + 1; p = (int)(sg - mc.s1) * kSeg; off = mn.off; len = mn.len;
            } else {
                int64_t rr = rc + 2;
                int64_t e = a.seg_cum[rr + 1];
                while (e <= sg) e = a.seg_cum[++rr + 1];
                r = (int32_t)rr;
                p = (int)(sg - a.seg_cum[rr]) * kSeg;
                off = a.v_off[rr];
                len = a.v_len[rr];
            }
            return true;
        };
        auto fetch = [&](int64_t off, int p, int len, uint32_t (&d)[10]) {
            const uint32_t *q = reinterpret_cast<const uint32_t *>(a.codes + off + p);
            const uint32_t *q1 = p + 16 <= len ? q + 4 : q;
            const uint32_t *q2 = p + 24 <= len ? q + 8 : q;
#pragma unroll
            for (int t = 0; t < 4; ++t) d[t] = q[t];
#pragma unroll
            for (int t = 0; t < 4; ++t) d[4 + t] = q1[t];
            d[8] = q2[0];
            d[9] = q2[1];
        };
        struct Seg {
            uint32_t d[10];
            int32_t rd;                                // the round's read (< 2^31 reads a round)
            int p, len;
            bool act;
        };
        auto issue = [&](int64_t bb, Seg &g) {
            g.act = false;
            if (bb >= hi) return;
            advance(bb);
            int64_t off = 0;
            g.act = map(bb, g.rd, g.p, off, g.len);
            if (g.act) fetch(off, g.p, g.len, g.d);
        };
        // every lane of the wave takes part (the hit slots are reserved with wave-wide ballots and
        // lane 63's prefix); a lane without a segment contributes no hit
        auto process = [&](const Seg &g) {
            const uint32_t (&d)[10] = g.d;
            const int32_t crd = g.rd;
            const int cp = g.p, clen = g.len;
            // ---- the segment's 32 positions: packed codes, one extract + one byte-map read each ----
            // (r05: 4 bases -> a byte with one v_dot4_u32_u8 of the masked codes against 64/16/4/1 --
            // 2 VALU per dword instead of 5)
            uint32_t v[10];
#pragma unroll
            for (int t = 0; t < 10; ++t) v[t] = pack4_dot(d[t]);
            const uint32_t P0 = (((v[0] << 8) | v[1]) << 16) | (v[2] << 8) | v[3];
            const uint32_t P1 = (((v[4] << 8) | v[5]) << 16) | (v[6] << 8) | v[7];
            const uint32_t P2 = ((v[8] << 8) | v[9]) << 16;                  // bases 32-39 on top
            const uint32_t Q0 = __builtin_amdgcn_alignbit(P0, P1, 16);   // bases 8-23
            const uint32_t Q1 = __builtin_amdgcn_alignbit(P1, P2, 16);   // bases 24-39
            // (the reads of 16 positions issued together: LDS latency, not issue, is the risk at the
            // 4 waves per SIMD the two byte maps leave)
            // one pair-map read per two positions: the byte of the 8-mer at even i, then the 2-bit
            // field of the base at i + 8 -- (hit at i, hit at i + 1) -- straight into the mask (r05:
            // half the LDS reads and bank-conflict cycles, ~58 % of the LDS array's time before; the
            // scan's time did not move, r05u / r05v: it is not LDS-bound, nor load-depth-bound -- a
            // third segment in flight per lane was measured neutral too)
            // r05: the selecting bases (i + 8 for even i = bases 8, 10, .., 38) doubled in place,
            // one per nibble of X0 (bases 8-22) / X1 (24-38), base 8 on top: pair k's field offset
            // is X >> (28 - 4 (k & 7)), whose low 5 bits -- all v_bfe_u32 reads of an offset -- are
            // the nibble and a zero bit. 3 VALU per pair (shift, bfe, shift-or) instead of ~5.5.
            const uint32_t X0 = (Q0 >> 1) & 0x66666666u, X1 = (Q1 >> 1) & 0x66666666u;
            uint32_t hits = 0;
#pragma unroll
            for (int h = 0; h < kSeg; h += 16) {
                uint32_t m[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int i = h + 2 * j;
                    const uint32_t src = i < 8 ? P0 : i < 16 ? Q0 : i < 24 ? P1 : Q1;
                    m[j] = bytes[(src >> (16 - 2 * (i & 7))) & 0xFFFFu];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int i = h + 2 * j;
                    const uint32_t x = h < 16 ? X0 : X1;
                    hits |= __builtin_amdgcn_ubfe(m[j], x >> (28 - 4 * j), 2u) << i;
                }
            }
            // ---- validity: N bytes and the read end (doubling ORs of the invalid-byte mask) ----
            const int rem = clen - cp;
            uint32_t nor = 0;
#pragma unroll
            for (int t = 0; t < 10; ++t) nor |= d[t];
            uint64_t inv = 0;
            uint32_t slow = 0;
            if ((nor & 0x04040404u) || rem < 40) {
#pragma unroll
                for (int t = 0; t < 10; ++t)
                    inv |= (uint64_t)((((d[t] >> 2) & 0x01010101u) * 0x10204080u) >> 28) << (4 * t);
                if (rem < 64) inv |= ~0ull << rem;
                const uint64_t t1 = inv | (inv >> 1), t2 = t1 | (t1 >> 2), t3 = t2 | (t2 >> 4);
                const uint32_t full8 = ~(uint32_t)t3;
                hits &= full8;
                if (a.min_k < kMaxK) slow = ~(uint32_t)(t2 | (t2 >> (a.min_k - kMinK))) & ~full8;
            }
            // the lane's hits go to consecutive slab slots: a wave prefix of the hit counts (one ballot
            // per count bit that any lane has), one LDS atomic per wave and segment, then each lane
            // writes its own (a loop of the wave's most hits per lane, usually 1-2)
            uint32_t left = g.act ? hits | slow : 0u;
            const int cnt = __popc(left);
            if (__any(cnt != 0)) {                     // wave-uniform
                int excl = 0;
                for (int bit = 0; bit < 6; ++bit) {    // wave-uniform
                    if (!__any((cnt >> bit) != 0)) break;
                    excl += __popcll(__ballot((cnt >> bit) & 1) & lt_mask) << bit;
                }
                const int total = __builtin_amdgcn_readlane(excl + cnt, 63);
                int slot = wcnt + excl;
                wcnt += total;
                while (left) {
                    const int i = __builtin_ctz(left);
                    left &= left - 1;
                    // the position's 8-mer from the packed words (N bytes read as code 0, as the
                    // bytes' low bits; bases past a short run are not used by the expansion)
                    const uint32_t src = i < 8 ? P0 : i < 16 ? Q0 : i < 24 ? P1 : Q1;
                    const uint32_t c8 = (src >> (16 - 2 * (i & 7))) & 0xFFFFu;
                    const uint32_t run = (slow >> i) & 1u ? (uint32_t)min(8, __builtin_ctzll(inv >> i)) : 8u;
                    if (slot < a.slab)
                        slab[slot] = make_uint4((uint32_t)crd, (uint32_t)(cp + i) | ((slow >> i) & 1u ? kSlowBit : 0u),
                                                c8 | (run << 16), (uint32_t)(clen - (cp + i)));
                    ++slot;
                }
            }
        };
        Seg sa, sb;
#pragma unroll
        for (int t = 0; t < 10; ++t) sa.d[t] = sb.d[t] = 0x04040404u;
        sb.rd = 0;
        sb.p = sb.len = 0;
        sb.act = false;
        int64_t b = lo;
        issue(b, sa);
        while (b < hi) {                               // wave-uniform
            issue(b + 64, sb);
            process(sa);
            b += 64;
            if (b >= hi) break;
            issue(b + 64, sa);
            process(sb);
            b += 64;
        }
    }
    if (lane == 0) {
        a.raw_cnt[gw] = min(wcnt, a.slab);
        if (wcnt > a.slab) atomicOr(&a.flags[0], 1);
    }
}

// Resident blocks striding over the slabs: the probe entries of the slabs' raw hits become tasks.
// The raw hits carry their 8-mer and valid run, so nothing here touches the reads: the slabs, the
// LDS image and the task stores. A block first counts its tasks per class (all its slabs) and
// takes its place with one atomic per class -- one per block, not per 256 hits: a few thousand
// same-address atomics serialise at the L2 -- then writes them, 256 hits at a time at the offsets
// of a block scan of their counts (the LDS lookups are repeated; they are cheap).
// Counts are packed per class pair: inside tasks (classes 0 | 1 << 32) and edge tasks likewise.
struct TaskCount {
    long long in, edge;
};

template <bool WRITE>
__device__ __forceinline__ TaskCount expand_hit(const ScanArgs &a, const uint32_t *lds, const uint16_t *rank,
                                                const uint16_t *estart, const int32_t *ent, const uint32_t *ent2,
                                                const uint4 &r, TaskCount at) {
    const int64_t rd = r.x;
    const int q = (int)(r.y & ~kSlowBit);
    const bool fast = !(r.y & kSlowBit);
    const uint32_t c8 = r.z & 0xFFFFu;
    const int run = (int)(r.z >> 16);
    const int dist = (int)r.w;                           // read length - q
    const int64_t probe0 = WRITE && (a.pin_cls[0] | a.pin_cls[1]) ? a.v_off[rd] + q : 0;
    TaskCount c{0, 0};
    for (int kk = fast ? kNK - 1 : 0; kk < (fast ? kNK : kNK - 1); ++kk) {
        const int K = kMinK + kk;
        if (a.bits_off[kk] < 0 || (!fast && K > run)) continue;
        const uint32_t code = c8 >> (2 * (kMaxK - K));
        const int dw = a.bits_off[kk] + (int)(code >> 5);
        const uint32_t word = lds[dw], bit = 1u << (code & 31);
        if (!(word & bit)) continue;
        const int rr = rank[dw] + __popc(word & (bit - 1));
        const int e = estart[rr + 1];
        for (int b = estart[rr]; b < e; ++b) {
            const int en = ent[b];                       // adapter << 12 | (K - 4) << 9 | class << 8 | offset
            const uint32_t lim = ent2[b];
            const bool inside = q >= (int)(lim & 0xFFFFu) && dist > (int)(lim >> 16);
            const int cls = (en >> 8) & 1;
            const long long one = cls ? (1ll << 32) : 1ll;
            if (WRITE) {
                const long long sh = cls ? 32 : 0;
                int4 *region = a.task + cls * (a.cap + a.ecap);
                if (inside) {
                    const long long g = (at.in >> sh) & 0xFFFFFFFFll;
                    at.in += one;
                    if (g < a.cap) {
                        if (a.pin_cls[cls])
                            region[g] = make_int4((int)rd, ((en >> 12) << 11) | (((en >> 9) & 7) << 8) | (en & 255), (int)(uint32_t)probe0,
                                                  (int)(uint32_t)((uint64_t)probe0 >> 32));
                        else
                            region[g] = make_int4((int)rd, en >> 12, q - (en & 255), en & 255);
                    }
                } else {
                    const long long g = (at.edge >> sh) & 0xFFFFFFFFll;
                    at.edge += one;
                    if (g < a.ecap) region[a.cap + g] = make_int4((int)rd, en >> 12, q - (en & 255), en & 255);
                }
            } else {
                if (inside) c.in += one;
                else c.edge += one;
            }
        }
    }
    return c;
}

// 1024-thread blocks (r04): the probe image takes ~60 KB of LDS, so two blocks fit a CU; with
// quarter-size blocks that was 8 waves per CU and the expansion waited on its loads and barriers
// (PMC: waves waiting ~88 % of their lifetime) over ~3.5 generations of blocks
constexpr int kExpandThreads = 1024;

// The probe image (up to ~60 KB) into LDS: 16-B loads, four in flight per thread (a dword loop
// waited out one load latency per dword: ~50 us of fixed cost per launch, most of a small round's).
__device__ __forceinline__ void expand_load_image(const ScanArgs &a, uint32_t *lds) {
    const int n4 = a.tab_dw / 4;
    const uint4 *src = reinterpret_cast<const uint4 *>(a.tabs);
    uint4 *dst = reinterpret_cast<uint4 *>(lds);
    constexpr int T = kExpandThreads;
    for (int i = threadIdx.x; i < n4; i += 4 * T) {
        const bool f1 = i + T < n4, f2 = i + 2 * T < n4, f3 = i + 3 * T < n4;
        const uint4 v0 = src[i];
        const uint4 v1 = src[f1 ? i + T : i], v2 = src[f2 ? i + 2 * T : i], v3 = src[f3 ? i + 3 * T : i];
        dst[i] = v0;
        if (f1) dst[i + T] = v1;
        if (f2) dst[i + 2 * T] = v2;
        if (f3) dst[i + 3 * T] = v3;
    }
    for (int i = 4 * n4 + (int)threadIdx.x; i < a.tab_dw; i += T) lds[i] = a.tabs[i];
}

// Two exclusive block sums at once (one set of barriers): s_w holds 2 x kExpandThreads / 64.
__device__ __forceinline__ void expand_excl_sum2(long long v0, long long v1, long long &ex0, long long &ex1,
                                                 long long &t0, long long &t1, long long *s_w) {
    constexpr int NW = kExpandThreads / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    long long x0 = v0, x1 = v1;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const long long y0 = __shfl_up(x0, d), y1 = __shfl_up(x1, d);
        if (lane >= d) {
            x0 += y0;
            x1 += y1;
        }
    }
    if (lane == 63) {
        s_w[w] = x0;
        s_w[NW + w] = x1;
    }
    __syncthreads();
    if (w == 0) {
        long long y0 = lane < NW ? s_w[lane] : 0, y1 = lane < NW ? s_w[NW + lane] : 0;
#pragma unroll
        for (int d = 1; d < NW; d <<= 1) {
            const long long z0 = __shfl_up(y0, d), z1 = __shfl_up(y1, d);
            if (lane >= d) {
                y0 += z0;
                y1 += z1;
            }
        }
        if (lane < NW) {
            s_w[lane] = y0;
            s_w[NW + lane] = y1;
        }
    }
    __syncthreads();
    t0 = s_w[NW - 1];
    t1 = s_w[2 * NW - 1];
    ex0 = x0 - v0 + (w ? s_w[w - 1] : 0);
    ex1 = x1 - v1 + (w ? s_w[NW + w - 1] : 0);
    __syncthreads();                                     // s_w is reused by the next call
}

// One-pass expansion (r04, the default): a block's slabs (blockIdx.x + k * gridDim.x) in
// groups of kExpandGroup are one flat run of hits (a prefix of their counts in LDS), taken
// kExpandHits per thread at a time: each hit's probe walk counts its tasks (kept in registers), a
// block scan places them, one atomic per class and pass takes the block's place, and the second
// walk writes. The two-pass kernel walks every hit three times and runs a slab at a time (~1.1 k
// hits per slab in round 1 of 8 kb reads: a 1024-thread pass half idle, two scans per slab; r04:
// 0.25 -> 0.18 ms per 8 kb step, profiles/r04/r04l/).
// kExpandHits hits per thread and pass (r05bb: 3 fits 64 VGPRs under amdgpu_waves_per_eu(8), two
// blocks per CU, and beats 2 in-process: 1.938 -> 1.924 ms at 8 kb, 2.495 -> 2.462 at 20 kb; 4
// spills there)
constexpr int kExpandGroup = 64;
constexpr int kExpandHits = 3;
template <int HITS>
__global__ __launch_bounds__(kExpandThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_seed_expand1(ScanArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    __shared__ long long s_w[2 * (kExpandThreads / 64)];
    __shared__ long long s_base[2];
    __shared__ int s_pre[kExpandGroup + 1];
    expand_load_image(a, lds);
    __syncthreads();
    const uint16_t *rank = reinterpret_cast<const uint16_t *>(lds + a.rank_off);
    const uint16_t *estart = reinterpret_cast<const uint16_t *>(lds + a.estart_off);
    const int32_t *ent = reinterpret_cast<const int32_t *>(lds + a.ent_off);
    const uint32_t *ent2 = lds + a.ent2_off;
    const int G = (int)gridDim.x, b = (int)blockIdx.x;
    const int mine = b < a.n_slab ? (a.n_slab - b + G - 1) / G : 0;     // block-uniform
    for (int g0 = 0; g0 < mine; g0 += kExpandGroup) {
        const int ng = min(kExpandGroup, mine - g0);
        if (threadIdx.x < 64) {                          // wave 0: inclusive prefix of the group's counts
            const int l = (int)threadIdx.x;
            int x = l < ng ? a.raw_cnt[b + (g0 + l) * G] : 0;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int y = __shfl_up(x, d);
                if (l >= d) x += y;
            }
            s_pre[l + 1] = x;
            if (l == 0) s_pre[0] = 0;
        }
        __syncthreads();
        const int total = s_pre[ng];
        for (int base = 0; base < total; base += HITS * kExpandThreads) {
            uint4 r[HITS];
            uint64_t pc[HITS];                    // a hit's four counts in 16 bits each (a hit
                                                         // has fewer tasks than the table has entries)
            long long si = 0, se = 0;
#pragma unroll
            for (int j = 0; j < HITS; ++j) {
                const int f = base + j * kExpandThreads + (int)threadIdx.x;
                pc[j] = 0;
                r[j] = make_uint4(0u, 0u, 0u, 0u);
                if (f < total) {
                    int lo = 0, hi = ng - 1;             // the slab k holding f: s_pre[k] <= f < s_pre[k + 1]
                    while (lo < hi) {
                        const int m = (lo + hi + 1) >> 1;
                        if (s_pre[m] <= f) lo = m;
                        else hi = m - 1;
                    }
                    r[j] = a.raw[(int64_t)(b + (g0 + lo) * G) * a.slab + (f - s_pre[lo])];
                    const TaskCount c = expand_hit<false>(a, lds, rank, estart, ent, ent2, r[j], TaskCount{0, 0});
                    si += c.in;
                    se += c.edge;
                    pc[j] = (uint64_t)(c.in & 0xFFFF) | (uint64_t)((c.in >> 32) & 0xFFFF) << 16 |
                            (uint64_t)(c.edge & 0xFFFF) << 32 | (uint64_t)((c.edge >> 32) & 0xFFFF) << 48;
                }
            }
            long long exi, exe, ti, te;
            expand_excl_sum2(si, se, exi, exe, ti, te, s_w);
            if (threadIdx.x == 0) {
                long long bb[2] = {0, 0};
                bool over = false;
                for (int cl = 0; cl < kCls; ++cl) {
                    const long long xi = (ti >> (32 * cl)) & 0xFFFFFFFFll, xe = (te >> (32 * cl)) & 0xFFFFFFFFll;
                    const long long bi = xi ? atomicAdd(&a.cnt[cl], (int)xi) : 0;
                    const long long be = xe ? atomicAdd(&a.cnt[kCls + cl], (int)xe) : 0;
                    bb[0] |= bi << (32 * cl);
                    bb[1] |= be << (32 * cl);
                    over |= bi + xi > a.cap || be + xe > a.ecap;
                }
                s_base[0] = bb[0];
                s_base[1] = bb[1];
                if (over) atomicOr(&a.flags[1], 1);
            }
            __syncthreads();
            TaskCount at{s_base[0] + exi, s_base[1] + exe};
#pragma unroll
            for (int j = 0; j < HITS; ++j) {
                if (pc[j]) {                             // hits without tasks write nothing
                    expand_hit<true>(a, lds, rank, estart, ent, ent2, r[j], at);
                    at.in += (long long)(pc[j] & 0xFFFF) | (long long)((pc[j] >> 16) & 0xFFFF) << 32;
                    at.edge += (long long)((pc[j] >> 32) & 0xFFFF) | (long long)(pc[j] >> 48) << 32;
                }
            }
            __syncthreads();                             // s_base is rewritten by the next pass
        }
        __syncthreads();                                 // s_pre likewise
    }
}

// The band's read bytes as a stream: rd[p], rd[p + 1], ... one dword load per 4 bytes, issued one
// dword ahead (the band DP of a random probe hit usually stops within a dozen rows, so the first
// loads cover most tasks). Reads at most 11 bytes past the last byte taken.
// CLAMP (edge bands, which run off the read): every dword address is clamped into [lo, hi] --
// the bytes outside the read are masked by the caller, so their values do not matter, but no load
// leaves the codes buffer.
template <bool CLAMP>
struct ByteStream {
    const uint32_t *q;
    uint64_t buf;
    uint32_t nx;
    int o;
    uintptr_t lo, hi;
    __device__ __forceinline__ uint32_t ld(const uint32_t *a) const {
        if (!CLAMP) return *a;
        const uintptr_t x = (uintptr_t)a;
        return *reinterpret_cast<const uint32_t *>(x < lo ? lo : (x > hi ? hi : x));
    }
    __device__ __forceinline__ ByteStream(const uint8_t *p, uintptr_t lo_ = 0, uintptr_t hi_ = 0) : lo(lo_), hi(hi_) {
        const int a0 = (int)((uintptr_t)p & 3);
        q = reinterpret_cast<const uint32_t *>(p - a0);
        buf = ((uint64_t)ld(q + 1) << 32) | ld(q);
        nx = ld(q + 2);
        q += 3;
        o = 8 * a0;
    }
    __device__ __forceinline__ int next() {
        const int v = (int)((buf >> o) & 0xFFu);
        o += 8;
        if (o == 32) {
            buf = (buf >> 32) | ((uint64_t)nx << 32);
            nx = ld(q++);
            o = 0;
        }
        return v;
    }
};

// Banded score DP of one task: rows i = 1..L of the adapter, per row the 2E+1 cells of the
// diagonals d0 - E .. d0 + E (cell x <-> read column j = i + d0 + x - E), free end gaps as the
// full DP: S(0, j) = 0, S(i, 0) = 0, ends in row L (j < len) or in the last column (j = len).
// CHECK: the band touches column 0 or the last column, or leaves the read. Only the rows whose
// columns reach 0 or len take the checked cells (r04: every row did, 20 k edge tasks cost ~75 us
// per round, a tail behind the pinned bands); the other rows of an edge band are inside rows.
// Early exit: no path gains more than best_sub per remaining row (gaps cost), so once every cell
// of row i satisfies S + best_sub (L - i) < T, every cell of the later rows does too -- row L and
// the last column's cells alike -- unless a later row restarts in column 0 (an edge band whose
// columns are not yet past 0). Then, if no last-column end so far reached T, the pair cannot reach
// T: the DP stops and returns a bound below T, which is all the caller compares. Random probe hits
// -- most tasks, edge tasks included (r04: an edge band never exited, and its last rows are all
// checked cells: ~75 us per launch, the band phase's critical path) -- stop early.
template <int E, bool CHECK>
__device__ __forceinline__ int band_best(const uint8_t *rd, int len, const uint8_t *ac, int L, int d0,
                                         const pcabi::Scoring &sc, int T, const uint8_t *codes) {
    constexpr int W = 2 * E + 1;
    int S[W], V[W], R[W];
    // rd[d0 - E] onwards; an edge band's columns outside 1 .. len are masked (7 never matches) and
    // its loads stay inside [rd, rd + len] (the read's own start and end, dword-aligned: the read may
    // lie in the caller's codes or in the scan's shadow arena of masked copies, r05)
    (void)codes;
    ByteStream<CHECK> bs(rd + (d0 - E), (uintptr_t)rd & ~(uintptr_t)3, ((uintptr_t)(rd + len)) & ~(uintptr_t)3);
#pragma unroll
    for (int x = 0; x < W; ++x) {
        const int j0 = d0 + x - E;                           // row 0
        S[x] = (!CHECK || (j0 >= 0 && j0 <= len)) ? 0 : kNeg;
        V[x] = kNeg;
        const int j1 = j0 + 1;                               // row 1's read column
        const int v = bs.next();
        R[x] = CHECK ? ((j1 >= 1 && j1 <= len) ? v : 7) : v;
    }
    int best = 0;                                            // S(L, 0) = 0 is always scouted
    for (int i = 1; i <= L; ++i) {
        const int ab = ac[i - 1];
        int h = kNeg, sl = kNeg;                             // H, S of the cell to the left
        const bool edge_row = CHECK && (i + d0 - E <= 0 || i + d0 + E >= len);
        if (edge_row) {
#pragma unroll
            for (int x = 0; x < W; ++x) {
                const int dg = S[x] + ((R[x] == ab) ? sc.ma : sc.mi);
                const int vu = (x + 1 < W) ? max(V[x + 1] + sc.ge, S[x + 1] + sc.go) : kNeg;
                h = max(h + sc.ge, sl + sc.go);
                int s = max(dg, max(vu, h)), v = vu;
                const int j = i + d0 + x - E;
                if (j == 0) { s = 0; v = kNeg; h = kNeg; }              // the adapter head hangs off
                else if (j < 0 || j > len) { s = kNeg; v = kNeg; h = kNeg; }
                if (j == len) best = max(best, s);                      // last column
                S[x] = s;
                V[x] = v;
                sl = s;
            }
        } else {
#pragma unroll
            for (int x = 0; x < W; ++x) {
                const int dg = S[x] + ((R[x] == ab) ? sc.ma : sc.mi);
                const int vu = (x + 1 < W) ? max(V[x + 1] + sc.ge, S[x + 1] + sc.go) : kNeg;
                h = max(h + sc.ge, sl + sc.go);
                const int s = max(dg, max(vu, h));
                S[x] = s;
                V[x] = vu;
                sl = s;
            }
        }
#pragma unroll
        for (int x = 0; x + 1 < W; ++x) R[x] = R[x + 1];
        const int jn = i + 1 + d0 + E;
        if (i < L) {
            const int v = bs.next();
            R[W - 1] = CHECK ? ((jn >= 1 && jn <= len) ? v : 7) : v;
        }
        if ((i % PCABI_BAND_EXIT) == 0 && (!CHECK || i + d0 - E >= 0)) {   // (no restart after row E - d0)
            int mx = S[0];
#pragma unroll
            for (int x = 1; x < W; ++x) mx = max(mx, S[x]);
            const int ub = mx + pcabi::best_sub(sc) * (L - i);
            if (ub < T && best < T) return max(ub, best);
        }
    }
#pragma unroll
    for (int x = 0; x < W; ++x) {                            // last row, j < len
        const int j = L + d0 + x - E;
        if (!CHECK || (j >= 0 && j < len)) best = max(best, S[x]);
    }
    return best;
}

// Grid-stride over the class's tasks (their count from the device, clamped to the capacity).
// adp_lds > 0: the flat adapter table (that many bytes) is copied to LDS first.
template <int E>
__global__ __launch_bounds__(256) void k_seed_band(const int4 *task, const int32_t *n_task, int64_t cap,
                                                   const uint8_t *codes, const int64_t *v_off, const int32_t *v_len,
                                                   const uint8_t *adp, int32_t adp_lds, const int32_t *adp_off,
                                                   const int32_t *adp_len, pcabi::Scoring sc, const int32_t *thr,
                                                   int32_t *bound, int64_t n, VerOut vo) {
    extern __shared__ uint32_t lds_adp[];
    const uint8_t *ad = adp;
    if (adp_lds > 0) {
        for (int i = threadIdx.x; i < adp_lds / 4; i += 256) lds_adp[i] = reinterpret_cast<const uint32_t *>(adp)[i];
        __syncthreads();
        ad = reinterpret_cast<const uint8_t *>(lds_adp);
    }
    const int64_t nt = min((int64_t)*n_task, cap);
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < nt; t += (int64_t)gridDim.x * 256) {
        const int4 tk = task[t];
        const int L = adp_len[tk.y];
        const int len = v_len[tk.x];
        const int d0 = tk.z;
        const uint8_t *rd = codes + v_off[tk.x];
        const uint8_t *ac = ad + adp_off[tk.y];
        const bool inside = d0 - E >= 1 && d0 + E + L + 1 < len;
        const int T = thr[tk.y];
        const int best = inside ? band_best<E, false>(rd, len, ac, L, d0, sc, T, codes)
                                : band_best<E, true>(rd, len, ac, L, d0, sc, T, codes);
        // only a bound that reaches T is ever read (k_cands, the host's >= T): lower ones stay
        // unwritten, so random probe hits -- most tasks -- cost no atomic
        if (best >= T) atomicMax(&bound[(int64_t)tk.y * n + tk.x], best);
        if (vo.list) put_verified(vo, best >= T, tk.x, tk.y, E, v_off[tk.x] + d0);
    }
}

// ---- the pinned band (inside tasks) ----------------------------------------------------------
// A task comes from probe p of adapter a found at read position q: the piece's first K bases sit on
// diagonal d0 = q - o as K matches (o = p * plen). The seed argument needs only the alignment whose
// piece p is exact -- it passes through those K diagonal matches -- so the bound is the best score
// of band alignments that do: B = P + K * match + Q, with
//   Q: the best suffix from the pinned run's end cell (row o + K, diagonal d0) to the adapter's last
//      row (inside bands end anywhere in it): the band DP of rows o + K + 1 .. L started from that
//      cell -- and from the read bases an alignment may insert right after the run in that same row
//      (a horizontal gap: go, ge, ... to the cell's right);
//   P: the best prefix from row 0 (free start, any band column) to the run's first cell (row o): the
//      same DP run backwards -- the adapter prefix and the read reversed, the band mirrored
//      (x' = 2E - x), which turns the reverse recurrence into the forward one -- started likewise,
//      its best over the last row (row 0).
// B <= the band best (a subset of its alignments) and B >= the score of any alignment whose piece p
// is exact, so a pair whose hit has exact piece p still reaches T through this task: the bound stays
// exact (tests/test_seed_pin_cpu.py checks B against the band DP constrained to the run). Both halves
// start from one cell, so random probe hits fall below T within a few rows, and rows o + 1 .. o + K
// are never computed. Early exit as band_best: the running maximum plus best_sub per remaining row
// plus the other half's bound (best_sub per row before it is known).
//
// Inside tasks (expand, pinned classes) carry (read, adapter << 11 | (K - 4) << 8 | o, the probe's byte offset in
// codes): the read bytes of the whole band, [probe - o - E, probe - o + L + E), are one range. Per
// lane the range of the NEXT task is loaded (uint4 loads) while the current task computes, then
// copied to the lane's LDS slot (NC4 x 16 bytes), where the rows read their one new byte each: the
// row loop touches no global memory, so no wait of the loop is a memory latency.
//
// STATS (the profiled launches of pcabi_scan_profile only): per wave, row iterations x 64 lanes,
// active lane-rows (the band cells computed: x (2E + 1)), tasks and passes, added to the wave's own
// four counters stats[4 * (block * 4 + wave) ..] at its end (plain stores: same-address atomics from
// every pass serialise at the L2 and cost more than the bands, r05l) -- the roofline's work and the
// lanes a pass leaves idle behind its longest task.
template <int E, int NC4, bool STATS>
__global__ __launch_bounds__(256) void k_seed_band_pin(const int4 *task, const int32_t *n_task, int64_t cap,
                                                       const uint8_t *codes, const uint8_t *adp, int32_t adp_dw,
                                                       const int32_t *adp_off, const int32_t *adp_meta, int32_t n_adp,
                                                       pcabi::Scoring sc, int32_t *bound, int64_t n, VerOut vo,
                                                       unsigned long long *stats) {
    constexpr int W = 2 * E + 1;
    extern __shared__ uint4 lds4[];
    uint32_t *lds = reinterpret_cast<uint32_t *>(lds4);
    // LDS: the flat adapters (adp_dw dwords), their offsets, their meta (L | T << 12), then
    // per lane NC4 uint4 of read bytes
    for (int i = threadIdx.x; i < adp_dw; i += 256) lds[i] = reinterpret_cast<const uint32_t *>(adp)[i];
    for (int i = threadIdx.x; i < n_adp; i += 256) {
        lds[adp_dw + i] = (uint32_t)adp_off[i];
        lds[adp_dw + n_adp + i] = (uint32_t)adp_meta[i];
    }
    __syncthreads();
    const uint8_t *ad = reinterpret_cast<const uint8_t *>(lds);
    const int32_t *aoffs = reinterpret_cast<const int32_t *>(lds + adp_dw);
    const int32_t *ameta = aoffs + n_adp;
    uint4 *slot4 = lds4 + ((adp_dw + 2 * n_adp + 3) >> 2) + (int)threadIdx.x * NC4;
    const uint8_t *slot = reinterpret_cast<const uint8_t *>(slot4);
    const int64_t nt = min((int64_t)*n_task, cap);
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int bs = pcabi::best_sub(sc), ma = sc.ma, mi = sc.mi, go = sc.go, ge = sc.ge;
    const uintptr_t lo_addr = (uintptr_t)codes & ~(uintptr_t)15;
    // the range of a task: [cb, cb + 16 * nld) with cb = (probe - o - E) & ~15. An inside band lies
    // within its read, so the range starts inside the read's buffer; the clamp to the start of the
    // caller's codes is a guard for reads there only (a masked copy in the scan's shadow arena, r05,
    // may lie below codes; the arena's first 256 bytes are a lead-in no copy uses)
    auto range_of = [&](const int4 &rc, uintptr_t &cb, int &nld) {
        const int a = rc.y >> 11, o = rc.y & 255;
        const int L = (int)((uint32_t)ameta[a] & 255u);
        const uintptr_t pa = (uintptr_t)codes + (uintptr_t)(((uint64_t)(uint32_t)rc.w << 32) | (uint32_t)rc.z);
        const uintptr_t lo = pa - (uintptr_t)(o + E), hi = pa - (uintptr_t)o + (uintptr_t)(L + E);
        cb = lo & ~(uintptr_t)15;
        if (pa >= lo_addr && cb < lo_addr) cb = lo_addr;
        nld = (int)((hi - cb + 15) >> 4);
    };
    // ---- pipeline: recA / chA = the task to copy into the slot next, recB = the one after
    int4 recA = make_int4(0, 0, 0, 0), recB = recA;
    bool vA = false, vB = false;
    uint4 chA[NC4];
    uintptr_t cbA = lo_addr;
    auto load_range = [&]() {                         // chA := recA's range (recA has arrived)
        int nld = 0;
        range_of(recA, cbA, nld);
#pragma unroll
        for (int k = 0; k < NC4; ++k)
            chA[k] = k < nld ? *reinterpret_cast<const uint4 *>(cbA + 16 * (uintptr_t)k) : make_uint4(0u, 0u, 0u, 0u);
    };
    if (t < nt) { recA = task[t]; vA = true; t += stride; }
    if (vA) load_range();
    if (t < nt) { recB = task[t]; vB = true; t += stride; }
    auto pin_start = [&](int x) -> int { return x == E ? 0 : (x > E ? go + (x - E - 1) * ge : kNeg); };
    unsigned long long st_it = 0, st_act = 0, st_tasks = 0, st_pass = 0;
    while (__any(vA)) {                               // one task per lane and pass
        bool active = vA;
        int4 rc = recA;
        uintptr_t cb = cbA;
        if (vA) {
#pragma unroll
            for (int k = 0; k < NC4; ++k) slot4[k] = chA[k];
        }
        // the pipeline moves on: B's range loads while this task computes
        vA = vB;
        recA = recB;
        if (vA) load_range();
        vB = t < nt;
        if (vB) {
            recB = task[t];
            t += stride;
        }
        // ---- this task
        const bool vA_was = active;
        const int a = rc.y >> 11, o = rc.y & 255, K = kMinK + ((rc.y >> 8) & 7);
        const uint32_t meta = (uint32_t)ameta[a];
        const int L = (int)(meta & 255u), T = (int)(meta >> 12);
        const int aoff = aoffs[a];
        const int64_t bidx = (int64_t)a * n + rc.x;
        const uintptr_t pa = (uintptr_t)codes + (uintptr_t)(((uint64_t)(uint32_t)rc.w << 32) | (uint32_t)rc.z);
        const int base = (int)(pa - cb);              // the probe's byte in the slot
        const int pin = ma * K;
        int S[W], V[W], R[W];
        int phase = 0, rows = L - o - K, other = pin + bs * o, mx = 0;
        int apos = aoff + o + K, adir = 1;
        int bpos = base + K + E + 1, bdir = 1;          // the slot byte entering the next row
#pragma unroll
        for (int x = 0; x < W; ++x) {
            S[x] = pin_start(x);
            V[x] = kNeg;
            R[x] = active ? slot[base + K + x - E] : 0;   // row o + K + 1: read q + K + x - E
        }
        auto begin_prefix = [&]() {                   // rows o .. 1 backwards, mirrored band
            phase = 1;
            rows = o;
            other = pin + mx;                         // K * match + Q
            mx = 0;
#pragma unroll
            for (int x = 0; x < W; ++x) {
                S[x] = pin_start(x);
                V[x] = kNeg;
                R[x] = slot[base - 1 + E - x];        // read q - 1 + E - x
            }
            bpos = base - 2 - E;
            bdir = -1;
            apos = aoff + o - 1;
            adir = -1;
        };
        // the task's diagonal as a codes offset (probe - o): the verified-seed record
        const int64_t dabs = (int64_t)(((uint64_t)(uint32_t)rc.w << 32) | (uint32_t)rc.z) - o;
        // the task's verified flag (set once, where its lane finishes): one record call per task
        // after the row loop, not a ballot per row (r05)
        bool ver = false;
        if (active && rows == 0) {                    // the run ends the adapter: Q = 0
            if (o == 0) {
                if (pin >= T) atomicMax(&bound[bidx], pin);
                ver = pin >= T;
                active = false;
            } else {
                begin_prefix();
            }
        }
        if constexpr (STATS) {
            st_tasks += __popcll(__ballot(vA_was));
            st_pass += 1;
        }
        while (__any(active)) {
            if constexpr (STATS) {
                st_it += 64;
                st_act += __popcll(__ballot(active));
            }
            if (active) {
                const int ab = ad[apos];
                apos += adir;
                const int nb = slot[bpos];
                bpos += bdir;
                int h = kNeg, sl = kNeg;
#pragma unroll
                for (int x = 0; x < W; ++x) {
                    const int dg = S[x] + (R[x] == ab ? ma : mi);
                    const int vu = (x + 1 < W) ? max(V[x + 1] + ge, S[x + 1] + go) : kNeg;
                    h = max(h + ge, sl + go);
                    const int sv = max(dg, max(vu, h));
                    S[x] = sv;
                    V[x] = vu;
                    sl = sv;
                }
#pragma unroll
                for (int x = 0; x + 1 < W; ++x) R[x] = R[x + 1];
                R[W - 1] = nb;
                --rows;
                mx = S[0];
#pragma unroll
                for (int x = 1; x < W; ++x) mx = max(mx, S[x]);
                const int ub = mx + bs * rows + other;
                if (ub < T) {                         // below T: nothing to record (k_seed_band)
                    active = false;
                } else if (rows == 0) {
                    if (phase == 0 && o > 0) {
                        begin_prefix();
                    } else {
                        ver = mx + other >= T;
                        if (ver) atomicMax(&bound[bidx], mx + other);
                        active = false;
                    }
                }
            }
        }
        if (vo.list) put_verified(vo, ver, rc.x, a, E, dabs);
    }
    if constexpr (STATS) {
        if ((threadIdx.x & 63) == 0) {
            unsigned long long *w = stats + 4 * ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6));
            w[0] += st_it;
            w[1] += st_act;
            w[2] += st_tasks;
            w[3] += st_pass;
        }
    }
}

// The pairs whose bound reaches their adapter's threshold T[a], as (a << 32 | read) keys
// (unordered; one atomic per wave), grid-stride over the n_dev x n_adp bounds (row stride n).
// pmap != nullptr (the device rounds; pmap may be `bound` itself): a candidate pair's entry becomes its
// index in the list, which its verified seeds' windows look up.
__global__ __launch_bounds__(256) void k_cands(const int32_t *bound, int64_t n, const int32_t *n_dev, int32_t n_adp,
                                               const int32_t *T, int64_t *out, int64_t cap, unsigned long long *cnt,
                                               int32_t *pmap) {
    const int64_t nr = dev_count(n_dev, n);
    const int64_t total = nr * n_adp;
    const int lane = threadIdx.x & 63;
    for (int64_t base = (int64_t)blockIdx.x * 256; base < total; base += (int64_t)gridDim.x * 256) {   // uniform
        const int64_t i = base + threadIdx.x;
        const int64_t a = nr > 0 ? i / nr : 0, r = i - a * nr;
        const bool want = i < total && bound[a * n + r] >= T[a];
        const uint64_t m = __ballot(want);
        if (!m) continue;
        const int leader = __ffsll((unsigned long long)m) - 1;
        unsigned long long b0 = 0;
        if (lane == leader) b0 = atomicAdd(cnt, (unsigned long long)__popcll(m));
        b0 = __shfl(b0, leader);
        if (want) {
            const unsigned long long slot = b0 + __popcll(m & ((1ull << lane) - 1));
            if ((int64_t)slot < cap) {
                out[slot] = (a << 32) | r;
                if (pmap) pmap[a * n + r] = (int32_t)slot;
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_bound16(const int32_t *bound, int64_t cnt, int16_t *s16) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < cnt) s16[i] = (int16_t)max(min(bound[i], 32767), -32768);
}

// bound[a * n + r] = NEG16 for the n_dev x n_adp live entries (row stride n); block 0 also zeroes
// the counters of the launches that follow (z32[0 .. nz32), *z64 when given).
__global__ __launch_bounds__(256) void k_bound_reset(int32_t *bound, int64_t n, const int32_t *n_dev, int32_t n_adp,
                                                     int32_t *z32, int nz32, unsigned long long *z64) {
    if (blockIdx.x == 0) {
        if (threadIdx.x < nz32) z32[threadIdx.x] = 0;
        if (z64 && threadIdx.x == 0) *z64 = 0ull;
    }
    const int64_t nr = dev_count(n_dev, n);
    const int64_t total = nr * n_adp;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t a = i / nr;
        bound[a * n + (i - a * nr)] = pcabi::sf::NEG16;
    }
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
        g_buf_gen.fetch_add(1);
        const hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
            return fail(PCABI_E_NOMEM, "hipMalloc failed (seeds, " + std::to_string(want) + " bytes): " + hipGetErrorString(e));
        }
        cap = want;
        pcabi_poison(p, want);
        return 0;
    }
    ~Buf() {
        if (p) (void)hipFree(p);
    }
};

struct State {
    // the second band class runs beside the first on a side stream (fork / join by events)
    hipStream_t side = nullptr, side2 = nullptr;   // class 1's inside tasks; both classes' edge tasks
    hipEvent_t fork = nullptr, join = nullptr, join2 = nullptr;
    ~State() {
        if (side) (void)hipStreamDestroy(side);
        if (side2) (void)hipStreamDestroy(side2);
        if (join2) (void)hipEventDestroy(join2);
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
    size_t lds_bytes = 0;                         // the whole probe image (k_seed_expand1)
    int32_t adp_bytes = 0;                        // flat adapter table, dword-rounded
    ScanArgs a{};
    Buf tabs, adp, adp_off, adp_len, adp_meta, task, cnt, bound, thr, cands, ccnt, raw, rawcnt, segcum, scantmp;
    int pin_nc4[kCls] = {0, 0};                   // class c's pinned band slot (uint4 per lane), 0: band_best
    int32_t n_adp = 0;
    int64_t cap = 0, ecap = 0, ccap = 0, raw_cap = 0;
    int scan_blocks = 0;                          // resident k_seed_scan blocks
    int n_slab = 0;                               // raw-hit slabs: one per scan wave
    int expand_blocks = 0;                        // resident k_seed_expand1 blocks
    int pin_blocks[kCls] = {0, 0};                // resident k_seed_band_pin blocks per class
    Buf vseed;                                    // verified seeds (device rounds)
    std::vector<int32_t> ucert;                   // per adapter: the candidate windows' certificate bound
    int64_t vcap = 0;
    int shrink = 0;                               // tests: the next seeding runs with 1 raw-hit slab entry (1)
                                                  // and / or 1 inside task per class (2), see shrink_next()
    bool serial = false;                          // the next seeding's band launches all on the caller's stream
    hipEvent_t *pev = nullptr;                    // profile (profile_events): 4 marks recorded on the caller's stream
    bool bstats_on = false;                       // profile (profile_band_stats): the pinned bands count their work
    Buf bstats;                                   //   into 2 classes x (lane-rows issued, active, tasks, passes)
    VerOut ver{nullptr, nullptr, nullptr, 0};     // the band launches' record target (list nullptr: off)
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
    if (!(threshold > 0.0) || sc.go >= 0 || sc.ge >= 0 || n_adp >= (1 << 19)) return 0;
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
        // e + 1 disjoint pieces covering the adapter, lengths L / (e + 1) or one more (the longer
        // first): any cut works for the seed argument, and an even one gives the longest probes
        // (a random position matches a K-probe with probability 4^-K; r02 cut L / (e + 1) bases
        // per piece and left the remainder out, so 27 bp at e = 3 had four 6-mers instead of 7, 7,
        // 7 and a 6-mer)
        const int plen = L / (e + 1), extra = L % (e + 1);
        if (std::min(kMaxK, plen) < kMinK) return 0;
        es[a] = e;
        thr[a] = T;
        e_lo = std::min(e_lo, e);
        e_hi = std::max(e_hi, e);
        filt += kFilterCell * fb_rows[a];
        for (int p = 0, o = 0; p <= e; o += plen + (p < extra ? 1 : 0), ++p) {
            const int K = std::min(kMaxK, plen + (p < extra ? 1 : 0));
            auto &lk = lists[K - kMinK];
            if (lk.empty()) lk.resize((size_t)1 << (2 * K));
            uint32_t code = 0;
            for (int t = 0; t < K; ++t) code = (code << 2) | hcodes[hoff[a] + o + t];
            lk[code].push_back((a << 12) | ((K - kMinK) << 9) | o);   // the class bit (8) is set below
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
    // The candidate windows' certificate (engine k_certify): a window best above U[a] is the whole
    // read's. Every alignment scoring above U[a] has an exact piece and at most E gap columns, so its
    // band task (E = its class's half-width) bounds it and is verified, and its end lies in that
    // task's window. Relative to the ideal L * match, an alignment with no exact piece loses in every
    // piece at least lam = min(match - mismatch, match + min|gap| (a deletion per touched piece),
    // |gap_open| (an insertion run inside it)), except that the two end pieces may instead hang off a
    // read end (match per hanging base); more than E gap columns cost at least min(|go| + E |ge|,
    // (E + 1) |go|). Schemes where a mismatch scores at least a match certify nothing.
    s->ucert.assign((size_t)n_adp, INT32_MAX);
    for (int32_t a = 0; a < n_adp; ++a) {
        if (es[a] < 0 || sc.mi >= sc.ma) continue;
        const long long L = hlen[a], ma = sc.ma, E = s->band[cls[a]], np = es[a] + 1, plen = L / np;
        const long long lam = std::min<long long>({ma - sc.mi, ma + std::min(-sc.go, -sc.ge), -sc.go});
        const long long loss = np >= 2 ? (np - 2) * std::min(lam, ma * plen) + 2 * std::min(lam, ma) : std::min(lam, ma);
        const long long gaps = std::min<long long>(-sc.go + E * -(long long)sc.ge, (E + 1) * -(long long)sc.go);
        const long long u = std::max<long long>({ma * L - loss, ma * L - gaps, (long long)thr[a] - 1});
        s->ucert[a] = (int32_t)std::min<long long>(u, INT32_MAX);
    }
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
                const int a = x >> 12;
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
    A.bits_dw = (int32_t)img.size();                // the scan copies only the bitmaps
    A.rank_off = append16(rank);
    A.estart_off = append16(estart);
    A.ent_off = (int32_t)img.size();
    for (int32_t x : ent) img.push_back((uint32_t)x);
    // per entry the inside-band limits of its tasks (k_seed_band: d0 - E >= 1, d0 + E + L + 1 < len)
    A.ent2_off = (int32_t)img.size();
    for (int32_t x : ent) {
        const int a = x >> 12, o = x & 255, E = s->band[(x >> 8) & 1];
        img.push_back((uint32_t)(o + E + 1) | ((uint32_t)(hlen[a] - o + E + 1) << 16));
    }
    A.tab_dw = (int32_t)img.size();
    s->lds_bytes = 4 * img.size();
    if (s->lds_bytes + 4096 > (size_t)kLdsMax) return 0;
    s->cost_seed = seed;
    s->cost_filter = filt;
    std::vector<int32_t> aoff((size_t)n_adp), alen((size_t)n_adp);
    int32_t tot = 0;
    for (int32_t a = 0; a < n_adp; ++a) {
        aoff[a] = tot;
        alen[a] = std::max(hlen[a], 0);
        tot += alen[a];
    }
    s->adp_bytes = (tot + 3) & ~3;
    std::vector<uint8_t> flat((size_t)tot + 16, 0);
    for (int32_t a = 0; a < n_adp; ++a) std::copy(hcodes + hoff[a], hcodes + hoff[a] + alen[a], flat.begin() + aoff[a]);
    if (int rc = s->tabs.ensure(4 * img.size())) return rc;
    if (int rc = s->adp.ensure(flat.size())) return rc;
    if (int rc = s->adp_off.ensure(4 * aoff.size())) return rc;
    if (int rc = s->adp_len.ensure(4 * alen.size())) return rc;
    if (int rc = s->cnt.ensure(4 * kCntAll)) return rc;
    if (int rc = s->thr.ensure(4 * thr.size())) return rc;
    // the pinned band: adapters and their (offset, meta) in LDS, meta = L | T << 12 (a task carries its K)
    {
        std::vector<int32_t> meta((size_t)n_adp, 0);
        bool fits = s->adp_bytes <= kAdpLds && (size_t)n_adp * 8 <= (size_t)kAdpLds;
        for (int32_t a = 0; a < n_adp && fits; ++a)
            if (es[a] >= 0) {
                if (thr[a] >= (1 << 19)) fits = false;
                meta[a] = alen[a] | (thr[a] << 12);
            }
        const bool on = fits;
        s->n_adp = n_adp;
        for (int c = 0; c < kCls; ++c) {
            // the slot holds the band's read range: L + 2E bytes from a 16-byte boundary, one more
            int lmax = 0;
            for (int32_t a = 0; a < n_adp; ++a)
                if (es[a] >= 0 && cls[a] == c) lmax = std::max(lmax, alen[a]);
            const int need = lmax + 2 * s->band[c] + 17;
            s->pin_nc4[c] = 0;
            if (on && s->band[c] <= kPinMaxE)
                for (int nc4 : {4, 6, 8})
                    if (16 * nc4 >= need) {
                        s->pin_nc4[c] = nc4;
                        break;
                    }
            A.pin_cls[c] = s->pin_nc4[c] ? 1 : 0;
            s->pin_blocks[c] = 0;
        }
        if (int rc = s->adp_meta.ensure(4 * meta.size())) return rc;
        SD_TRY(hipMemcpy(s->adp_meta.p, meta.data(), 4 * meta.size(), hipMemcpyHostToDevice));
    }
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

// One band class: its inside tasks (the pinned band when the plan allows, else band_best) and its
// edge tasks (band_best with the read-end checks). n_in / n_edge: the host's task counts, or -1
// when they live only on the device (the launches then stride over the device counts).
template <int E, int NC4>
int launch_pin(State *s, int c, const int4 *task, const uint8_t *codes, const pcabi::Scoring &sc, int64_t n,
               int64_t n_in, hipStream_t st) {
    const size_t lds = 16 * (((size_t)s->adp_bytes / 4 + 2 * (size_t)s->n_adp + 3) / 4) + 16 * 256 * (size_t)NC4;
    if (!s->pin_blocks[c]) {
        int dev = 0, cus = 0, per_cu = 0;
        SD_TRY(hipGetDevice(&dev));
        SD_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        SD_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_seed_band_pin<E, NC4, false>, 256, lds));
        s->pin_blocks[c] = std::max(1, cus * std::max(1, per_cu));
    }
    const int64_t blocks = n_in >= 0 ? std::max<int64_t>(1, std::min<int64_t>((n_in + 255) / 256, s->pin_blocks[c]))
                                     : s->pin_blocks[c];
    if (s->bstats_on && blocks <= kStatBlocks)       // a profiled round (pcabi_scan_profile)
        hipLaunchKernelGGL((k_seed_band_pin<E, NC4, true>), dim3((unsigned)blocks), dim3(256), lds, st, task,
                           (const int32_t *)s->cnt.p + c, s->cap, codes, (const uint8_t *)s->adp.p, s->adp_bytes / 4,
                           (const int32_t *)s->adp_off.p, (const int32_t *)s->adp_meta.p, s->n_adp, sc,
                           (int32_t *)s->bound.p, n, s->ver,
                           (unsigned long long *)s->bstats.p + (size_t)c * 4 * 4 * kStatBlocks);
    else
        hipLaunchKernelGGL((k_seed_band_pin<E, NC4, false>), dim3((unsigned)blocks), dim3(256), lds, st, task,
                           (const int32_t *)s->cnt.p + c, s->cap, codes, (const uint8_t *)s->adp.p, s->adp_bytes / 4,
                           (const int32_t *)s->adp_off.p, (const int32_t *)s->adp_meta.p, s->n_adp, sc,
                           (int32_t *)s->bound.p, n, s->ver, nullptr);
    return 0;
}

template <int E>
int launch_pin_e(State *s, int c, const int4 *task, const uint8_t *codes, const pcabi::Scoring &sc, int64_t n,
                 int64_t n_in, hipStream_t st) {
    switch (s->pin_nc4[c]) {
    case 4: return launch_pin<E, 4>(s, c, task, codes, sc, n, n_in, st);
    case 6: return launch_pin<E, 6>(s, c, task, codes, sc, n, n_in, st);
    default: return launch_pin<E, 8>(s, c, task, codes, sc, n, n_in, st);
    }
}

// One band class: its inside tasks (the pinned band when the plan chose it, else band_best) and
// its edge tasks (band_best with the read-end checks). n_in / n_edge: the host's task counts, or -1
// when they live only on the device (the launches then stride over the device counts).
int launch_band(State *s, int E, int c, const uint8_t *codes, const int64_t *v_off, const int32_t *v_len,
                const pcabi::Scoring &sc, int64_t n, int64_t n_in, int64_t n_edge, hipStream_t st, hipStream_t st_edge) {
    const int4 *task = (const int4 *)s->task.p + c * (s->cap + s->ecap);
    const int32_t *cnt = (const int32_t *)s->cnt.p;
    const uint8_t *adp = (const uint8_t *)s->adp.p;
    const int32_t *aoff = (const int32_t *)s->adp_off.p, *alen = (const int32_t *)s->adp_len.p;
    int32_t *bound = (int32_t *)s->bound.p;
    const int32_t lds = s->adp_bytes <= kAdpLds ? s->adp_bytes : 0;
    auto grid_of = [](int64_t cnt_host, int64_t dflt) {
        return (unsigned)(cnt_host >= 0 ? std::max<int64_t>(1, std::min<int64_t>((cnt_host + 255) / 256, dflt)) : dflt);
    };
    if (n_in != 0 && s->pin_nc4[c]) {
        int rc = 0;
        switch (E) {
        case 1: rc = launch_pin_e<1>(s, c, task, codes, sc, n, n_in, st); break;
        case 2: rc = launch_pin_e<2>(s, c, task, codes, sc, n, n_in, st); break;
        case 3: rc = launch_pin_e<3>(s, c, task, codes, sc, n, n_in, st); break;
        case 4: rc = launch_pin_e<4>(s, c, task, codes, sc, n, n_in, st); break;
        case 5: rc = launch_pin_e<5>(s, c, task, codes, sc, n, n_in, st); break;
        case 6: rc = launch_pin_e<6>(s, c, task, codes, sc, n, n_in, st); break;
        case 7: rc = launch_pin_e<7>(s, c, task, codes, sc, n, n_in, st); break;
        default: rc = launch_pin_e<kPinMaxE>(s, c, task, codes, sc, n, n_in, st); break;
        }
        if (rc) return rc;
        n_in = 0;
    }
    switch (E) {
#define C(X)                                                                                                    \
    case X:                                                                                                     \
        if (n_in != 0)                                                                                          \
            hipLaunchKernelGGL(k_seed_band<X>, dim3(grid_of(n_in, kBandGrid)), dim3(256), (size_t)lds, st, task,  \
                               cnt + c, s->cap, codes, v_off, v_len, adp, lds, aoff, alen, sc,                  \
                               (const int32_t *)s->thr.p, bound, n, s->ver);                                    \
        if (n_edge != 0)                                                                                        \
            hipLaunchKernelGGL(k_seed_band<X>, dim3(grid_of(n_edge, 512)), dim3(256), (size_t)lds, st_edge,      \
                               task + s->cap, cnt + kCls + c, s->ecap, codes, v_off, v_len, adp, lds, aoff,     \
                               alen, sc, (const int32_t *)s->thr.p, bound, n, s->ver);                          \
        break;
        C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13) C(14) C(15)
#undef C
    }
    SD_TRY(hipGetLastError());
    return 0;
}

// Both band classes side by side (atomicMax into one bound array). c: host task counts (kCnt, as
// the counters) or nullptr (device counts only).
int launch_bands(State *s, const uint8_t *codes, const int64_t *v_off, const int32_t *v_len, const pcabi::Scoring &sc,
                 int64_t n, const int32_t *c, hipStream_t st) {
    auto in_of = [&](int k) { return c ? (int64_t)std::min<int64_t>(c[k], s->cap) : (int64_t)-1; };
    auto edge_of = [&](int k) { return c ? (int64_t)std::min<int64_t>(c[kCls + k], s->ecap) : (int64_t)-1; };
    if (!s->side) {
        SD_TRY(hipStreamCreateWithFlags(&s->side, hipStreamNonBlocking));
        SD_TRY(hipStreamCreateWithFlags(&s->side2, hipStreamNonBlocking));
        SD_TRY(hipEventCreateWithFlags(&s->fork, hipEventDisableTiming));
        SD_TRY(hipEventCreateWithFlags(&s->join, hipEventDisableTiming));
        SD_TRY(hipEventCreateWithFlags(&s->join2, hipEventDisableTiming));
    }
    if (s->serial) {
        // a small round (serial_next): the fork / join events cost more than the side streams gain
        s->serial = false;
        for (int k = 0; k < kCls; ++k)
            if (int rc = launch_band(s, s->band[k], k, codes, v_off, v_len, sc, n, in_of(k), edge_of(k), st, st)) return rc;
        return 0;
    }
    // class 0's inside tasks on `st`, class 1's on a side stream, the (few, latency-bound) edge tasks
    // of both on a second side stream: the three run side by side (atomicMax into one bound array)
    SD_TRY(hipEventRecord(s->fork, st));
    SD_TRY(hipStreamWaitEvent(s->side, s->fork, 0));
    SD_TRY(hipStreamWaitEvent(s->side2, s->fork, 0));
    // (submission order: the inside launches first -- streams may share a hardware queue, and the
    // edge launches are the ones that can wait)
    if (int rc = launch_band(s, s->band[0], 0, codes, v_off, v_len, sc, n, in_of(0), 0, st, s->side2)) return rc;
    if (int rc = launch_band(s, s->band[1], 1, codes, v_off, v_len, sc, n, in_of(1), 0, s->side, s->side2)) return rc;
    for (int k = 0; k < kCls; ++k)
        if (int rc = launch_band(s, s->band[k], k, codes, v_off, v_len, sc, n, 0, edge_of(k), s->side2, s->side2))
            return rc;
    SD_TRY(hipEventRecord(s->join, s->side));
    SD_TRY(hipEventRecord(s->join2, s->side2));
    SD_TRY(hipStreamWaitEvent(st, s->join, 0));
    SD_TRY(hipStreamWaitEvent(st, s->join2, 0));
    return 0;
}

// Queue the seeds of one round on `st`: bounds reset, scan, expand, the band classes side by side.
// n: reads (host upper bound); n_dev: their count on the device (nullptr: n). band_grid: the band
// launches' grid (0: sized from the host task counts in `tasks`).
int enqueue_seeds(State *s, const uint8_t *codes, const int64_t *v_off, const int32_t *v_len, int64_t n,
                  const int32_t *n_dev, int32_t n_adp, const pcabi::Scoring &sc, const int32_t *tasks, hipStream_t st) {
    if (s->scan_blocks == 0) {
        int dev = 0, cus = 0, per_cu = 0;
        SD_TRY(hipGetDevice(&dev));
        SD_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        SD_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_seed_scan<kScanThreads>, kScanThreads, 0));
        s->scan_blocks = std::max(1, cus * std::max(1, per_cu));
        s->n_slab = s->scan_blocks * (kScanThreads / 64);   // one slab per scan wave
        per_cu = 0;
        SD_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_seed_expand1<kExpandHits>, kExpandThreads,
                                                            s->lds_bytes));
        s->expand_blocks = std::min(s->n_slab, std::max(1, cus * std::max(1, per_cu)));
    }
    const int grid = s->scan_blocks;
    if (s->raw_cap == 0 || s->cap == 0) {
        // first sizing; PCABI_MIDDLE_INIT_CAPS="raw,task[,slots]" (tests: small buffers that overflow
        // and grow) overrides the defaults, 0 keeps one
        int64_t raw = 0, task = 0;
        if (const char *e = std::getenv("PCABI_MIDDLE_INIT_CAPS"))
            if (std::sscanf(e, "%lld,%lld", (long long *)&raw, (long long *)&task) < 1) raw = task = 0;
        // (4096 raw hits per r03 scan block: the same total for the byte-map scan's wave slabs)
        if (s->raw_cap == 0) s->raw_cap = raw > 0 ? std::max<int64_t>(raw, s->n_slab) : (int64_t)std::max(grid * 4096, 1536 * 4096);
        if (s->cap == 0) s->cap = task > 0 ? task : 1 << 22;
    }
    // tests (shrink_next): this seeding's buffers shrunk to nothing, restored when it is queued
    const int64_t cap_keep = s->cap;
    const int shrink = s->shrink;
    s->shrink = 0;
    if (shrink & 2) s->cap = 1;
    s->ecap = std::max<int64_t>(s->cap / 4, 1 << 16);
    struct Restore {
        State *s;
        int64_t cap;
        ~Restore() {
            s->cap = cap;
            s->ecap = std::max<int64_t>(cap / 4, 1 << 16);
        }
    } restore{s, cap_keep};
    if (int rc = s->raw.ensure(sizeof(uint4) * (size_t)s->raw_cap)) return rc;
    if (int rc = s->rawcnt.ensure(4 * (size_t)s->n_slab)) return rc;
    if (int rc = s->task.ensure(sizeof(int4) * kCls * (size_t)(s->cap + s->ecap))) return rc;
    if (int rc = s->cnt.ensure(4 * kCntAll)) return rc;
    if (int rc = s->bound.ensure(sizeof(int32_t) * (size_t)n * n_adp)) return rc;
    ScanArgs A = s->a;
    A.codes = codes;
    A.v_off = v_off;
    A.v_len = v_len;
    A.n = n;
    A.n_dev = n_dev;
    A.raw = (uint4 *)s->raw.p;
    A.n_slab = s->n_slab;
    A.slab = (shrink & 1) ? 1 : (int32_t)std::min<int64_t>(s->raw_cap / s->n_slab, INT32_MAX);
    A.raw_cnt = (int32_t *)s->rawcnt.p;
    A.cnt = (int32_t *)s->cnt.p;
    A.flags = A.cnt + kFlag;
    A.task = (int4 *)s->task.p;
    A.cap = s->cap;
    A.ecap = s->ecap;
    if (int rc = s->ccnt.ensure(8)) return rc;
    // the scan's segment space: seg_cum[r] = segments before read r, seg_cum[n_dev] = all (entries
    // past n_dev repeat the total). r04 measured one-block scans against hipcub's device scan (two
    // launches): 40 us per round against ~11-23, so hipcub's stays.
    if (int rc = s->segcum.ensure(sizeof(int64_t) * (size_t)(n + 1))) return rc;
    {
        hipcub::CountingInputIterator<int64_t> idx(0);
        hipcub::TransformInputIterator<int64_t, SegCount, hipcub::CountingInputIterator<int64_t>> segs(
            idx, SegCount{v_len, n_dev, n});
        size_t tmp = 0;
        SD_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, segs, (int64_t *)nullptr, n + 1, st));
        if (int rc = s->scantmp.ensure(tmp)) return rc;
        SD_TRY(hipcub::DeviceScan::ExclusiveSum(s->scantmp.p, tmp, segs, (int64_t *)s->segcum.p, n + 1, st));
    }
    A.seg_cum = (const int64_t *)s->segcum.p;
    hipLaunchKernelGGL(k_bound_reset, dim3(1024), dim3(256), 0, st, (int32_t *)s->bound.p, n, n_dev, n_adp, A.cnt,
                       kCntAll, (unsigned long long *)s->ccnt.p);
    if (s->pev) SD_TRY(hipEventRecord(s->pev[0], st));
    hipLaunchKernelGGL(k_seed_scan<kScanThreads>, dim3(grid), dim3(kScanThreads), 0, st, A);
    if (s->pev) SD_TRY(hipEventRecord(s->pev[1], st));
    hipLaunchKernelGGL(k_seed_expand1<kExpandHits>, dim3(s->expand_blocks), dim3(kExpandThreads), s->lds_bytes, st, A);
    if (s->pev) SD_TRY(hipEventRecord(s->pev[2], st));
    SD_TRY(hipGetLastError());
    if (tasks) return 0;                                // the caller launches the bands (host counts)
    return launch_bands(s, codes, v_off, v_len, sc, n, nullptr, st);
}

// Device -> host: the task counts and the overflow flags (synchronises `st`).
int read_counts(State *s, int32_t (&out)[kCnt], hipStream_t st) {
    SD_TRY(hipMemcpyAsync(out, s->cnt.p, sizeof(out), hipMemcpyDeviceToHost, st));
    SD_TRY(hipStreamSynchronize(st));
    return 0;
}

// Larger buffers after an overflow; false when they would pass sane limits.
bool grow(State *s, const int32_t (&c)[kCnt]) {
    g_buf_gen.fetch_add(1);           // new capacities: launch arguments of captured rounds change
    if (c[kFlag]) {
        if (s->raw_cap > (1ll << 31)) return false;
        s->raw_cap *= 2;
    }
    if (c[kFlag + 1]) {
        int64_t most = 0;
        for (int k = 0; k < kCls; ++k) most = std::max<int64_t>(most, std::max<int64_t>(c[k], 4 * (int64_t)c[kCls + k]));
        if (most > (1ll << 30)) return false;
        s->cap = std::max<int64_t>(2 * s->cap, most + most / 4);   // ecap follows (cap / 4)
        if (s->vcap) s->vcap *= 2;                   // the verified-seed list shares the flag
    }
    return true;
}

int check_plan(State *s, const uint8_t *hcodes, const int32_t *hoff, const int32_t *hlen, int32_t n_adp,
               const std::vector<int> &fb_rows, const pcabi::Scoring &sc, double threshold, hipStream_t st) {
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
        g_buf_gen.fetch_add(1);
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
    return 0;
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
    s->ver = VerOut{nullptr, nullptr, nullptr, 0};   // no verified seeds on this path
    if (int rc = check_plan(s, hcodes, hoff, hlen, n_adp, fb_rows, sc, threshold, st)) return rc;
    if (!s->ok) return 0;
    if (mode == 1 && !(s->cost_seed < 0.5 * s->cost_filter)) return 0;
    // the scan and the expansion, again with larger buffers after an overflow; then the band
    // launches sized from the task counts
    int32_t c[kCnt];
    for (int tries = 0;; ++tries) {
        int32_t none[kCls] = {0, 0};
        // scan + expand only (tasks given: the band kernels are not queued)
        if (int rc = enqueue_seeds(s, codes, v_off, v_len, n, nullptr, n_adp, sc, none, st)) return rc;
        if (int rc = read_counts(s, c, st)) return rc;
        if (!c[kFlag] && !c[kFlag + 1]) break;
        if (tries > 8 || !grow(s, c)) return fail(PCABI_E_DEVICE, "seed scan did not settle");
    }
    if (const char *dbg = std::getenv("PCABI_DEBUG"))
        if (dbg[0] == '1')
            std::fprintf(stderr, "[pcabi] seeds: %lld windows, band tasks %d + %d edge (E=%d), %d + %d edge (E=%d), "
                         "scan grid %d, pinned slots %d\n", (long long)n, c[0], c[kCls], s->band[0], c[1], c[kCls + 1],
                         s->band[1], s->scan_blocks, s->pin_nc4[0] * 10 + s->pin_nc4[1]);
    // the band classes from the counted tasks (the tasks are still in place)
    if (int rc = launch_bands(s, codes, v_off, v_len, sc, n, c, st)) return rc;
    const int64_t tot = n * (int64_t)n_adp;
    if (!cands && !dcands) {
        hipLaunchKernelGGL(k_bound16, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (const int32_t *)s->bound.p,
                           tot, s16);
        SD_TRY(hipGetLastError());
        g_runs.fetch_add(1);
        return 1;
    }
    if (s->ccap < tot) s->ccap = tot;                 // every pair fits: no overflow pass
    if (int rc = s->cands.ensure(sizeof(int64_t) * (size_t)s->ccap)) return rc;
    if (int rc = s->ccnt.ensure(8)) return rc;
    SD_TRY(hipMemsetAsync(s->ccnt.p, 0, 8, st));
    hipLaunchKernelGGL(k_cands, dim3((unsigned)std::min<int64_t>((tot + 255) / 256, kBandGrid)), dim3(256), 0, st,
                       (const int32_t *)s->bound.p, n, nullptr, n_adp, (const int32_t *)s->thr.p, (int64_t *)s->cands.p,
                       s->ccap, (unsigned long long *)s->ccnt.p, nullptr);
    SD_TRY(hipGetLastError());
    unsigned long long nc = 0;
    SD_TRY(hipMemcpyAsync(&nc, s->ccnt.p, 8, hipMemcpyDeviceToHost, st));
    SD_TRY(hipStreamSynchronize(st));
    if (dcands) {                                     // the keys stay on the device, unordered
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

// The device-resident form for the engine's queued rounds (no host synchronisation): the plan must
// be ready (bounds() ran it this call or earlier: s->ok); n_dev is the round's read count on the
// device, n its host upper bound (the bound array's row stride). Queues bounds reset, scan,
// expansion, both band classes (grid-stride over the device task counts) and k_cands; the keys
// (a << 32 | read, unordered) land in *dcands, their count in *dcount (device uint64), and
// *flags (device int32[2]) is set when a buffer overflowed (the caller reruns the round after
// grow_after_overflow()). vlist != nullptr (candidate windows): the band kernels also record the
// verified seeds (*vlist, their count *vcount on the device: int4 (read, adapter | E << 24, diagonal
// codes offset lo, hi)) and *pmap (n_adp x n, row stride n) maps a candidate pair to its index in
// *dcands.
int bounds_dev(State *s, const uint8_t *codes, const int64_t *v_off, const int32_t *v_len, int64_t n,
               const int32_t *n_dev, int32_t n_adp, const pcabi::Scoring &sc, const int64_t **dcands,
               const unsigned long long **dcount, const int32_t **flags, const int4 **vlist, const int32_t **vcount,
               const int32_t **pmap, int64_t *vcap, hipStream_t st) {
    const bool win = vlist != nullptr;
    if (!s->ok) return fail(PCABI_E_ARG, "seed plan not ready");
    s->ver = VerOut{nullptr, nullptr, nullptr, 0};
    if (win) {
        if (s->vcap == 0) s->vcap = std::max<int64_t>(1 << 16, n);
        if (int rc = s->vseed.ensure(sizeof(int4) * (size_t)s->vcap)) return rc;
        if (int rc = s->cnt.ensure(4 * kCntAll)) return rc;
        s->ver = VerOut{(int4 *)s->vseed.p, (int32_t *)s->cnt.p + kVer, (int32_t *)s->cnt.p + kFlag + 1, s->vcap};
    }
    if (int rc = enqueue_seeds(s, codes, v_off, v_len, n, n_dev, n_adp, sc, nullptr, st)) return rc;
    if (s->pev) SD_TRY(hipEventRecord(s->pev[3], st));   // the band classes joined
    const int64_t tot = n * (int64_t)n_adp;
    if (s->ccap < tot) s->ccap = tot;
    if (int rc = s->cands.ensure(sizeof(int64_t) * (size_t)s->ccap)) return rc;
    // (ccnt zeroed by k_bound_reset)
    hipLaunchKernelGGL(k_cands, dim3((unsigned)std::min<int64_t>((tot + 255) / 256, kBandGrid)), dim3(256), 0, st,
                       (const int32_t *)s->bound.p, n, n_dev, n_adp, (const int32_t *)s->thr.p, (int64_t *)s->cands.p,
                       s->ccap, (unsigned long long *)s->ccnt.p, win ? (int32_t *)s->bound.p : nullptr);
    SD_TRY(hipGetLastError());
    *dcands = (const int64_t *)s->cands.p;
    *dcount = (const unsigned long long *)s->ccnt.p;
    *flags = (const int32_t *)s->cnt.p + kFlag;
    if (win) {
        *vlist = (const int4 *)s->vseed.p;
        *vcount = (const int32_t *)s->cnt.p + kVer;
        *pmap = (const int32_t *)s->bound.p;
        *vcap = s->vcap;
    }
    s->ver = VerOut{nullptr, nullptr, nullptr, 0};
    g_runs.fetch_add(1);
    return 0;
}

// The last seeding's segment scan (kSeg positions per segment, n + 1 entries, the total last):
// the engine reads round 1's total to size its next call (candidate windows on long reads).
const int64_t *seg_cum_dev(State *s) { return (const int64_t *)s->segcum.p; }
int seg_positions() { return kSeg; }

// Tests (the engine's PCABI_MIDDLE_FAULT): the next queued seeding runs with its raw-hit slabs
// (bits & 1) and / or its inside-task regions (bits & 2) shrunk to one entry, so its kernels overflow
// for real and flag the round; the buffers keep their sizes.
void shrink_next(State *s, int bits) { s->shrink = bits & 3; }

// The next queued seeding launches its band classes one after the other on the caller's stream.
void serial_next(State *s) { s->serial = true; }

// Profiling (pcabi_scan_profile): the next seedings record ev[0] before k_seed_scan, ev[1] after it,
// ev[2] after k_seed_expand and ev[3] after the band classes (nullptr: off).
void profile_events(State *s, hipEvent_t *ev) { s->pev = ev; }

// Profiling: the pinned band classes count their work while on (k_seed_band_pin<..., true>); on
// zeroes the counters. band_stats reads them: per class lane-rows issued, active, tasks, passes.
int profile_band_stats(State *s, bool on) {
    s->bstats_on = false;
    if (!on) return 0;
    const size_t bytes = sizeof(unsigned long long) * kCls * 4 * 4 * kStatBlocks;
    if (int rc = s->bstats.ensure(bytes)) return rc;
    SD_TRY(hipMemset(s->bstats.p, 0, bytes));
    s->bstats_on = true;
    return 0;
}

// The band half-width E of class c (0 before a plan).
int band_e(State *s, int c) { return (c >= 0 && c < kCls) ? s->band[c] : 0; }

int band_stats(State *s, unsigned long long (&out)[8]) {
    std::fill(out, out + 8, 0ull);
    if (!s->bstats.p) return 0;
    std::vector<unsigned long long> w((size_t)kCls * 4 * 4 * kStatBlocks);
    SD_TRY(hipMemcpy(w.data(), s->bstats.p, 8 * w.size(), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < w.size(); ++i) out[4 * (i / (4 * 4 * kStatBlocks)) + i % 4] += w[i];
    return 0;
}

// Profiling: the last seeding's raw hits (slabs, clamped), inside and edge band tasks (synchronises `st`).
int profile_counts(State *s, int64_t (&out)[3], hipStream_t st) {
    std::vector<int32_t> raw((size_t)std::max(1, s->n_slab));
    int32_t c[kCnt] = {};
    SD_TRY(hipMemcpyAsync(raw.data(), s->rawcnt.p, 4 * raw.size(), hipMemcpyDeviceToHost, st));
    SD_TRY(hipMemcpyAsync(c, s->cnt.p, sizeof(c), hipMemcpyDeviceToHost, st));
    SD_TRY(hipStreamSynchronize(st));
    out[0] = 0;
    for (int32_t x : raw) out[0] += x;
    out[1] = (int64_t)std::min<int64_t>(c[0], s->cap) + std::min<int64_t>(c[1], s->cap);
    out[2] = (int64_t)std::min<int64_t>(c[kCls], s->ecap) + std::min<int64_t>(c[kCls + 1], s->ecap);
    return 0;
}

// The candidate windows' certificate bounds per adapter (plan(): INT32_MAX = never certified).
void cert_bounds(State *s, std::vector<int32_t> &U) { U = s->ucert; }

// After a device-resident run reported an overflow (flags from bounds_dev, read by the caller):
// larger buffers for the rerun. Returns false past the limits.
bool grow_after_overflow(State *s, int raw_overflow, int task_overflow) {
    int32_t c[kCnt] = {};
    c[0] = (int32_t)std::min<int64_t>(4 * s->cap, INT32_MAX);
    c[kFlag] = raw_overflow;
    c[kFlag + 1] = task_overflow;
    return grow(s, c);
}

// Debugging (PCABI_DEBUG=1): the last queued seeding's band task counts per class (inside, edge)
// and candidate count (synchronises `st`).
int debug_counts(State *s, int64_t (&out)[5], hipStream_t st) {
    int32_t c[kCnt] = {};
    unsigned long long nc = 0;
    SD_TRY(hipMemcpyAsync(c, s->cnt.p, sizeof(c), hipMemcpyDeviceToHost, st));
    SD_TRY(hipMemcpyAsync(&nc, s->ccnt.p, 8, hipMemcpyDeviceToHost, st));
    SD_TRY(hipStreamSynchronize(st));
    out[0] = c[0];
    out[1] = c[kCls];
    out[2] = c[1];
    out[3] = c[kCls + 1];
    out[4] = (int64_t)nc;
    return 0;
}

// the plan for these adapters, without running anything: true when seeds apply (mode as bounds()).
int plan_ready(State *s, const uint8_t *hcodes, const int32_t *hoff, const int32_t *hlen, int32_t n_adp,
               const std::vector<int> &fb_rows, const pcabi::Scoring &sc, double threshold, int mode, hipStream_t st) {
    if (mode <= 0) return 0;
    if (int rc = check_plan(s, hcodes, hoff, hlen, n_adp, fb_rows, sc, threshold, st)) return rc;
    if (!s->ok) return 0;
    if (mode == 1 && !(s->cost_seed < 0.5 * s->cost_filter)) return 0;
    return 1;
}

}  // namespace pcabi_seed

extern "C" int64_t pcabi_middle_seed_runs(void) { return pcabi_seed::g_runs.load(); }

