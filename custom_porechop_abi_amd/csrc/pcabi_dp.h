// pcabi_dp.h -- per-lane semi-global Gotoh DP with forward traceback-attribute propagation.
//
// This is the arithmetic core of the MI355X adapter-alignment engine. One invocation aligns ONE
// read window (horizontal sequence, columns j = 1..n) against ONE adapter (vertical sequence,
// rows i = 1..L) and produces exactly the integers the reference's ScoredAlignment derives from
// its gapped rows (porechop_abi/src/alignment.cpp:6-110), WITHOUT a trace matrix and WITHOUT a
// traceback walk:
//
//   * The reference runs SeqAn globalAlignment with free end gaps on all four sides
//     (porechop_abi/src/adapter_align.cpp:26-27), Gotoh when gap_open != gap_extend and linear
//     otherwise (S/align/global_alignment_unbanded.h:213-221), then walks the trace matrix back
//     from the first maximum of the last row / last column (S/align/dp_scout.h:175,
//     S/align/dp_traceback_impl.h:379-548).
//   * The walk's predecessor of every (cell, state) is a LOCAL function of that cell's trace bits
//     (D / V-ext / V-open / H-ext / H-open / MAX_FROM_V|H, tie rules of S/align/dp_formula.h:153-163).
//     So every state can carry forward the few attributes of "the path the traceback would take
//     from here": its start cell (i0, j0), its match count m and its diagonal count nD. They are
//     packed in one 32-bit word and selected with the same predicates that select the scores.
//   * The end-of-path details (trailing gap run length and whether a diagonal precedes it) only
//     matter in the last row / last column and are kept as O(1) running values there.
//   * ScoredAlignment's st/en/a0/a1/identities reduce to closed forms of those values
//     (finish(), documented in DESIGN.md §3 and fuzzed against the oracle in tests/).
//
// The code is plain C++ usable on the host (tests fuzz it against oracle/) and on the device,
// where one wave64 lane owns one (window, adapter) pair and the adapter is wave-uniform
// (SGPR-resident), so every instruction is a full-width VALU op with no cross-lane traffic.
//
// (S/ = porechop_abi/include/seqan/ of the reference.)
#pragma once

// Scheduling fence every N rows in the fast cores (0 = none); see DESIGN.md §5.
#ifndef PCABI_ROW_FENCE
#define PCABI_ROW_FENCE 1
#endif
// Packed core: substitution-key quads fetched this many quads ahead (0 = one read per slot).
// Packed-core substitution keys (LanePacked<.., PD>): PD = 0, one LDS read per row, issued a row
// ahead -- the end-window buckets (k_align<24>: 3.58 vs 4.07 ms per launch against quads, 74
// instead of 88 VGPRs, the waves interleave at every row's wait); PD > 0, quads
// (4 slots) fetched at the column top, PD quads ahead -- the long two-pass buckets, where the
// per-row reads measured 1.5x slower. PCABI_TAB_PD overrides the end-window default.
#ifndef PCABI_TAB_PD
#define PCABI_TAB_PD 0
#endif
#ifndef PCABI_TAB_PD_LONG
#define PCABI_TAB_PD_LONG 1
#endif

#include <stdint.h>
#include <algorithm>

#ifdef __HIPCC__
#define PCABI_HD __host__ __device__ __forceinline__
#else
#define PCABI_HD inline
#endif

namespace pcabi {

// SeqAn's DPCellDefaultInfinity is INT_MIN/2 (S/align/dp_cell.h:144-145). Any value far below
// every reachable score behaves identically under max/compare: a NEG-derived candidate never
// wins and never ties (|scores| <= 2^20 for all supported sizes).
constexpr int NEG = -(1 << 28);

// Attribute word: [ (c + CBIAS) mod 2^16 : 16 ][ nD : 8 ][ m : 8 ]
//   c  = j0 - i0  (path start cell; at least one of i0, j0 is zero)
//   m  = matching diagonal columns on the path, nD = diagonal columns on the path
// The c field WRAPS (uint32 arithmetic, top field): every live path spans fewer than
// span_bound() < 2^15 columns (gap costs < 0 bound its horizontal moves), so c is recovered
// exactly from the end column in finish(). Reads of any length are therefore supported.
constexpr int ATTR_B = 8;
constexpr uint32_t ATTR_MASK = (1u << ATTR_B) - 1u;
constexpr int ATTR_CSH = 2 * ATTR_B;
constexpr int ATTR_CBIAS = 255;            // c >= -L >= -255
constexpr int MAX_ADAPTER_LEN = 255;       // m, nD <= L fit 8 bits
constexpr int MAX_WINDOW_LEN = 1 << 30;
constexpr uint32_t INC_D = 1u << ATTR_B;                 // mismatching diagonal: nD + 1
constexpr uint32_t INC_M = INC_D + 1u;                   // matching diagonal: nD + 1, m + 1

PCABI_HD uint32_t attr_start(int c) { return (uint32_t)(c + ATTR_CBIAS) << ATTR_CSH; }

// Upper bound on the columns spanned by any path the DP keeps (S-, H- or V-state). A path
// ending at row i scores >= i*mi (the all-diagonal path is always available) and <= i*ma minus
// the cost of its horizontal moves, each costing >= g = min(|go|, |ge|); a trailing H run is
// bounded the same way. Returns -1 if gap costs are not both negative (no bound).
PCABI_HD int span_bound(int L, int ma, int mi, int go, int ge) {
    if (go >= 0 || ge >= 0) return -1;
    const int g = (-go < -ge) ? -go : -ge;
    const int d = (ma > mi ? ma - mi : mi - ma) + 1;   // mismatch may outscore match
    const long long t = ((long long)L * d + g - 1) / g + 2;
    const long long b = (long long)L + 2 * t + 4;
    return b > (1 << 30) ? (1 << 30) : (int)b;
}

// last-column types of a path
enum : int { LT_NONE = 0, LT_D = 1, LT_V = 2, LT_H = 3 };

struct Scoring {
    int ma, mi, go, ge;  // match, mismatch, gap open, gap extend (Python order)
};

// The most a diagonal column can add: match, or mismatch when a scheme scores it higher (the
// reference accepts any --scoring_scheme; every range and span bound below uses this).
PCABI_HD int best_sub(const Scoring &s) { return s.ma > s.mi ? s.ma : s.mi; }

// What the scout keeps for the current best end cell.
struct Best {
    int score;
    int bi, bj;      // end cell (row in adapter coordinates 0..L, column 0..n)
    uint32_t attr;   // attributes of the path of the corrected end state
    int ltype;       // last path column type (LT_*)
    int trail;       // length of the trailing gap run (only meaningful when it is used)
    int precd;       // 1 if the column before the trailing run is diagonal
};

// Final integers, same meaning as ScoredAlignment + the two identity fractions m/l1, m/l2.
struct Result {
    int rs, re, as, ae, score, m, l1, l2;
    int diag_en;   // the aligned region's last column is a diagonal (both rows hold a base)
};

// Closed forms of ScoredAlignment (porechop_abi/src/alignment.cpp:27-109) in terms of the path.
// Derivation in DESIGN.md §3. bi/bj: end cell, L/n: sequence lengths.
// finish_path: the same from the path's start diagonal c, match count m and diagonal count nd
// (b.attr unused); finish: from the packed attribute word.
PCABI_HD Result finish_path(const Best &b, int c, int m, int nd, int L, int n) {
    Result r;
    const int i0 = c < 0 ? -c : 0;
    const int j0 = c > 0 ? c : 0;
    const int h = i0 + j0;                             // head length == first path column
    const int K = (b.bi - i0) + (b.bj - j0) - nd;      // path columns
    const bool tailA = b.bi < L;                       // adapter tail after the path
    const bool tailR = b.bj < n;                       // read tail after the path
    const int trailV = b.ltype == LT_V ? b.trail : 0;
    const int trailH = b.ltype == LT_H ? b.trail : 0;
    const int lastD = b.ltype == LT_D ? 1 : 0;
    // A run that spans the whole path has no column before it (the fast kernel's pass-through
    // padding rows would otherwise report a virtual diagonal there).
    const int precd = (b.trail < K) ? b.precd : 0;
    const int kR = K - 1 - trailV;                     // last path column holding a read base
    const int kA = K - 1 - trailH;                     // last path column holding an adapter base
    bool readSide;
    if (tailA) readSide = true;
    else if (tailR) readSide = false;
    else readSide = (kR <= kA);
    int ek;
    if (readSide) {
        ek = kR;
        r.re = b.bj - 1;
        r.ae = b.bi - trailV - (trailV > 0 ? precd : lastD);
    } else {
        ek = kA;
        r.ae = b.bi - 1;
        r.re = b.bj - trailH - (trailH > 0 ? precd : lastD);
    }
    r.rs = j0;
    r.as = i0;
    r.score = b.score;
    r.m = m;
    r.l1 = ek + 1;
    const int a0 = j0 > 0 ? h : 0;
    const int a1 = tailA ? (h + K + (L - b.bi) - 1) : (h + kA);
    r.l2 = a1 - a0 + 1;
    r.diag_en = readSide ? (trailV > 0 ? precd : lastD) : (trailH > 0 ? precd : lastD);
    return r;
}

PCABI_HD Result finish(const Best &b, int L, int n) {
    // c lies in [bj - span, bj] with span < 2^15: undo the mod-2^16 wrap
    const int u = (int)(b.attr >> ATTR_CSH) - ATTR_CBIAS;
    const int c = b.bj - ((b.bj - u) & 0xFFFF);
    const int m = (int)(b.attr & ATTR_MASK);
    const int nd = (int)((b.attr >> ATTR_B) & ATTR_MASK);
    return finish_path(b, c, m, nd, L, n);
}

// check_compatibility (porechop_abi/ab_initio_src/compatibility.cpp:124-170) from the aligned
// region of the longer sequence (row 0, n bases) against the shorter: the reference counts
// mismatching columns on [st, en) only, so mapped - distance = 1 + m - [column en matches];
// identity = that * 100 / mapped in INTEGER arithmetic, linked at >= 87.5; "included" when the
// region starts or ends more than OVERLAP_LIMIT = 3 bases inside row 0.
// en_match: column en is a diagonal with equal bases. mapped <= 0 (no overlap: the reference
// divides by zero there) -> 0.
PCABI_HD int compat_flag(const Result &r, int n, int en_match) {
    if (r.rs < 0 || r.l1 <= 0) return 0;
    const int identity = (1 + r.m - en_match) * 100 / r.l1;
    if (identity < 88) return 0;
    return (r.rs > 3 || (n - r.re) > 3) ? 2 : 1;
}

// The reference prints 100.0*m/l with "%f" (std::to_string, porechop_abi/src/alignment.cpp:118-119)
// and Python parses it back (porechop_abi/nanopore_read.py:497-498). pid6 returns the same
// double: d = (100.0*m)/l (IEEE, as in alignment.cpp:82,89), round d*1e6 to an integer with
// round-half-even on its EXACT value (fma residual), then q/1e6 correctly rounded -- which is
// what both printf and Python's float() do. l == 0 -> NaN (the reference's "-nan").
PCABI_HD double pid6(int m, int l) {
    if (l == 0) return __builtin_nan("");
    const double d = (100.0 * (double)m) / (double)l;
    const double p = d * 1e6;
    const double e = __builtin_fma(d, 1e6, -p);   // d*1e6 == p + e exactly
    double k = __builtin_rint(p);                 // half-even on p
    const double f = p - k;                       // exact
    if (f == 0.5 && e > 0.0) k += 1.0;
    else if (f == -0.5 && e < 0.0) k -= 1.0;
    return k / 1e6;
}

// Trailing-run bookkeeping when a gap state opens from an S-state whose last column type is
// `slt` (and whose own trailing run of the same gap kind is (t, p) when slt == same kind).
PCABI_HD void open_run(int slt, int same_kind, int t_prev, int p_prev, int &t, int &p) {
    if (slt == same_kind) { t = t_prev + 1; p = p_prev; }
    else { t = 1; p = (slt == LT_D) ? 1 : 0; }
}

// ------------------------------------------------------------------------------------------
// align_lane<RPL, AFFINE>: rows live in registers (RPL compile-time slots). The adapter occupies
// slots off+1..RPL (off = RPL - L, "top padding"): slots <= off are skipped by a branch that is
// uniform across a wave (all lanes share the adapter), and the running "up" values entering
// slot off+1 are exactly the free-end-gap boundary row, so padding costs nothing.
//
//   rd(j)  : read code at column j (1-based), 0..4
//   adp[s] : adapter code of slot s (1-based; slots off+1..RPL), 0..4
// ------------------------------------------------------------------------------------------
// CHUNK: as align_lane_packed's (sf::chunk_plan): the end cell only in owned columns
// [own_lo, own_hi), own_hi < 0 = the read's last chunk.
template <int RPL, bool AFFINE, bool CHUNK = false, typename ReadFn, typename AdpFn>
PCABI_HD Result align_lane_generic(ReadFn rd, int n, AdpFn adp, int L, const Scoring sc, int own_lo = 1,
                                   int own_hi = -1) {
    const int off = RPL - L;
    const bool fin = !CHUNK || own_hi < 0;
    const int hi = own_hi < 0 ? n + 1 : own_hi;
    int S[RPL + 1], H[RPL + 1];
    uint32_t SA[RPL + 1], HA[RPL + 1];
#pragma unroll
    for (int s = 1; s <= RPL; ++s) {
        S[s] = 0;
        H[s] = NEG;
        SA[s] = attr_start(-(s - off));
        HA[s] = 0;
    }

    Best best;
    best.score = 0;          // first scouted cell: (L, 0), S = 0 (S/align/dp_meta_info.h:204-216)
    best.bi = L;
    best.bj = 0;
    best.attr = attr_start(-L);
    best.ltype = LT_NONE;
    best.trail = 0;
    best.precd = 0;

    // last-row running state: S-state last type of (L, j-1) and H-state trailing run (t, p)
    int slt_last = LT_NONE, ht_last = 0, hp_last = 0;

    for (int j = 1; j <= n; ++j) {
        const int r = rd(j);
        const bool lastcol = (j == n) && fin;   // an inner chunk's last column is an inner read column
        int sup = 0, vup = NEG, sdg = 0;
        uint32_t saup = attr_start(j), vaup = 0, sadg = attr_start(j - 1);
        // last-column running state: S-state last type of (i-1, n), V-state run (t, p)
        int slt_up = LT_NONE, vt_up = 0, vp_up = 0;
        // last-row cell products, kept for the row-L scout / running state
        int lv = NEG, lh = NEG, ls = 0, lt_type = LT_NONE;
        bool l_hext = false;
        uint32_t lva = 0, lha = 0, lsa = 0;
#pragma unroll
        for (int s = 1; s <= RPL; ++s) {
            if (s > off) {
                const bool match = (r == adp(s));
                const int diag = sdg + (match ? sc.ma : sc.mi);
                const uint32_t da = sadg + (match ? INC_M : INC_D);
                int hn, vn, g, sn;
                uint32_t han, van, ga, san;
                bool hext, vext, fromv, isd;
                if (AFFINE) {
                    const int hx = H[s] + sc.ge, ho = S[s] + sc.go;
                    hext = !(hx < ho);
                    hn = hext ? hx : ho;
                    han = hext ? HA[s] : SA[s];
                    const int vx = vup + sc.ge, vo = sup + sc.go;
                    vext = !(vx < vo);
                    vn = vext ? vx : vo;
                    van = vext ? vaup : saup;
                    fromv = !(vn < hn);
                    g = fromv ? vn : hn;
                    ga = fromv ? van : han;
                } else {
                    hext = false;
                    vext = false;
                    const int vv = sup + sc.ge, hh = S[s] + sc.ge;
                    fromv = !(vv < hh);
                    g = fromv ? vv : hh;
                    ga = fromv ? saup : SA[s];
                    hn = NEG; vn = NEG; han = 0; van = 0;
                }
                isd = !(diag < g);
                sn = isd ? diag : g;
                san = isd ? da : ga;
                const int slt = isd ? LT_D : (fromv ? LT_V : LT_H);

                if (lastcol) {
                    // V run of this cell's V-state (affine) / S-state-from-V (linear)
                    int vt, vp;
                    if (AFFINE) {
                        if (vext) { vt = vt_up + 1; vp = vp_up; }
                        else open_run(slt_up, LT_V, vt_up, vp_up, vt, vp);
                    } else {
                        open_run(slt_up, LT_V, vt_up, vp_up, vt, vp);
                    }
                    if (s < RPL && sn > best.score) {   // last column, rows 1..L-1
                        best.score = sn; best.bi = s - off; best.bj = n;
                        if (AFFINE) {
                            if (vn == sn)      { best.attr = van; best.ltype = LT_V; best.trail = vt; best.precd = vp; }
                            else if (hn == sn) { best.attr = han; best.ltype = LT_H; best.trail = 0; best.precd = 0; }
                            else               { best.attr = san; best.ltype = LT_D; best.trail = 0; best.precd = 0; }
                        } else {
                            best.attr = san; best.ltype = slt;
                            best.trail = (slt == LT_V) ? vt : 0; best.precd = (slt == LT_V) ? vp : 0;
                        }
                    }
                    // running V-run state for the next row: V-state (affine) or S-state (linear)
                    if (AFFINE) {
                        // S-state of this cell, as seen by an opening V below it:
                        //   slt == LT_V: S path == V path -> carries (vt, vp)
                        vt_up = vt; vp_up = vp;
                    } else {
                        if (slt == LT_V) { vt_up = vt; vp_up = vp; }
                        else { vt_up = 0; vp_up = 0; }
                    }
                    slt_up = slt;
                }
                if (s == RPL) {
                    lv = vn; lh = hn; ls = sn; lva = van; lha = han; lsa = san;
                    lt_type = slt; l_hext = hext;
                }
                sdg = S[s];
                sadg = SA[s];
                S[s] = sn;
                H[s] = hn;
                SA[s] = san;
                HA[s] = han;
                sup = sn;
                vup = vn;
                saup = san;
                vaup = van;
                // In the AFFINE V-run chain the next row needs the V-state run of THIS cell
                // (vt_up/vp_up above) and this cell's S type (slt_up): an extending V continues
                // the V-state run, an opening V starts from the S-state (same run iff slt==V).
            }
        }

        // ---- row L (the adapter's last row): H-state run and scout ----
        int ht, hp;
        if (AFFINE) {
            if (l_hext) { ht = ht_last + 1; hp = hp_last; }
            else open_run(slt_last, LT_H, ht_last, hp_last, ht, hp);
        } else {
            open_run(slt_last, LT_H, ht_last, hp_last, ht, hp);
        }
        if (ls > best.score && (!CHUNK || (j >= own_lo && j < hi))) {   // last row, columns 1..n-1 in order; (L, n) ends the last column
            best.score = ls; best.bi = L; best.bj = j;
            int vt = 0, vp = 0;
            if (lastcol) { vt = vt_up; vp = vp_up; }
            if (AFFINE) {
                if (lv == ls)      { best.attr = lva; best.ltype = LT_V; best.trail = vt; best.precd = vp; }
                else if (lh == ls) { best.attr = lha; best.ltype = LT_H; best.trail = ht; best.precd = hp; }
                else               { best.attr = lsa; best.ltype = LT_D; best.trail = 0; best.precd = 0; }
            } else {
                best.attr = lsa; best.ltype = lt_type;
                best.trail = (lt_type == LT_V) ? vt : (lt_type == LT_H ? ht : 0);
                best.precd = (lt_type == LT_V) ? vp : (lt_type == LT_H ? hp : 0);
            }
        }
        if (AFFINE) {
            ht_last = ht; hp_last = hp;
        } else {
            if (lt_type == LT_H) { ht_last = ht; hp_last = hp; }
            else { ht_last = 0; hp_last = 0; }
        }
        slt_last = lt_type;
    }
    return finish(best, L, fin ? n : n + 1);
}

// ------------------------------------------------------------------------------------------
// align_lane_striped<R, AFFINE>: adapters of any length up to MAX_STRIPED_LEN and any scoring --
// the core for everything the register-resident cores cannot hold (L > 128; the reference puts
// no bound on the adapter, porechop_abi/src/adapter_align.cpp:11-31).
//
// The adapter's rows are cut into stripes of R rows (the table is top-padded to rt rows, a
// multiple of R; the first stripe skips its padding slots by a wave-uniform branch, as the
// generic core does). One lane sweeps the window once per stripe with the stripe's rows in
// registers, running exactly align_lane_generic's recurrences; between stripes the stripe's
// bottom row (S- and V-state values with their attributes, per column) goes through a per-lane
// boundary buffer `bnd`, which the next stripe reads as its row 0. Two more things cross
// stripes, in registers: the last column's running V-run state (its rows flow top-down), and
// `bc`, the first maximum of the last column over the rows above the final stripe. The final
// stripe merges bc into its last-row scout at column n before its own last-column rows: the
// reference's visit order (S/align/dp_scout.h:175: the last row left to right, then the last
// column top-down, strict '>').
// Attributes are two words and never wrap: c = j0 - i0, and nD << 16 | m.
//
//   bnd.load(j, BndCell &) / bnd.store(j, const BndCell &), j = 1..n: the boundary row
//   adp.load(k) loads stripe k (table slots kR+1 .. kR+R), adp(s) = code of slot s of it
// CHUNK semantics as align_lane_generic's (own_lo / own_hi).
// ------------------------------------------------------------------------------------------
constexpr int MAX_STRIPED_LEN = 65535;           // nD, m <= L fit 16 bits each
constexpr uint32_t INC2_D = 1u << 16;            // mismatching diagonal: nD + 1
constexpr uint32_t INC2_M = INC2_D + 1u;         // matching diagonal: nD + 1, m + 1
constexpr int SCORE_FLOOR = -(1 << 30);          // below every reachable score

// One column of the row above a stripe: S- and V-state values with their attributes.
struct BndCell {
    int s, v;
    int32_t sc, vc;     // start diagonals
    uint32_t sn, vn;    // nD << 16 | m
};

// Scout state: the end cell (Best's geometry; attr unused) and the path's two attribute words.
struct BestS {
    Best b;
    int32_t c;
    uint32_t n;
};

template <int R, bool AFFINE>
struct StripeDP {
    int S[R + 1], H[R + 1];
    int32_t SC[R + 1], HC[R + 1];
    uint32_t SN[R + 1], HN[R + 1];
    BestS best;                          // last row (final stripe) and, from column n on, everything
    BestS bc;                            // last column, rows above the final stripe
    int cslt, cvt, cvp;                  // last column: S type and V run (t, p) at the row above
    int slt_last, ht_last, hp_last;      // row L running state (final stripe)
    int sdg;                             // S(row above the stripe, j - 1) and its attributes
    int32_t sdc;
    uint32_t sdn;

    PCABI_HD void init_stripe(int ib, int off) {
#pragma unroll
        for (int s = 1; s <= R; ++s) {
            S[s] = 0;
            H[s] = NEG;
            SC[s] = -(ib + s);           // S(i, 0) = 0, the path starts at (i, 0)
            SN[s] = 0;
            HC[s] = 0;
            HN[s] = 0;
        }
        sdg = 0;
        sdc = -(ib + off);
        sdn = 0;
        slt_last = LT_NONE;
        ht_last = 0;
        hp_last = 0;
    }

    // One column of the stripe. ib: absolute row of slot s is ib + s; off: padding slots to skip;
    // fin: the stripe holds row L; owned: this column may hold the last-row end cell.
    // Writes the stripe's bottom row at this column to `bot`.
    template <bool LAST, typename AdpFn>
    PCABI_HD void column(const int r, const int j, const BndCell &up, const AdpFn &adp, const int off, const int ib,
                         const int L, const bool fin, const bool owned, const Scoring &sc, BndCell &bot) {
        int sup = up.s, vup = up.v;
        int32_t scup = up.sc, vcup = up.vc;
        uint32_t snup = up.sn, vnup = up.vn;
        int dg = sdg;
        int32_t dgc = sdc;
        uint32_t dgn = sdn;
        int slt_up = cslt, vt_up = cvt, vp_up = cvp;
        if (LAST && fin && bc.b.score > best.b.score) best = bc;
        int lv = NEG, lh = NEG, ls = 0, lt_type = LT_NONE;
        bool l_hext = false;
        int32_t lvc = 0, lhc = 0, lsc = 0;
        uint32_t lvn = 0, lhn = 0, lsn = 0;
#pragma unroll
        for (int s = 1; s <= R; ++s) {
            if (s > off) {
                const bool match = (r == adp(s));
                const int diag = dg + (match ? sc.ma : sc.mi);
                const uint32_t dn = dgn + (match ? INC2_M : INC2_D);
                int hn, vn, g;
                int32_t hc, vc, gc;
                uint32_t hnn, vnn, gn;
                bool hext, vext, fromv;
                if (AFFINE) {
                    const int hx = H[s] + sc.ge, ho = S[s] + sc.go;
                    hext = !(hx < ho);
                    hn = hext ? hx : ho;
                    hc = hext ? HC[s] : SC[s];
                    hnn = hext ? HN[s] : SN[s];
                    const int vx = vup + sc.ge, vo = sup + sc.go;
                    vext = !(vx < vo);
                    vn = vext ? vx : vo;
                    vc = vext ? vcup : scup;
                    vnn = vext ? vnup : snup;
                    fromv = !(vn < hn);
                    g = fromv ? vn : hn;
                    gc = fromv ? vc : hc;
                    gn = fromv ? vnn : hnn;
                } else {
                    hext = vext = false;
                    const int vv = sup + sc.ge, hh = S[s] + sc.ge;
                    fromv = !(vv < hh);
                    g = fromv ? vv : hh;
                    gc = fromv ? scup : SC[s];
                    gn = fromv ? snup : SN[s];
                    hn = NEG; vn = NEG; hc = vc = 0; hnn = vnn = 0;
                }
                const bool isd = !(diag < g);
                const int sn = isd ? diag : g;
                const int32_t snc = isd ? dgc : gc;
                const uint32_t snn = isd ? dn : gn;
                const int slt = isd ? LT_D : (fromv ? LT_V : LT_H);
                const bool lastrow = fin && s == R;
                if (LAST) {
                    int vt, vp;
                    if (AFFINE && vext) { vt = vt_up + 1; vp = vp_up; }
                    else open_run(slt_up, LT_V, vt_up, vp_up, vt, vp);
                    if (!lastrow) {                 // last column, rows 1..L-1 in order
                        BestS &t = fin ? best : bc;
                        if (sn > t.b.score) {
                            t.b.score = sn;
                            t.b.bi = ib + s;
                            t.b.bj = j;
                            if (AFFINE) {
                                if (vn == sn)      { t.c = vc; t.n = vnn; t.b.ltype = LT_V; t.b.trail = vt; t.b.precd = vp; }
                                else if (hn == sn) { t.c = hc; t.n = hnn; t.b.ltype = LT_H; t.b.trail = 0; t.b.precd = 0; }
                                else               { t.c = snc; t.n = snn; t.b.ltype = LT_D; t.b.trail = 0; t.b.precd = 0; }
                            } else {
                                t.c = snc; t.n = snn; t.b.ltype = slt;
                                t.b.trail = (slt == LT_V) ? vt : 0;
                                t.b.precd = (slt == LT_V) ? vp : 0;
                            }
                        }
                    }
                    if (AFFINE || slt == LT_V) { vt_up = vt; vp_up = vp; }
                    else { vt_up = 0; vp_up = 0; }
                    slt_up = slt;
                }
                if (lastrow) {
                    lv = vn; lh = hn; ls = sn; lvc = vc; lhc = hc; lsc = snc; lvn = vnn; lhn = hnn; lsn = snn;
                    lt_type = slt; l_hext = hext;
                }
                dg = S[s];
                dgc = SC[s];
                dgn = SN[s];
                S[s] = sn;
                SC[s] = snc;
                SN[s] = snn;
                if (AFFINE) {
                    H[s] = hn;
                    HC[s] = hc;
                    HN[s] = hnn;
                }
                sup = sn; scup = snc; snup = snn;
                vup = vn; vcup = vc; vnup = vnn;
            }
        }
        if (LAST) { cslt = slt_up; cvt = vt_up; cvp = vp_up; }
        sdg = up.s;
        sdc = up.sc;
        sdn = up.sn;
        bot.s = sup; bot.v = vup; bot.sc = scup; bot.vc = vcup; bot.sn = snup; bot.vn = vnup;
        if (!fin) return;
        // ---- row L: H-state run and the last-row scout ----
        int ht, hp;
        if (AFFINE && l_hext) { ht = ht_last + 1; hp = hp_last; }
        else open_run(slt_last, LT_H, ht_last, hp_last, ht, hp);
        if (ls > best.b.score && owned) {
            best.b.score = ls;
            best.b.bi = L;
            best.b.bj = j;
            const int vt = LAST ? vt_up : 0, vp = LAST ? vp_up : 0;
            if (AFFINE) {
                if (lv == ls)      { best.c = lvc; best.n = lvn; best.b.ltype = LT_V; best.b.trail = vt; best.b.precd = vp; }
                else if (lh == ls) { best.c = lhc; best.n = lhn; best.b.ltype = LT_H; best.b.trail = ht; best.b.precd = hp; }
                else               { best.c = lsc; best.n = lsn; best.b.ltype = LT_D; best.b.trail = 0; best.b.precd = 0; }
            } else {
                best.c = lsc; best.n = lsn; best.b.ltype = lt_type;
                best.b.trail = (lt_type == LT_V) ? vt : (lt_type == LT_H ? ht : 0);
                best.b.precd = (lt_type == LT_V) ? vp : (lt_type == LT_H ? hp : 0);
            }
        }
        if (AFFINE || lt_type == LT_H) { ht_last = ht; hp_last = hp; }
        else { ht_last = 0; hp_last = 0; }
        slt_last = lt_type;
    }
};

template <int R, bool AFFINE, typename ReadFn, typename AdpFn, typename BndFn>
PCABI_HD Result align_lane_striped(const ReadFn &rd0, int n, AdpFn &adp, int L, int rt, const Scoring sc, BndFn &bnd,
                                   int own_lo = 1, int own_hi = -1) {
    const bool fin_read = own_hi < 0;      // the window's last column is the read's last column
    const int hi = fin_read ? n + 1 : own_hi;
    const int pad = rt - L, k0 = pad / R, nst = rt / R;
    StripeDP<R, AFFINE> st;
    st.best.b.score = 0;                   // first scouted cell: (L, 0), S = 0
    st.best.b.bi = L;
    st.best.b.bj = 0;
    st.best.b.attr = 0;
    st.best.b.ltype = LT_NONE;
    st.best.b.trail = 0;
    st.best.b.precd = 0;
    st.best.c = -L;
    st.best.n = 0;
    st.bc = st.best;
    st.bc.b.score = SCORE_FLOOR;
    st.cslt = LT_NONE;
    st.cvt = 0;
    st.cvp = 0;
#pragma unroll 1
    for (int k = k0; k < nst; ++k) {
        adp.load(k);
        const bool first = k == k0, fin = k == nst - 1;
        const int off = first ? pad - k0 * R : 0;
        const int ib = k * R - pad;
        st.init_stripe(ib, off);
        ReadFn rd = rd0;
        BndCell up, nx, bot;
        auto row0 = [](int j, BndCell &u) { u.s = 0; u.v = NEG; u.sc = j; u.vc = 0; u.sn = 0; u.vn = 0; };
        if (first) row0(1, up);
        else bnd.load(1, up);
        int r = rd(1);
#pragma unroll 1
        for (int j = 1; j < n; ++j) {
            const int rn = rd(j + 1);
            if (first) row0(j + 1, nx);
            else bnd.load(j + 1, nx);
            st.template column<false>(r, j, up, adp, off, ib, L, fin, j >= own_lo && j < hi, sc, bot);
            if (!fin) bnd.store(j, bot);
            up = nx;
            r = rn;
        }
        if (fin_read) st.template column<true>(r, n, up, adp, off, ib, L, fin, n >= own_lo && n < hi, sc, bot);
        else st.template column<false>(r, n, up, adp, off, ib, L, fin, n >= own_lo && n < hi, sc, bot);
        if (!fin) bnd.store(n, bot);
    }
    return finish_path(st.best.b, st.best.c, (int)(st.best.n & 0xFFFFu), (int)(st.best.n >> 16), L,
                       fin_read ? n : n + 1);
}

}  // namespace pcabi

namespace pcabi {

// ------------------------------------------------------------------------------------------
// align_lane_fast<RPL, AFFINE>: the production core. Branch-free rows.
//
// The adapter (length L) sits in register slots off+1..RPL, off = RPL - L in 0..3 (buckets are
// multiples of 4). Instead of skipping the padding slots (a branch per row that wrecks register
// allocation), the padding slots COMPUTE a pass-through row: their adapter code never matches
// (5), their mismatch score is 0 and their attribute increment advances the start column by one.
// With gap_open < 0 and gap_extend < 0 every padding cell then takes the diagonal with S = 0,
// V = H = gap_open (< 0), and attribute == attr_start(j): exactly the free-end-gap boundary row
// the first real row expects. Only slots 1..3 can be padding, so only they
// carry the two per-slot constants.
//
// Column n (the last) is peeled out of the loop: it alone scouts rows 1..L-1 and tracks the
// trailing-V bookkeeping. The last-row scout of every column uses selects, not branches.
// Preconditions (checked by the host): 1 <= L <= RPL <= L + 3; off == 0 or (go < 0 && ge < 0).
// ------------------------------------------------------------------------------------------
constexpr uint32_t INC_PAD = 1u << ATTR_CSH;   // padding diagonal: start column + 1

// gfx950 issues a VOP2 instruction that reads an SGPR at half rate: 4.4 cycles per wave64
// instruction against 2.45 for the same op on VGPRs or a literal (tools/replay_k24.hip rate probes,
// profiles/r06/replay). A core's per-call constants (gap extend / open keys) are uniform, so the
// compiler keeps them in SGPRs and every cell's adds pay that; vreg() pins such a value in a VGPR
// (an empty asm the compiler cannot see through) so the cell's adds read VGPRs only.
PCABI_HD int32_t vreg(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(x));
#endif
    return x;
}

PCABI_HD int max3i(int a, int b, int c) {   // one v_max3_i32 on gfx950
    const int ab = a > b ? a : b;
    return ab > c ? ab : c;
}
constexpr int PAD_CODE = 5;                     // never equal to a read code (0..4)

template <int RPL, bool AFFINE>
struct LaneDP {
    int S[RPL + 1], H[RPL + 1];
    uint32_t SA[RPL + 1], HA[RPL + 1];
    // best end cell so far
    int bscore, bi, bj, blt, btrail, bprec;
    uint32_t battr;
    // row-L running state: S-state last type at (L, j-1), H-state run (t, p) at (L, j-1)
    int slt_last, ht_last, hp_last;
    // per-slot constants for the only slots that may be padding
    int mis[4];
    uint32_t ids[4];

    template <typename AdpFn, bool LAST>
    PCABI_HD void column(const int r, const int j, const AdpFn &adp, const int L, const int off,
                         const Scoring &sc) {
        int sup = 0, vup = NEG;
        uint32_t saup = attr_start(j), vaup = 0;
        int slt_up = LT_NONE, vt_up = 0, vp_up = 0;
        int lv = 0, lh = 0, ls = 0, lslt = LT_D;
        bool lhext = false;
        uint32_t lva = 0, lha = 0, lsa = 0;
        // diagonal candidate of row 1 (from the boundary cell (0, j-1)); every row computes the
        // next row's candidate from its OLD S/SA before overwriting them (no rotation copies)
        bool match = (r == adp(1));
        int diag = 0 + (match ? sc.ma : mis[1]);
        uint32_t da = attr_start(j - 1) + ids[1] + (uint32_t)match;
#pragma unroll
        for (int s = 1; s <= RPL; ++s) {
            int diag_nx = 0;
            uint32_t da_nx = 0;
            if (s < RPL) {
                const bool mt = (r == adp(s + 1));
                const int mi_n = (s + 1 <= 3) ? mis[s + 1] : sc.mi;
                const uint32_t id_n = (s + 1 <= 3) ? ids[s + 1] : INC_D;
                diag_nx = S[s] + (mt ? sc.ma : mi_n);
                da_nx = SA[s] + id_n + (uint32_t)mt;
            }
            int hn, vn, sn;
            uint32_t han, van;
            bool hext, vext, fromv;
            if (AFFINE) {
                const int hx = H[s] + sc.ge, ho = S[s] + sc.go;
                hext = !(hx < ho);
                hn = hext ? hx : ho;
                han = hext ? HA[s] : SA[s];
                const int vx = vup + sc.ge, vo = sup + sc.go;
                vext = !(vx < vo);
                vn = vext ? vx : vo;
                van = vext ? vaup : saup;
            } else {
                hext = vext = false;
                vn = sup + sc.ge;
                hn = S[s] + sc.ge;
                van = saup;
                han = SA[s];
            }
            // S = max(diag, V, H); ties: diagonal, then V (S/align/dp_formula.h:153-163)
            sn = max3i(diag, vn, hn);
            const bool isd = (diag == sn);
            fromv = (vn == sn);
            const uint32_t san = isd ? da : (fromv ? van : han);
            if (LAST && s < RPL) {
                const int slt = isd ? LT_D : (fromv ? LT_V : LT_H);
                // trailing V run of the V-state (affine) or of the S-state from V (linear)
                const bool cont = AFFINE ? (vext || slt_up == LT_V) : (slt_up == LT_V);
                const int vt = cont ? vt_up + 1 : 1;
                const int vp = cont ? vp_up : (slt_up == LT_D ? 1 : 0);
                if (sn > bscore) {
                    bscore = sn;
                    bi = s - off;
                    bj = j;
                    if (AFFINE) {
                        const bool isv = (vn == sn), ish = !isv && (hn == sn);
                        battr = isv ? van : (ish ? han : san);
                        blt = isv ? LT_V : (ish ? LT_H : LT_D);
                        btrail = isv ? vt : 0;
                        bprec = isv ? vp : 0;
                    } else {
                        battr = san;
                        blt = slt;
                        btrail = (slt == LT_V) ? vt : 0;
                        bprec = (slt == LT_V) ? vp : 0;
                    }
                }
                if (AFFINE) { vt_up = vt; vp_up = vp; }
                else { vt_up = (slt == LT_V) ? vt : 0; vp_up = (slt == LT_V) ? vp : 0; }
                slt_up = slt;
            }
            if (s == RPL) {
                lv = vn; lh = hn; ls = sn; lva = van; lha = han; lsa = san; lhext = hext;
                lslt = isd ? LT_D : (fromv ? LT_V : LT_H);
                if (LAST) {
                    const bool cont = AFFINE ? (vext || slt_up == LT_V) : (slt_up == LT_V);
                    const int vt = cont ? vt_up + 1 : 1;
                    const int vp = cont ? vp_up : (slt_up == LT_D ? 1 : 0);
                    vt_up = vt;
                    vp_up = vp;
                }
            }
            S[s] = sn;
            SA[s] = san;
            if (AFFINE) {
                H[s] = hn;
                HA[s] = han;
            }
            sup = sn;
            vup = vn;
            saup = san;
            vaup = van;
            diag = diag_nx;
            da = da_nx;
#if defined(__HIP_DEVICE_COMPILE__)
            // keep the scheduler from hoisting every row's diagonal work to the column top
            // (it raises VGPR/SGPR pressure and costs occupancy)
            if (PCABI_ROW_FENCE > 0 && (s % (PCABI_ROW_FENCE > 0 ? PCABI_ROW_FENCE : 1)) == 0) __builtin_amdgcn_sched_barrier(0);
#endif
        }
        // ---- row L: H-state trailing run at (L, j) and the last-row scout ----
        const bool hcont = AFFINE ? (lhext || slt_last == LT_H) : (slt_last == LT_H);
        const int ht = hcont ? ht_last + 1 : 1;
        const int hp = hcont ? hp_last : (slt_last == LT_D ? 1 : 0);
        const bool upd = ls > bscore;
        int clt, ctrail, cprec;
        uint32_t cattr;
        if (AFFINE) {
            const bool isv = (lv == ls), ish = !isv && (lh == ls);
            cattr = isv ? lva : (ish ? lha : lsa);
            clt = isv ? LT_V : (ish ? LT_H : LT_D);
            ctrail = isv ? (LAST ? vt_up : 0) : (ish ? ht : 0);
            cprec = isv ? (LAST ? vp_up : 0) : (ish ? hp : 0);
        } else {
            cattr = lsa;
            clt = lslt;
            ctrail = (lslt == LT_V) ? (LAST ? vt_up : 0) : (lslt == LT_H ? ht : 0);
            cprec = (lslt == LT_V) ? (LAST ? vp_up : 0) : (lslt == LT_H ? hp : 0);
        }
        bscore = upd ? ls : bscore;
        bi = upd ? L : bi;
        bj = upd ? j : bj;
        battr = upd ? cattr : battr;
        blt = upd ? clt : blt;
        btrail = upd ? ctrail : btrail;
        bprec = upd ? cprec : bprec;
        if (AFFINE) { ht_last = ht; hp_last = hp; }
        else { ht_last = (lslt == LT_H) ? ht : 0; hp_last = (lslt == LT_H) ? hp : 0; }
        slt_last = lslt;
    }
};

template <int RPL, bool AFFINE, typename ReadFn, typename AdpFn>
PCABI_HD Result align_lane_fast(ReadFn &rd, int n, const AdpFn &adp, int L, const Scoring sc) {
    LaneDP<RPL, AFFINE> st;
    const int off = RPL - L;
#pragma unroll
    for (int s = 1; s <= RPL; ++s) {
        st.S[s] = 0;
        st.H[s] = NEG;
        st.SA[s] = attr_start(-(s > off ? s - off : 0));
        st.HA[s] = 0;
    }
#pragma unroll
    for (int s = 1; s <= 3; ++s) {
        st.mis[s] = (s <= off) ? 0 : sc.mi;
        st.ids[s] = (s <= off) ? INC_PAD : INC_D;
    }
    st.bscore = 0;   // first scouted cell (L, 0), S = 0
    st.bi = L;
    st.bj = 0;
    st.battr = attr_start(-L);
    st.blt = LT_NONE;
    st.btrail = 0;
    st.bprec = 0;
    st.slt_last = LT_NONE;
    st.ht_last = 0;
    st.hp_last = 0;
    // The code of column j+1 is requested at the top of column j and only consumed after the
    // column body, so the load has a whole column (RPL rows of VALU work) to land.
    int r = rd(1);
#pragma unroll 1
    for (int j = 1; j < n; ++j) {
        const int rn = rd(j + 1);      // buffers are padded: reading column n+... is safe
        st.template column<AdpFn, false>(r, j, adp, L, off, sc);
        r = rn;
    }
    st.template column<AdpFn, true>(r, n, adp, L, off, sc);
    Best b;
    b.score = st.bscore; b.bi = st.bi; b.bj = st.bj; b.attr = st.battr;
    b.ltype = st.blt; b.trail = st.btrail; b.precd = st.bprec;
    return finish(b, L, n);
}

// Which kernel core a (length, scoring) pair may use.
PCABI_HD bool fast_ok(int L, int rpl, const Scoring &sc) {
    const int off = rpl - L;
    if (off < 0 || off > 3) return false;
    if (off == 0) return true;
    return (sc.go != sc.ge) ? (sc.go < 0 && sc.ge < 0) : (sc.ge < 0);
}

}  // namespace pcabi

namespace pcabi {

// ==========================================================================================
// align_lane_packed<RPL, AFFINE>: the end-window core (RPL <= 32, windows <= 223 columns).
//
// Every DP value is ONE 32-bit signed key
//      [ score : 10 (signed) ][ tb : 2 ][ c + 32 : 8 ][ nD : 6 ][ m : 6 ]      (MSB .. LSB)
// so a plain signed max compares scores first, then the tie-break field tb, and carries the
// traceback attributes of the winner along for free: the reference's tie rules become tb
// values (S/align/dp_formula.h:153-163, dp_formula_affine.h:66-125):
//      stored S keys tb = 0, stored H keys tb = 1, V keys tb = 2, diagonal candidates tb = 3
//   H = max(H + ge [tb 1], S + go [tb 0])      -> extend wins ties
//   V = max(V + ge [tb 2], S + go [tb 0])      -> extend wins ties
//   S = max3(diag [tb 3], V|tb2 [tb 2], H [tb <= 1])  -> diagonal, then V, then H
// The substitution score and the attribute increment of a diagonal step are ONE add of a
// key-shaped constant (match / mismatch / padding). Per cell: 13 VALU ops (affine), 7 (linear),
// and 2 (affine) / 1 (linear) registers per adapter row -- versus 21 ops and 4 registers when
// scores and attributes live in separate registers (align_lane_fast).
//
// The start diagonal c is kept mod 256: nothing but the start keys ever writes the c field
// (padding rows add 0 to it -- the row-0 keys already carry the c of the real cell the padded
// path reaches), so it never carries into tb, and finish() recovers c from the end column
// because the best path spans < 256 columns (packed_ok). Windows of any length are accepted.
//
// Range conditions (checked by the host, packed_ok): every reachable score and the NEG
// sentinel fit the 10-bit field, m, nD <= L <= 63 fit 6 bits, span bound <= 255.
// ==========================================================================================
namespace pk {
// Key layout of a register bucket: RPL <= 64 keeps the layout above (score 10 bits, m / nD six
// bits each = m + 64 nD); the wide buckets (64 < RPL <= 88: the 63-111 bp "full sequence" barcode
// adapters) trade a score bit for a mixed-radix count field m + (RPL + 1) nD of 13 bits:
//      [ score : 9 (signed) ][ tb : 2 ][ c mod 256 : 8 ][ m + (RPL+1) nD : 13 ]
// Both counts grow only by adding the diagonal step's constant (INC_D / INC_M), so the field
// never carries (m <= nD <= L <= RPL).
template <int RPL>
struct Lay {
    static constexpr bool WIDE = RPL > 64;
    static constexpr bool TAGGED = false;
    static constexpr int SC_SH = WIDE ? 23 : 22;
    static constexpr int TB_SH = SC_SH - 2;
    static constexpr int C_SH = TB_SH - 8;
    static constexpr int MB = WIDE ? RPL + 1 : 64;              // radix of the count field
    static constexpr int32_t TB1 = 1 << TB_SH, TB2 = 2 << TB_SH, TB3 = 3 << TB_SH, TBM = 3 << TB_SH;
    static constexpr int32_t INC_D = MB, INC_M = MB + 1;
    static constexpr int SC_MIN = -(1 << (31 - SC_SH)), SC_MAX = (1 << (31 - SC_SH)) - 1;
    static PCABI_HD int32_t sc(int v) { return (int32_t)((uint32_t)v << SC_SH); }   // score -> key units
    static PCABI_HD int32_t start(int c) { return (int32_t)(((uint32_t)c & 255u) << C_SH); }   // c mod 256
    static PCABI_HD int score(int32_t k) { return k >> SC_SH; }
    static PCABI_HD int tb(int32_t k) { return (k >> TB_SH) & 3; }
    static PCABI_HD uint32_t attr(int32_t k) { return (uint32_t)k & ((1u << TB_SH) - 1u); }
    // packed attribute of a path ending in column bj -> standard attribute word (finish()):
    // c in [bj - 255, bj] is recovered from its residue mod 256
    static PCABI_HD uint32_t to_std(uint32_t a, int bj) {
        const uint32_t cnt = a & ((1u << C_SH) - 1u);
        const uint32_t m = cnt % (uint32_t)MB, nd = cnt / (uint32_t)MB;
        const int c = bj - (int)(((uint32_t)bj - (a >> C_SH)) & 255u);
        return attr_start(c) | (nd << ATTR_B) | m;
    }
};
// Long buckets (88 < RPL <= 128: the 102 / 111 bp full rapid-barcode sequences): the counts no
// longer fit next to the score, so the DP runs twice with the same scores and tie-break bits --
// which select the same path in both runs -- and a different payload each time:
//      pass 0: [ score : 12 (signed) ][ tb : 2 ][ c mod 1024 : 10 ][ nD : 8 ]
//      pass 1: [ score : 12 (signed) ][ tb : 2 ][ 0 : 10 ][ m : 8 ]
// A max never decides on the payload (candidates of one max differ in tb), so both passes keep
// the same winners everywhere, and their attributes merge into one path (align_lane_packed_long).
template <int RPL, int PASS>
struct LayL {
    static constexpr bool WIDE = true;
    static constexpr bool TAGGED = false;
    static constexpr int SC_SH = 20;
    static constexpr int TB_SH = 18;
    static constexpr int C_SH = 8;
    static constexpr int32_t TB1 = 1 << TB_SH, TB2 = 2 << TB_SH, TB3 = 3 << TB_SH, TBM = 3 << TB_SH;
    static constexpr int32_t INC_D = PASS == 0 ? 1 : 0, INC_M = 1;
    static constexpr int SC_MIN = -(1 << (31 - SC_SH)), SC_MAX = (1 << (31 - SC_SH)) - 1;
    static PCABI_HD int32_t sc(int v) { return (int32_t)((uint32_t)v << SC_SH); }
    static PCABI_HD int32_t start(int c) { return PASS == 0 ? (int32_t)(((uint32_t)c & 1023u) << C_SH) : 0; }
    static PCABI_HD int score(int32_t k) { return k >> SC_SH; }
    static PCABI_HD int tb(int32_t k) { return (k >> TB_SH) & 3; }
    static PCABI_HD uint32_t attr(int32_t k) { return (uint32_t)k & ((1u << TB_SH) - 1u); }
    static PCABI_HD uint32_t to_std(uint32_t a, int bj) {
        if (PASS == 1) return a & 255u;                         // m
        const uint32_t nd = a & 255u;
        const int c = bj - (int)(((uint32_t)bj - (a >> C_SH)) & 1023u);
        return attr_start(c) | (nd << ATTR_B);
    }
};
// Run-tagged buckets (affine gaps, adapters <= 31 bp: the end-window adapters): the tie-break
// field widens to a 7-bit tag that COUNTS the extends of the current gap run, so the H key needs
// no re-tagging before it is stored (one VALU op per cell less than Lay):
//      [ score : 8 (signed) ][ tag : 7 ][ c mod 128 : 7 ][ nD : 5 ][ m : 5 ]
//   H:  open = tag 0 (G = S + go as stored), extend = previous H tag + 1   -> extend wins ties
//   V:  open = tag VB = 127 - RPL (G + TVB), extend = previous V tag + 1   -> extend wins ties
//   diagonal candidates tag 127                                            -> D > V > H on ties
// H runs are bounded by the score range ((Smax - Smin) / |ge| extends, layt_ok checks < VB), V
// runs by the rows (a V run holds at most RPL - 1 extends: tags VB .. 126), so H tags stay below
// every V tag and V tags below 127. r02 used an 8-bit tag with c mod 64 (span < 64: adapters of
// <= 25 bp under the default scheme); the 7-bit tag frees a c bit and the 26-31 bp adapters (the
// 28 / 32-row buckets) fit too (span <= 76 at the default scheme).
template <int RPL>
struct LayT {
    static constexpr bool WIDE = false;
    static constexpr bool TAGGED = true;
    static constexpr int SC_SH = 24;
    static constexpr int TB_SH = 17;
    static constexpr int C_SH = 10;
    static constexpr int CB = 7;                        // c mod 128
    static constexpr int MB = 32;
    static constexpr int TD = 127;                      // diagonal tag (the tag field's maximum)
    static constexpr int VB = TD - RPL;                 // V-open tag
    static constexpr int32_t TAG1 = 1 << TB_SH, TVB = VB << TB_SH;
    static constexpr int32_t TB1 = TAG1, TB2 = TVB;   // the untagged core's names (unused here)
    static constexpr int32_t TB3 = TD << TB_SH, TBM = TD << TB_SH;
    static constexpr int32_t INC_D = MB, INC_M = MB + 1;
    static constexpr int SC_MIN = -128, SC_MAX = 127;
    static PCABI_HD int32_t sc(int v) { return (int32_t)((uint32_t)v << SC_SH); }
    static PCABI_HD int32_t start(int c) { return (int32_t)(((uint32_t)c & ((1u << CB) - 1u)) << C_SH); }
    static PCABI_HD int score(int32_t k) { return k >> SC_SH; }
    static PCABI_HD int tb(int32_t k) { return (k >> TB_SH) & TD; }
    static PCABI_HD uint32_t attr(int32_t k) { return (uint32_t)k & ((1u << TB_SH) - 1u); }
    static PCABI_HD uint32_t to_std(uint32_t a, int bj) {
        const uint32_t cnt = a & ((1u << C_SH) - 1u);
        const uint32_t m = cnt % (uint32_t)MB, nd = cnt / (uint32_t)MB;
        const int c = bj - (int)(((uint32_t)bj - (a >> C_SH)) & ((1u << CB) - 1u));
        return attr_start(c) | (nd << ATTR_B) | m;
    }
};
constexpr int MAX_RPL = 88;
constexpr int MAX_L = 88;
constexpr int MAX_L_LONG = 128;
// The sentinel NEG (H(., 0), V(0, .)) only ever competes in column 1 (H-extend vs H-open from
// S(i, 0) = 0) and row 1 (V-extend vs V-open from S(0, j) = 0): it must lose there, NEG + ge <
// gap_open, and nothing else (after those maxes every value is a real DP value).
PCABI_HD int neg_score(const Scoring &s) { return s.go - s.ge - 1; }
}  // namespace pk

// Columns spanned by the reported path: it scores >= 0 (the scout is seeded with 0), so its
// horizontal moves (each costing >= g) are paid for by at most L diagonal matches.
PCABI_HD int packed_span_bound(int L, const Scoring &s) {
    const int g = (-s.go < -s.ge) ? -s.go : -s.ge;
    const int p = best_sub(s);
    return L + (p > 0 ? (p * L) / g : 0);
}

// Range conditions of the packed core for an adapter of L bases in register bucket rpl:
//   * gaps cost (go, ge < 0): padding rows pass scores through, and the span bound exists;
//   * every key value fits the score field. All DP values of real rows are >= Smin = the
//     vertical path from row 0 (go + (L-1) ge; L ge linear) and <= L ma; the candidates and
//     stored keys add at most one gap pair or one substitution to a DP value: [Smin + min(go + ge,
//     mi, ma), max(L ma, 0)]; the sentinel and its one extension NEG + ge must fit too;
//   * m, nD <= L fit the count field, and the reported path spans < 256 columns (c mod 256).
template <int RPL>
PCABI_HD bool packed_ok_t(int L, const Scoring &s) {
    using Y = pk::Lay<RPL>;
    if (L < 1 || L > RPL || L > pk::MAX_L) return false;
    if (!(s.go < 0 && s.ge < 0)) return false;
    if (packed_span_bound(L, s) > 255) return false;
    const long long smin = (s.go != s.ge) ? (long long)s.go + (long long)(L - 1) * s.ge : (long long)L * s.ge;
    const long long lo_sub = s.mi < s.ma ? s.mi : s.ma;
    const long long lo_gap = (long long)s.go + s.ge;
    long long lo = smin + (lo_gap < lo_sub ? lo_gap : lo_sub);
    const long long neg = pk::neg_score(s);
    if (neg + s.ge < lo) lo = neg + s.ge;
    if (neg < lo) lo = neg;
    if (s.go < lo) lo = s.go;
    long long hi = (long long)L * best_sub(s);
    if (hi < 0) hi = 0;
    if (best_sub(s) > hi) hi = best_sub(s);
    if (!Y::WIDE && L > 63) return false;
    return lo >= Y::SC_MIN && hi <= Y::SC_MAX;
}

// Range conditions of the long (two-pass) layout: as packed_ok_t with the 12-bit score field,
// counts <= 255 and a reported path spanning < 1024 columns.
PCABI_HD bool long_ok(int L, int rpl, const Scoring &s) {
    using Y = pk::LayL<128, 0>;
    if (L < 1 || L > rpl || L > pk::MAX_L_LONG) return false;
    if (!(s.go < 0 && s.ge < 0)) return false;
    if (packed_span_bound(L, s) > 1023) return false;
    const long long smin = (s.go != s.ge) ? (long long)s.go + (long long)(L - 1) * s.ge : (long long)L * s.ge;
    const long long lo_sub = s.mi < s.ma ? s.mi : s.ma;
    const long long lo_gap = (long long)s.go + s.ge;
    long long lo = smin + (lo_gap < lo_sub ? lo_gap : lo_sub);
    const long long neg = pk::neg_score(s);
    if (neg + s.ge < lo) lo = neg + s.ge;
    if (neg < lo) lo = neg;
    if (s.go < lo) lo = s.go;
    long long hi = (long long)L * best_sub(s);
    if (hi < 0) hi = 0;
    if (best_sub(s) > hi) hi = best_sub(s);
    return lo >= Y::SC_MIN && hi <= Y::SC_MAX;
}

// Range conditions of the run-tagged layout (pk::LayT): affine gaps, the packed ranges with an
// 8-bit score field, counts <= 31, a reported path spanning < 128 columns (c mod 128), and every H
// run shorter than VB = 127 - rpl extends: an extend at (i, j) needs H(i, j-1) + ge >= S(i, j-1) +
// go >= Smin + go, and a run that opened at <= Smax + go loses |ge| per extend, so a run holds at
// most (Smax - Smin) / |ge| extends (Smax = max(L best_sub, 0), Smin = go + (L-1) ge; padding rows
// stay at S = 0 and never extend).
PCABI_HD bool layt_ok(int L, int rpl, const Scoring &s) {
    using Y = pk::LayT<32>;
    if (L < 1 || L > rpl || rpl > 32 || L > 31) return false;
    if (!(s.go < 0 && s.ge < 0) || s.go == s.ge) return false;
    if (packed_span_bound(L, s) >= (1 << Y::CB)) return false;
    const long long smin = (long long)s.go + (long long)(L - 1) * s.ge;
    const long long lo_sub = s.mi < s.ma ? s.mi : s.ma;
    const long long lo_gap = (long long)s.go + s.ge;
    long long lo = smin + (lo_gap < lo_sub ? lo_gap : lo_sub);
    const long long neg = pk::neg_score(s);
    if (neg + s.ge < lo) lo = neg + s.ge;
    if (neg < lo) lo = neg;
    if (s.go < lo) lo = s.go;
    long long hi = (long long)L * best_sub(s);
    if (hi < 0) hi = 0;
    if (best_sub(s) > hi) hi = best_sub(s);
    if (lo < Y::SC_MIN || hi > Y::SC_MAX) return false;
    const long long smax = hi;
    return (smax - smin) / (-(long long)s.ge) + 1 < Y::TD - rpl;
}

PCABI_HD bool packed_ok(int L, int rpl, const Scoring &s) {
    switch (rpl) {
#define PCABI_PK(R) case R: return packed_ok_t<R>(L, s);
    PCABI_PK(4) PCABI_PK(8) PCABI_PK(12) PCABI_PK(16) PCABI_PK(20) PCABI_PK(24) PCABI_PK(28) PCABI_PK(32)
    PCABI_PK(36) PCABI_PK(40) PCABI_PK(44) PCABI_PK(48) PCABI_PK(52) PCABI_PK(56) PCABI_PK(60) PCABI_PK(64)
    PCABI_PK(68) PCABI_PK(72) PCABI_PK(76) PCABI_PK(80) PCABI_PK(84) PCABI_PK(88)
#undef PCABI_PK
    default: return false;
    }
}

template <int RPL, bool AFFINE, typename LAY = pk::Lay<RPL>, int PD = PCABI_TAB_PD>
struct LanePacked {
    using Y = LAY;
    int32_t G[RPL + 1];    // S keys with tb cleared, plus the gap-open key: G = S + go
    int32_t HK[RPL + 1];   // H keys, tb = 1 (affine only)
    int bscore, bi, bj, blt, btrail, bprec;
    uint32_t battr;        // packed attribute
    int slt_last, ht_last, hp_last;
    int32_t k_ge, k_go, k_gev, k_geh, neg2;
    int32_t k_gex, k_vo;   // run-tagged layout: gap extend + one tag, V-open tag
    // Last-row scout of the inner columns (column_tail): the best so far as ONE corrected key
    // (score | tag | attributes), its column, and the H-run descriptor at that column; the
    // fields above are materialised from them before the last column (materialize()).
    int32_t bkey;

    // tab: substitution-key table of this lane's read code, tab(s) = key increment of the
    // diagonal step into slot s (match / mismatch / padding), see pk::fill_sub_table.
    // GATE (chunked reads): only owned columns may become the row-L best (owned per column).
    template <typename TabRow, bool LAST, bool GATE = false>
    PCABI_HD void column(const TabRow &tab, const int j, const int L, const int off, const bool owned = true) {
        int32_t gup = Y::start(j + off) + k_go;   // G(0, j): S(0, j) = score 0, tb 0
        int32_t vup = neg2;                        // V(0, j) = NEG, tb 2
        int slt_up = LT_NONE, vt_up = 0, vp_up = 0;
        int32_t lv = 0, lh = 0, ls = 0;
        int lslt = LT_D;
        bool lhext = false;
        // Substitution keys of this column, fetched a quad (4 slots) at a time, PD
        // quads ahead of use so the LDS latency hides behind the rows in flight.
        constexpr int NQ = RPL / 4;
        int32_t t[RPL + 2];
        if (PD > 0) {
#pragma unroll
            for (int q = 0; q <= PD && q < NQ; ++q) tab.quad(q, t + 4 * q + 1);
        }
        int32_t diag = (Y::start(j - 1 + off) + k_go) + (PD > 0 ? t[1] : tab(1));
#pragma unroll
        for (int s = 1; s <= RPL; ++s) {
            if (PD > 0 && (s & 3) == 1) {
                const int q = (s - 1) / 4 + PD + 1;
                if (q < NQ) tab.quad(q, t + 4 * q + 1);
            }
            int32_t diag_nx = 0;
            if (s < RPL) diag_nx = G[s] + (PD > 0 ? t[s + 1] : tab(s + 1));
            int32_t hn, vn2, sn;
            bool hext = false, vext = false;
            if (AFFINE && Y::TAGGED) {
                const int32_t hx = HK[s] + k_gex, ho = G[s];
                hn = hx > ho ? hx : ho;                  // tag > 0 iff extend
                const int32_t vx = vup + k_gex, vo = gup + k_vo;
                vn2 = vx > vo ? vx : vo;                 // tag > VB iff extend
                if (LAST || s == RPL) { hext = Y::tb(hn) != 0; vext = Y::tb(vn2) > Y::TB2 >> Y::TB_SH; }
            } else if (AFFINE) {
                const int32_t hx = HK[s] + k_ge, ho = G[s];
                hn = hx > ho ? hx : ho;                  // tb 1 iff extend
                const int32_t vx = vup + k_ge, vo = gup;
                const int32_t vn = vx > vo ? vx : vo;    // tb 2 iff extend
                vn2 = vn | Y::TB2;
                if (LAST || s == RPL) { hext = Y::tb(hn) == 1; vext = Y::tb(vn) == 2; }
            } else {
                vn2 = gup + k_gev;                       // tb 2
                hn = G[s] + k_geh;                       // tb 1
            }
            sn = max3i(diag, vn2, hn);
            const int t = Y::tb(sn);
            const int slt = Y::TAGGED ? (t == (Y::TBM >> Y::TB_SH) ? LT_D : (t >= (Y::TB2 >> Y::TB_SH) ? LT_V : LT_H))
                                      : (t == 3 ? LT_D : (t == 2 ? LT_V : LT_H));
            if (LAST && s < RPL) {
                const bool cont = AFFINE ? (vext || slt_up == LT_V) : (slt_up == LT_V);
                const int vt = cont ? vt_up + 1 : 1;
                const int vp = cont ? vp_up : (slt_up == LT_D ? 1 : 0);
                const int sc_s = Y::score(sn);
                if (sc_s > bscore) {
                    bscore = sc_s;
                    bi = s - off;
                    bj = j;
                    if (AFFINE) {
                        const bool isv = Y::score(vn2) == sc_s, ish = !isv && Y::score(hn) == sc_s;
                        battr = Y::attr(isv ? vn2 : (ish ? hn : sn));
                        blt = isv ? LT_V : (ish ? LT_H : LT_D);
                        btrail = isv ? vt : 0;
                        bprec = isv ? vp : 0;
                    } else {
                        battr = Y::attr(sn);
                        blt = slt;
                        btrail = (slt == LT_V) ? vt : 0;
                        bprec = (slt == LT_V) ? vp : 0;
                    }
                }
                if (AFFINE) { vt_up = vt; vp_up = vp; }
                else { vt_up = (slt == LT_V) ? vt : 0; vp_up = (slt == LT_V) ? vp : 0; }
                slt_up = slt;
            }
            if (s == RPL) {
                lv = vn2; lh = hn; ls = sn; lslt = slt; lhext = hext;
                if (LAST) {
                    const bool cont = AFFINE ? (vext || slt_up == LT_V) : (slt_up == LT_V);
                    const int vt = cont ? vt_up + 1 : 1;
                    const int vp = cont ? vp_up : (slt_up == LT_D ? 1 : 0);
                    vt_up = vt;
                    vp_up = vp;
                }
            }
            G[s] = (sn & ~Y::TBM) + k_go;
            if (AFFINE) HK[s] = Y::TAGGED ? hn : (hn | Y::TB1);
            gup = G[s];
            vup = vn2;
            diag = diag_nx;
#if defined(__HIP_DEVICE_COMPILE__)
            if (PCABI_ROW_FENCE > 0 && (s % (PCABI_ROW_FENCE > 0 ? PCABI_ROW_FENCE : 1)) == 0) __builtin_amdgcn_sched_barrier(0);
#endif
        }
        if (!LAST) {
            column_tail<GATE>(lv, lh, ls, j, owned);
            return;
        }
        // ---- row L (last column) ----
        const bool hcont = AFFINE ? (lhext || slt_last == LT_H) : (slt_last == LT_H);
        const int ht = hcont ? ht_last + 1 : 1;
        const int hp = hcont ? hp_last : (slt_last == LT_D ? 1 : 0);
        const int lsc = Y::score(ls);
        const bool upd = lsc > bscore;
        int clt, ctrail, cprec;
        uint32_t cattr;
        if (AFFINE) {
            const bool isv = Y::score(lv) == lsc, ish = !isv && Y::score(lh) == lsc;
            cattr = Y::attr(isv ? lv : (ish ? lh : ls));
            clt = isv ? LT_V : (ish ? LT_H : LT_D);
            ctrail = isv ? (LAST ? vt_up : 0) : (ish ? ht : 0);
            cprec = isv ? (LAST ? vp_up : 0) : (ish ? hp : 0);
        } else {
            cattr = Y::attr(ls);
            clt = lslt;
            ctrail = (lslt == LT_V) ? (LAST ? vt_up : 0) : (lslt == LT_H ? ht : 0);
            cprec = (lslt == LT_V) ? (LAST ? vp_up : 0) : (lslt == LT_H ? hp : 0);
        }
        bscore = upd ? lsc : bscore;
        bi = upd ? L : bi;
        bj = upd ? j : bj;
        battr = upd ? cattr : battr;
        blt = upd ? clt : blt;
        btrail = upd ? ctrail : btrail;
        bprec = upd ? cprec : bprec;
        if (AFFINE) { ht_last = ht; hp_last = hp; }
        else { ht_last = (lslt == LT_H) ? ht : 0; hp_last = (lslt == LT_H) ? hp : 0; }
        slt_last = lslt;
    }

    // Row-L scout of an inner column, with the reference's rules (S/align/dp_scout.h:175, strict
    // '>' so the first maximum wins; start-state correction V, then H, then S). Affine: the
    // corrected state is ONE max over re-tagged keys -- V (tag 3) beats S (tag 0) on equal
    // scores, a higher score always wins. Linear gaps: no correction, the S key's own tb (3 D,
    // 2 V, 1 H) is the type.
    // The H state never wins a scout update here, so neither H nor its trailing run is tracked:
    // the packed cores need gap costs < 0, and an update at (L, j) means S(L, j) > S(L, j') for
    // every earlier column j' (the (L, 0) seed's 0 included), while H(L, j) <= max(H(L, j-1),
    // S(L, j-1)) + max(go, ge) < S(L, j-1) -- so H(L, j) == S(L, j) (the H correction, or an S
    // that came from H) is impossible there. In a chunk (GATE) the first owned column can
    // update after an unowned higher one, but then the previous chunk holds a strictly higher
    // score and wins the merge (sf::chunk_plan); the same holds for the last column's (L, n).
    template <bool GATE = false>
    PCABI_HD void column_tail(int32_t lv, int32_t lh, int32_t ls, int j, bool owned = true) {
        (void)lh;
        int32_t corr;
        if (AFFINE && Y::TAGGED) corr = std::max(lv, ls & ~Y::TBM);   // V tags >= VB > 0
        else if (AFFINE) corr = std::max(lv | Y::TB3, ls & ~Y::TBM);
        else corr = ls;
        bool upd = corr > (bkey | ((1 << Y::SC_SH) - 1));   // score(corr) > score(bkey)
        if (GATE) upd = upd && owned;
        bkey = upd ? corr : bkey;
        bj = upd ? j : bj;
    }

    // Inner-column scout state -> the fields the last column and finish() use (no H-state
    // best, see column_tail: the trailing-H bookkeeping of the last column starts empty).
    PCABI_HD void materialize(int L) {
        const int t = Y::tb(bkey);
        int lt;
        if (bj == 0) lt = LT_NONE;                          // still the (L, 0) seed
        else if (AFFINE) lt = (Y::TAGGED ? t != 0 : t == 3) ? LT_V : LT_D;
        else lt = t == 3 ? LT_D : (t == 2 ? LT_V : LT_H);
        bscore = Y::score(bkey);
        bi = L;
        battr = Y::attr(bkey);
        blt = lt;
        btrail = 0;                                        // a V run in row L before the last
        bprec = 0;                                         // column is a 1-column trail: 0 here
        slt_last = LT_NONE;
        ht_last = 0;
        hp_last = 0;
    }
};

// Substitution-key table: row c (read code 0..7) holds, for slots s = 1..RPL at index s - 1, the
// key increment of a diagonal step into slot s: match / mismatch keys, or the pass-through
// padding key for slots <= off. Rows are RPL int32 long (RPL % 4 == 0) so a quad of slots is one
// 16-byte LDS read.
// One table per adapter (wave-uniform); kernels keep it in LDS so the per-cell substitution is
// one LDS read + one add instead of a compare + select.
namespace pk {
constexpr int TAB_W = 8;
template <int RPL, typename AdpFn, typename Y = Lay<RPL>>
PCABI_HD int32_t sub_key(int s, int c, const AdpFn &adp, int off, const Scoring &sc) {
    // the core adds these to G = S + go, so the gap-open key is taken back out here
    if (s <= off) return Y::TB3 - Y::sc(sc.go);
    return (c == adp(s)) ? (Y::sc(sc.ma) + Y::TB3 + Y::INC_M - Y::sc(sc.go))
                         : (Y::sc(sc.mi) + Y::TB3 + Y::INC_D - Y::sc(sc.go));
}
}  // namespace pk

// CHUNK: the window is one chunk of a longer read (middle-scan candidates): only
// columns [own_lo, own_hi) may hold the reported end cell, and own_hi < 0 marks the read's last
// chunk (its last column is the read end); an inner chunk ends on an inner read column, so no
// last-column cell of it is an alignment end and its tail is reported as not at the read end.
template <int RPL, bool AFFINE, bool CHUNK = false, typename Y = pk::Lay<RPL>, int PD = PCABI_TAB_PD,
          typename ReadFn, typename TabFn>
PCABI_HD Best packed_best(ReadFn &rd, int n, const TabFn &tabfn, int L, const Scoring sc, int own_lo, int own_hi,
                          int &n_fin) {
    // tabfn(r) returns a callable row(s) -> substitution key for read code r
    LanePacked<RPL, AFFINE, Y, PD> st;
    const int off = RPL - L;
    const int32_t neg = Y::sc(pk::neg_score(sc));
    st.k_ge = Y::sc(sc.ge);
    st.k_go = Y::sc(sc.go);
    // linear gaps: V / H straight from G (= S + go), so the constants take go back out
    st.k_gev = Y::sc(sc.ge) - Y::sc(sc.go) + Y::TB2;
    st.k_geh = Y::sc(sc.ge) - Y::sc(sc.go) + Y::TB1;
    st.k_gex = Y::sc(sc.ge) + (Y::TAGGED ? Y::TB1 : 0);
    st.k_vo = Y::TAGGED ? Y::TB2 : 0;
    // the cell's adds read these: VGPR operands, not SGPR (vreg)
    st.k_ge = vreg(st.k_ge);
    st.k_go = vreg(st.k_go);
    st.k_gex = vreg(st.k_gex);
#pragma unroll
    for (int s = 1; s <= RPL; ++s) {
        st.G[s] = Y::start(off - s) + st.k_go;    // padded (s, 0) reaches real (0, off - s)
        st.HK[s] = Y::TAGGED ? neg : (neg | Y::TB1);
    }
    st.neg2 = neg | Y::TB2;
    st.bkey = Y::start(-L);                       // the (L, 0) seed: score 0, c = -L
    st.bj = 0;
    int r = rd(1);
    const int hi = own_hi < 0 ? n + 1 : own_hi;
#pragma unroll 1
    for (int j = 1; j < n; ++j) {
        const int rn = rd(j + 1);
        if (CHUNK) st.template column<decltype(tabfn(r)), false, true>(tabfn(r), j, L, off, j >= own_lo && j < hi);
        else st.template column<decltype(tabfn(r)), false>(tabfn(r), j, L, off);
        r = rn;
    }
    n_fin = n;
    if (CHUNK && own_hi >= 0) {
        st.template column<decltype(tabfn(r)), false, true>(tabfn(r), n, L, off, n >= own_lo && n < hi);
        st.materialize(L);
        n_fin = n + 1;                            // the read goes on past the chunk
    } else {
        st.materialize(L);
        st.template column<decltype(tabfn(r)), true>(tabfn(r), n, L, off);
    }
    Best b;
    b.score = st.bscore; b.bi = st.bi; b.bj = st.bj; b.attr = Y::to_std(st.battr, st.bj);
    b.ltype = st.blt; b.trail = st.btrail; b.precd = st.bprec;
    return b;
}

template <int RPL, bool AFFINE, bool CHUNK = false, typename Y = pk::Lay<RPL>, typename ReadFn, typename TabFn>
PCABI_HD Result align_lane_packed(ReadFn &rd, int n, const TabFn &tabfn, int L, const Scoring sc, int own_lo = 1,
                                  int own_hi = -1) {
    int n_fin;
    const Best b = packed_best<RPL, AFFINE, CHUNK, Y>(rd, n, tabfn, L, sc, own_lo, own_hi, n_fin);
    return finish(b, L, n_fin);
}

// Long buckets: pass 0 (c, nD) and pass 1 (m) over the same window (two readers, two tables);
// the passes end in the same cell with the same trailing run, so one Best carries all three.
template <int RPL, bool AFFINE, bool CHUNK = false, typename ReadFn, typename TabFn0, typename TabFn1>
PCABI_HD Result align_lane_packed_long(ReadFn &rd0, ReadFn &rd1, int n, const TabFn0 &tab0, const TabFn1 &tab1,
                                       int L, const Scoring sc, int own_lo = 1, int own_hi = -1) {
    int n_fin;
    Best b = packed_best<RPL, AFFINE, CHUNK, pk::LayL<RPL, 0>, PCABI_TAB_PD_LONG>(rd0, n, tab0, L, sc, own_lo, own_hi,
                                                                                 n_fin);
    const Best bm = packed_best<RPL, AFFINE, CHUNK, pk::LayL<RPL, 1>, PCABI_TAB_PD_LONG>(rd1, n, tab1, L, sc, own_lo,
                                                                                        own_hi, n_fin);
    b.attr |= bm.attr;
    return finish(b, L, n_fin);
}

// ==========================================================================================
// Row-split packed core (k_align_split: launches too small to fill the chip). One
// adapter over 100k end windows is 1.5 waves per SIMD, and a lane's DP over its 150 columns is a
// dependency chain the SIMD cannot hide with so few waves. Here K lanes share a window, lane l
// holding the bucket's rows r0 + 1 .. r0 + R (r0 = l R, K R = RPL), and the lanes form a systolic
// pipeline: at step t lane l computes column j = t - l from row r0's G and V keys at column j,
// which lane l - 1 computed at step t - 1 (lane 0 takes row 0). The inner columns' row-L scout is
// the last lane's. The last column runs in K phases, lane p in phase p, passing down the running
// first maximum over the column's rows (B2) and the V-run state; the last lane merges B2 into its
// row-L best -- the reference's visit order: the last row, then the last column top down, strict
// '>' (S/align/dp_scout.h:175) -- and finishes. Same keys, maxes and tie rules as LanePacked, so
// the results are identical. The steps are member functions: the kernel runs the K lanes of a
// window side by side (a lane shift per exchanged value), the host model in lockstep.
// ==========================================================================================
struct SplitIn {   // lane l - 1's state after its part of the last column
    int32_t gup, vup;             // its bottom row's G and V keys
    int slt, vt, vp;              // the V-run state there
    int score, bi, lt, trail, prec;   // the running first maximum of the column's rows (B2)
    uint32_t attr;
};

template <int R, bool AFFINE, typename LAY>
struct LaneSplit {
    using Y = LAY;
    int32_t G[R + 1];     // S keys with tb cleared + gap open (LanePacked's G)
    int32_t HK[R + 1];    // H keys (affine)
    int r0, off, L;
    bool last;            // this lane holds row RPL (adapter row L)
    int32_t k_go, k_ge, k_gex, k_vo, k_gev, k_geh, neg2;
    int32_t gdiag;        // row r0's G key at the previous column (the first row's diagonal source)
    int32_t bkey;         // last lane: row-L scout of the inner columns (LanePacked::column_tail)
    int bj;
    int bscore, bi, blt, btrail, bprec;
    uint32_t battr;
    int slt_last, ht_last, hp_last;
    int32_t gbot, vbot;   // bottom row keys of the last column computed (sent to lane l + 1)
    SplitIn out;          // after the last column: what lane l + 1 needs

    PCABI_HD void init(int lane, int K, int L_, int RPL, const Scoring &sc) {
        r0 = lane * R;
        off = RPL - L_;
        L = L_;
        last = lane == K - 1;
        const int32_t neg = Y::sc(pk::neg_score(sc));
        k_go = Y::sc(sc.go);
        k_ge = Y::sc(sc.ge);
        k_gev = Y::sc(sc.ge) - Y::sc(sc.go) + Y::TB2;
        k_geh = Y::sc(sc.ge) - Y::sc(sc.go) + Y::TB1;
        k_gex = Y::sc(sc.ge) + (Y::TAGGED ? Y::TB1 : 0);
        k_vo = Y::TAGGED ? Y::TB2 : 0;
#pragma unroll
        for (int s = 1; s <= R; ++s) {
            G[s] = Y::start(off - (r0 + s)) + k_go;   // padded (s, 0) reaches real (0, off - s)
            HK[s] = Y::TAGGED ? neg : (neg | Y::TB1);
        }
        neg2 = neg | Y::TB2;
        gdiag = Y::start(off - r0) + k_go;            // row r0 at column 0 (row 0 for lane 0)
        bkey = Y::start(-L_);                         // the (L, 0) seed
        bj = 0;
        gbot = G[R];
        vbot = neg2;
    }

    PCABI_HD int32_t row0_g(int j) const { return Y::start(j + off) + k_go; }   // G(0, j)

    // one row's candidates (LanePacked::column's recurrences)
    PCABI_HD void cell(int s, int32_t diag, int32_t gup, int32_t vup, int32_t &hn, int32_t &vn2, int32_t &sn,
                       bool &hext, bool &vext) const {
        if (AFFINE && Y::TAGGED) {
            const int32_t hx = HK[s] + k_gex, ho = G[s];
            hn = hx > ho ? hx : ho;
            const int32_t vx = vup + k_gex, vo = gup + k_vo;
            vn2 = vx > vo ? vx : vo;
            hext = Y::tb(hn) != 0;
            vext = Y::tb(vn2) > (Y::TB2 >> Y::TB_SH);
        } else if (AFFINE) {
            const int32_t hx = HK[s] + k_ge, ho = G[s];
            hn = hx > ho ? hx : ho;
            const int32_t vx = vup + k_ge, vo = gup;
            const int32_t vn = vx > vo ? vx : vo;
            vn2 = vn | Y::TB2;
            hext = Y::tb(hn) == 1;
            vext = Y::tb(vn) == 2;
        } else {
            vn2 = gup + k_gev;
            hn = G[s] + k_geh;
            hext = vext = false;
        }
        sn = max3i(diag, vn2, hn);
    }

    // inner column j (1 <= j < n); gup / vup: row r0's G / V keys at column j. owned == false (a
    // chunk's lead-in columns, LanePacked::column's GATE): the column cannot become the row-L best
    template <typename TabRow>
    PCABI_HD void inner(const TabRow &tab, int j, int32_t gup, int32_t vup, bool owned = true) {
        const int32_t g_in = gup;
        int32_t diag = gdiag + tab(1);
        int32_t lv = 0, ls = 0;
#pragma unroll
        for (int s = 1; s <= R; ++s) {
            int32_t diag_nx = 0;
            if (s < R) diag_nx = G[s] + tab(s + 1);
            int32_t hn, vn2, sn;
            bool hext, vext;
            cell(s, diag, gup, vup, hn, vn2, sn, hext, vext);
            if (s == R) { lv = vn2; ls = sn; }
            G[s] = (sn & ~Y::TBM) + k_go;
            if (AFFINE) HK[s] = Y::TAGGED ? hn : (hn | Y::TB1);
            gup = G[s];
            vup = vn2;
            diag = diag_nx;
        }
        gdiag = g_in;
        gbot = G[R];
        vbot = vup;
        // row-L scout (meaningful in the last lane only): LanePacked::column_tail
        int32_t corr;
        if (AFFINE && Y::TAGGED) corr = std::max(lv, ls & ~Y::TBM);
        else if (AFFINE) corr = std::max(lv | Y::TB3, ls & ~Y::TBM);
        else corr = ls;
        const bool upd = owned && corr > (bkey | ((1 << Y::SC_SH) - 1));
        bkey = upd ? corr : bkey;
        bj = upd ? j : bj;
    }

    // A chunk that ends before the read end (its last column ran as an inner column): the last
    // lane's row-L best from the scout (LanePacked::materialize); result(n + 1) then reports it.
    PCABI_HD void materialize() {
        if (!last) return;
        const int t = Y::tb(bkey);
        int lt;
        if (bj == 0) lt = LT_NONE;
        else if (AFFINE) lt = (Y::TAGGED ? t != 0 : t == 3) ? LT_V : LT_D;
        else lt = t == 3 ? LT_D : (t == 2 ? LT_V : LT_H);
        bscore = Y::score(bkey);
        bi = L;
        battr = Y::attr(bkey);
        blt = lt;
        btrail = 0;
        bprec = 0;
    }

    // the last column (j = n) of this lane's rows, after lane l - 1's part of it (`in`; lane 0:
    // row 0 -- empty_in())
    PCABI_HD SplitIn empty_in(int n) const {
        SplitIn e;
        e.gup = row0_g(n);
        e.vup = neg2;
        e.slt = LT_NONE;
        e.vt = e.vp = 0;
        e.score = (int)0x80000000;
        e.bi = e.lt = e.trail = e.prec = 0;
        e.attr = 0;
        return e;
    }

    template <typename TabRow>
    PCABI_HD void last_col(const TabRow &tab, int n, const SplitIn &in) {
        if (last) {
            // the row-L best of the inner columns (LanePacked::materialize), then B2
            const int t = Y::tb(bkey);
            int lt;
            if (bj == 0) lt = LT_NONE;
            else if (AFFINE) lt = (Y::TAGGED ? t != 0 : t == 3) ? LT_V : LT_D;
            else lt = t == 3 ? LT_D : (t == 2 ? LT_V : LT_H);
            bscore = Y::score(bkey);
            bi = L;
            battr = Y::attr(bkey);
            blt = lt;
            btrail = 0;
            bprec = 0;
            slt_last = LT_NONE;
            ht_last = 0;
            hp_last = 0;
            if (in.score > bscore) {
                bscore = in.score; bi = in.bi; bj = n; battr = in.attr; blt = in.lt; btrail = in.trail; bprec = in.prec;
            }
        } else {
            bscore = in.score; bi = in.bi; bj = n; battr = in.attr; blt = in.lt; btrail = in.trail; bprec = in.prec;
        }
        int32_t gup = in.gup, vup = in.vup;
        int slt_up = in.slt, vt_up = in.vt, vp_up = in.vp;
        int32_t diag = gdiag + tab(1);
        int32_t lv = 0, lh = 0, ls = 0;
        int lslt = LT_D;
        bool lhext = false;
#pragma unroll
        for (int s = 1; s <= R; ++s) {
            int32_t diag_nx = 0;
            if (s < R) diag_nx = G[s] + tab(s + 1);
            int32_t hn, vn2, sn;
            bool hext, vext;
            cell(s, diag, gup, vup, hn, vn2, sn, hext, vext);
            const int t = Y::tb(sn);
            const int slt = Y::TAGGED ? (t == (Y::TBM >> Y::TB_SH) ? LT_D : (t >= (Y::TB2 >> Y::TB_SH) ? LT_V : LT_H))
                                      : (t == 3 ? LT_D : (t == 2 ? LT_V : LT_H));
            const bool cont = AFFINE ? (vext || slt_up == LT_V) : (slt_up == LT_V);
            const int vt = cont ? vt_up + 1 : 1;
            const int vp = cont ? vp_up : (slt_up == LT_D ? 1 : 0);
            if (s < R || !last) {
                // a column-n row above row L: the scout, strict '>'
                const int sc_s = Y::score(sn);
                if (sc_s > bscore) {
                    bscore = sc_s;
                    bi = r0 + s - off;
                    bj = n;
                    if (AFFINE) {
                        const bool isv = Y::score(vn2) == sc_s, ish = !isv && Y::score(hn) == sc_s;
                        battr = Y::attr(isv ? vn2 : (ish ? hn : sn));
                        blt = isv ? LT_V : (ish ? LT_H : LT_D);
                        btrail = isv ? vt : 0;
                        bprec = isv ? vp : 0;
                    } else {
                        battr = Y::attr(sn);
                        blt = slt;
                        btrail = (slt == LT_V) ? vt : 0;
                        bprec = (slt == LT_V) ? vp : 0;
                    }
                }
                if (AFFINE) { vt_up = vt; vp_up = vp; }
                else { vt_up = (slt == LT_V) ? vt : 0; vp_up = (slt == LT_V) ? vp : 0; }
                slt_up = slt;
            } else {
                // row L (last lane): its cell is scouted below with the trailing runs
                lv = vn2; lh = hn; ls = sn; lslt = slt; lhext = hext;
                vt_up = vt;
                vp_up = vp;
            }
            G[s] = (sn & ~Y::TBM) + k_go;
            if (AFFINE) HK[s] = Y::TAGGED ? hn : (hn | Y::TB1);
            gup = G[s];
            vup = vn2;
            diag = diag_nx;
        }
        out.gup = gup; out.vup = vup;
        out.slt = slt_up; out.vt = vt_up; out.vp = vp_up;
        out.score = bscore; out.bi = bi; out.lt = blt; out.trail = btrail; out.prec = bprec; out.attr = battr;
        if (!last) return;
        // ---- row L, last column (LanePacked::column's tail) ----
        const bool hcont = AFFINE ? (lhext || slt_last == LT_H) : (slt_last == LT_H);
        const int ht = hcont ? ht_last + 1 : 1;
        const int hp = hcont ? hp_last : (slt_last == LT_D ? 1 : 0);
        const int lsc = Y::score(ls);
        const bool upd = lsc > bscore;
        int clt, ctrail, cprec;
        uint32_t cattr;
        if (AFFINE) {
            const bool isv = Y::score(lv) == lsc, ish = !isv && Y::score(lh) == lsc;
            cattr = Y::attr(isv ? lv : (ish ? lh : ls));
            clt = isv ? LT_V : (ish ? LT_H : LT_D);
            ctrail = isv ? vt_up : (ish ? ht : 0);
            cprec = isv ? vp_up : (ish ? hp : 0);
        } else {
            cattr = Y::attr(ls);
            clt = lslt;
            ctrail = (lslt == LT_V) ? vt_up : (lslt == LT_H ? ht : 0);
            cprec = (lslt == LT_V) ? vp_up : (lslt == LT_H ? hp : 0);
        }
        bscore = upd ? lsc : bscore;
        bi = upd ? L : bi;
        bj = upd ? n : bj;
        battr = upd ? cattr : battr;
        blt = upd ? clt : blt;
        btrail = upd ? ctrail : btrail;
        bprec = upd ? cprec : bprec;
    }

    PCABI_HD Result result(int n) const {
        Best b;
        b.score = bscore; b.bi = bi; b.bj = bj; b.attr = Y::to_std(battr, bj);
        b.ltype = blt; b.trail = btrail; b.precd = bprec;
        return finish(b, L, n);
    }
};

// Range conditions: a split bucket runs the packed (or run-tagged) layout of its RPL rows.
PCABI_HD bool split_ok(int rpl, int K) { return K >= 2 && rpl % K == 0 && rpl / K >= 2 && rpl <= 64; }

// ==========================================================================================
// Score-only filter for the middle-adapter scan.
//
// The scan only needs the alignments whose full-adapter identity reaches the threshold, and
// such an alignment must score high: pid2 = m / l2 >= theta with l2 >= L (the adapter span holds
// all L adapter bases) and every non-matching column of the span costs at most
// c = max(|mismatch|, |gap_open|, |gap_extend|), so the best score is at least
// L * (theta * match - c * (1 - theta))  (filter_threshold; the reported path never ends in a
// last-row H run, which would score below its own start). The filter computes the best score
// S* alone -- no tie-break, no attributes -- in 16-bit lanes, TWO adapters per lane
// (v_pk_add_u16 / v_pk_max_i16: 8 packed ops per row for two cells), and only the pairs at or
// above the bound go through the attribute DP. S* is the same value the full DP returns.
// ==========================================================================================
namespace sf {
typedef int16_t v2 __attribute__((vector_size(4)));
PCABI_HD v2 vmax(v2 a, v2 b) {
#if defined(__clang__)
    return __builtin_elementwise_max(a, b);
#else
    return a > b ? a : b;
#endif
}
PCABI_HD v2 splat(int x) { v2 r = {(int16_t)x, (int16_t)x}; return r; }
constexpr int NEG16 = -8192;
constexpr int MAX_RPL = 88;

// Smallest best score an alignment with pid2 >= threshold_pct can have (-32768: no bound).
// The threshold is lowered by 1e-5 % first: the reference compares the identity after its
// 6-decimal text round trip (pid6), which can round a value up by < 5e-7 %.
inline int filter_threshold(int L, double threshold_pct, const Scoring &sc) {
    const double th = (threshold_pct - 1e-5) / 100.0;
    if (th <= 0.0 || sc.ma <= 0) return -32768;
    int c = -sc.mi;
    c = c > -sc.go ? c : -sc.go;
    c = c > -sc.ge ? c : -sc.ge;
    if (c < 0) c = 0;
    const double b = (double)L * (th * sc.ma - c * (1.0 - th));
    if (b <= 0.0) return -32768;
    return (int)b;   // floor: S* is an integer >= b
}

// Range: scores, the NEG sentinel and their sums stay inside int16 (and gaps cost something,
// for the pass-through padding rows).
PCABI_HD bool filter_ok(int rpl, const Scoring &s) {
    if (rpl > MAX_RPL || !(s.go < 0 && s.ge < 0)) return false;
    const int hi = rpl * (best_sub(s) > 0 ? best_sub(s) : 0);
    const int lo = rpl * (s.mi < 0 ? s.mi : 0) + 4 * (s.go < s.ge ? s.go : s.ge);
    return hi < 4000 && lo > -4000 && s.go > -2000 && s.ge > -2000;
}

// Chunks of a long read for the middle scan's candidate DP (align_lane_packed<.., CHUNK>), so a
// long read no longer serialises one lane over all its columns. Only alignments
// scoring >= T matter (a hit's full identity >= theta forces it), and such an alignment holds
// at most L diagonal columns and at most (L * match - T) / g inserted read bases (g = the
// cheapest gap column), so its read span is at most D columns (chunk_span). A chunk owns C
// consecutive end columns and starts D + 1 columns before the first of them:
//   * an owned cell whose true best score is >= T has that alignment inside the chunk, and the
//     chunk's own DP cannot do better there: its only extra alignments let the adapter head
//     hang off for free at the chunk start, and those reach the owned columns only with a span
//     > D, i.e. a score < T. Along the alignment's path every prefix is optimal in both DPs, so
//     the tie-break bits agree too: the chunk reports the same cell, score and attributes;
//   * an owned cell below T stays below T in the chunk.
// Merging the chunks in read order, the first with the largest score, is then the full DP's
// answer whenever that score is >= T (first maximum = the reference's strict '>' scan); below
// T the pair cannot hit either way.
struct Chunk {
    int start, len, own_lo, own_hi;   // read offset, columns, owned end columns [lo, hi) (hi -1: last chunk)
};

inline int chunk_span(int L, int T, const Scoring &sc) {   // D, or -1 when chunking does not apply
    const int g = std::min(-sc.go, -sc.ge);
    if (g <= 0 || T <= 0 || sc.ma <= 0 || L <= 0) return -1;
    return L + (L * best_sub(sc) - T + g - 1) / g + 2;
}

template <typename F>
inline void chunk_plan(int n, int D, int C, F &&emit) {
    for (int lo = 1; lo <= n; lo += C) {
        const int hi = lo + C;
        const int start = std::max(0, lo - 1 - D);
        if (hi > n) {
            emit(Chunk{start, n - start, lo - start, -1});
            break;
        }
        emit(Chunk{start, hi - 1 - start, lo - start, hi - start});
    }
}
}  // namespace sf

// tabfn(r) -> row(s) / row.quad(q, v2 *dst): per slot the packed (adapter A, adapter B)
// substitution score of read code r MINUS gap_open (it is added to G = S + gap_open); padding
// slots hold -gap_open (score 0). Returns S* of both adapters (lo = A, hi = B).
template <int RPL, bool AFFINE, typename ReadFn, typename TabFn>
PCABI_HD sf::v2 filter_lane(ReadFn &rd, int n, const TabFn &tabfn, const Scoring sc) {
    using sf::v2;
    const v2 go2 = sf::splat(sc.go), ge2 = sf::splat(sc.ge), lin2 = sf::splat(sc.ge - sc.go);
    v2 G[RPL + 1], H[RPL + 1];
#pragma unroll
    for (int s = 1; s <= RPL; ++s) { G[s] = go2; H[s] = sf::splat(sf::NEG16); }   // S(i, 0) = 0
    v2 best = sf::splat(0);                         // the (L, 0) seed
    constexpr int NQ = RPL / 4;
    int r = rd(1);
#pragma unroll 1
    for (int j = 1; j <= n; ++j) {
        const int rn = j < n ? rd(j + 1) : 0;
        const auto tab = tabfn(r);
        v2 t[RPL + 2];
#pragma unroll
        for (int q = 0; q <= 1 && q < NQ; ++q) tab.quad(q, t + 4 * q + 1);
        v2 gup = go2;                               // S(0, j) = 0
        v2 vup = sf::splat(sf::NEG16);
        v2 diag = go2 + t[1];                       // S(0, j - 1) = 0
#pragma unroll
        for (int s = 1; s <= RPL; ++s) {
            if ((s & 3) == 1) {
                const int q = (s - 1) / 4 + 2;
                if (q < NQ) tab.quad(q, t + 4 * q + 1);
            }
            v2 diag_nx = diag;
            if (s < RPL) diag_nx = G[s] + t[s + 1];
            v2 hn, vn;
            if (AFFINE) {
                hn = sf::vmax(H[s] + ge2, G[s]);
                vn = sf::vmax(vup + ge2, gup);
            } else {
                hn = G[s] + lin2;
                vn = gup + lin2;
            }
            const v2 sn = sf::vmax(sf::vmax(diag, vn), hn);
            G[s] = sn + go2;
            if (AFFINE) H[s] = hn;
            gup = G[s];
            vup = vn;
            diag = diag_nx;
        }
        best = sf::vmax(best, G[RPL] - go2);        // last row
        r = rn;
    }
    v2 cm = G[1];                                   // last column (padding rows hold 0)
#pragma unroll
    for (int s = 2; s <= RPL; ++s) cm = sf::vmax(cm, G[s]);
    return sf::vmax(best, cm - go2);
}

}  // namespace pcabi
