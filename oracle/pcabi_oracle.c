/*
 * pcabi_oracle.c -- CPU ORACLE (test infrastructure only; see pcabi_oracle.h).
 *
 * A straightforward restatement of what the reference computes for one (read, adapter)
 * pair, written from the reference sources, step by step:
 *
 *   1. Dna5 mapping ........ S/basic/alphabet_residue_tabs.h:113-140
 *   2. Unbanded DP, free end gaps on all four sides (AlignConfig<1,1,1,1>,
 *      porechop_abi/src/adapter_align.cpp:26-27), Gotoh affine recurrences
 *      (S/align/dp_formula_affine.h:66-125) or linear when open == extend
 *      (S/align/global_alignment_unbanded.h:213-221, S/align/dp_formula_linear.h:65-105);
 *      ties resolved by _maxScore "left unless left < right" (S/align/dp_formula.h:153-163).
 *   3. Max scout over the last row then the last column, strict '>'
 *      (S/align/dp_meta_info.h:187-216, S/align/dp_scout.h:175).
 *   4. Start correction of the trace value (S/align/dp_algorithm_impl.h:1170-1186).
 *   5. GapsLeft traceback with Gotoh run-to-open loops
 *      (S/align/dp_traceback_impl.h:197-370, 379-455, 497-548).
 *   6. Gapped rows -> ScoredAlignment fields (porechop_abi/src/alignment.cpp:6-110)
 *      and "%d,%d,%d,%d,%d,%f,%f" text (alignment.cpp:113-120).
 *
 * Full (n+1)x(l+1) matrices; O(n*l) memory, intended for checking, not speed.
 * (S/ = porechop_abi/include/seqan/ under /root/reference.)
 */
#include "pcabi_oracle.h"

#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* trace bits (our own encoding of SeqAn's TraceBitMap_ roles) */
enum { T_NONE = 0, T_D = 1, T_H = 2, T_HO = 4, T_V = 8, T_VO = 16, T_MAXV = 32, T_MAXH = 64 };

#define NEG (INT_MIN / 2) /* DPCellDefaultInfinity, S/align/dp_cell.h:144-145 */

static int dna5(unsigned char c) {
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': case 'U': case 'u': return 3;
    default: return 4;
    }
}
static const char DNA5_CHARS[5] = {'A', 'C', 'G', 'T', 'N'};

/* SeqAn String<Dna> (the ab-initio compatibility check): A C G T/U, anything else -> A */
static int dna4(unsigned char c) {
    int v = dna5(c);
    return v == 4 ? 0 : v;
}

/* DP + scout + GapsLeft traceback: the gapped rows SeqAn's Align holds after globalAlignment
 * with AlignConfig<1,1,1,1>. Returns the row length (0 and score INT_MIN for an empty input);
 * *rr_out / *ar_out are malloc'd. */
static int build_rows(const char *read, int n, const char *adapter, int l, int ma, int mi, int go, int ge,
                      int four, char **rr_out, char **ar_out, int *score_out) {
    *rr_out = *ar_out = NULL;
    if (n <= 0 || l <= 0) {            /* _isValidDPSettings: empty sequence -> no alignment */
        *score_out = INT_MIN;
        return 0;
    }
    const int affine = (go != ge);
    const size_t cells = (size_t)(l + 1) * (size_t)(n + 1);
    /* per-thread matrices, grown on demand and kept (fresh pages on every call cost more than
     * the DP); every cell read below is written first (row 0 / column 0 by the init loops) */
    static _Thread_local int *S, *H, *V;
    static _Thread_local unsigned char *T;
    static _Thread_local size_t cap_cells;
    if (cells > cap_cells) {
        free(S); free(H); free(V); free(T);
        S = (int *)malloc(cells * sizeof(int));
        H = (int *)malloc(cells * sizeof(int));
        V = (int *)malloc(cells * sizeof(int));
        T = (unsigned char *)malloc(cells);
        cap_cells = cells;
    }
    unsigned char *rc = (unsigned char *)malloc((size_t)n);
    unsigned char *ac = (unsigned char *)malloc((size_t)l);
    for (int j = 0; j < n; ++j) rc[j] = (unsigned char)(four ? dna4((unsigned char)read[j]) : dna5((unsigned char)read[j]));
    for (int i = 0; i < l; ++i) ac[i] = (unsigned char)(four ? dna4((unsigned char)adapter[i]) : dna5((unsigned char)adapter[i]));
/* column-major (the DP walks columns j, rows i inside): contiguous inner loop */
#define IDX(i, j) ((size_t)(j) * (size_t)(l + 1) + (size_t)(i))

    /* free end gaps: first row and column are RecursionDirectionZero */
    for (int j = 0; j <= n; ++j) { S[IDX(0, j)] = 0; H[IDX(0, j)] = NEG; V[IDX(0, j)] = NEG; T[IDX(0, j)] = T_NONE; }
    for (int i = 0; i <= l; ++i) { S[IDX(i, 0)] = 0; H[IDX(i, 0)] = NEG; V[IDX(i, 0)] = NEG; T[IDX(i, 0)] = T_NONE; }

    /* (selects written as masks: the same values, without data-dependent branches) */
    for (int j = 1; j <= n; ++j) {
        const int *Sp = S + IDX(0, j - 1), *Hp = H + IDX(0, j - 1);
        int *Sc = S + IDX(0, j), *Hc = H + IDX(0, j), *Vc = V + IDX(0, j);
        unsigned char *Tc = T + IDX(0, j);
        const unsigned char r = rc[j - 1];
        for (int i = 1; i <= l; ++i) {
            int sub = (r == ac[i - 1]) ? ma : mi;
            int diag = Sp[i - 1] + sub;
            unsigned char tv;
            int s;
            if (affine) {
                int hx = Hp[i] + ge, ho = Sp[i] + go;
                int hopen = hx < ho;
                int h = hopen ? ho : hx;
                unsigned char hb = (unsigned char)(hopen ? T_HO : T_H);
                int vx = Vc[i - 1] + ge, vo = Sc[i - 1] + go;
                int vopen = vx < vo;
                int v = vopen ? vo : vx;
                unsigned char vb = (unsigned char)(vopen ? T_VO : T_V);
                int fromh = v < h;
                int g = fromh ? h : v;
                unsigned char gb = (unsigned char)(fromh ? T_MAXH : T_MAXV);
                int notd = diag < g;
                s = notd ? g : diag;
                tv = (unsigned char)((notd ? gb : T_D) | hb | vb);
                Hc[i] = h;
                Vc[i] = v;
            } else {
                int v = Sc[i - 1] + ge, h = Sp[i] + ge;
                int fromh = v < h;
                int g = fromh ? h : v;
                unsigned char gb = (unsigned char)(fromh ? (T_H | T_MAXH) : (T_V | T_MAXV));
                int notd = diag < g;
                s = notd ? g : diag;
                tv = notd ? gb : (unsigned char)T_D;
                Hc[i] = NEG;
                Vc[i] = NEG;
            }
            Sc[i] = s;
            Tc[i] = tv;
        }
    }

    /* scout: last row j = 0..n-1, then last column rows 0..l; strict '>' */
    int best = NEG, bi = 0, bj = 0;
    for (int j = 0; j < n; ++j)
        if (S[IDX(l, j)] > best) { best = S[IDX(l, j)]; bi = l; bj = j; }
    for (int i = 0; i <= l; ++i)
        if (S[IDX(i, n)] > best) { best = S[IDX(i, n)]; bi = i; bj = n; }
    *score_out = best;

    /* traceback (GapsLeft). path columns are collected in reverse: type 'D','V','H' */
    char *path = (char *)malloc((size_t)(n + l + 2));
    int plen = 0;
    int i = bi, j = bj;
    if (i > 0 && j > 0) {
        unsigned char tv = T[IDX(i, j)];
        if (affine) {
            if (V[IDX(i, j)] == best)      { tv = (unsigned char)((tv & ~T_D) | T_MAXV); }
            else if (H[IDX(i, j)] == best) { tv = (unsigned char)((tv & ~T_D) | T_MAXH); }
        }
        while (i > 0 && j > 0 && tv != T_NONE) {
            if (tv & T_D) {
                path[plen++] = 'D';
                --i; --j;
                tv = T[IDX(i, j)];
            } else if ((tv & T_MAXV) && (tv & T_V)) {
                if (affine) {
                    while ((!(tv & T_VO) || (tv & T_V)) && i != 1) {
                        path[plen++] = 'V';
                        --i;
                        tv = T[IDX(i, j)];
                    }
                }
                path[plen++] = 'V';
                --i;
                tv = T[IDX(i, j)];
            } else if ((tv & T_MAXV) && (tv & T_VO)) {
                path[plen++] = 'V';
                --i;
                tv = T[IDX(i, j)];
            } else if ((tv & T_MAXH) && (tv & T_H)) {
                if (affine) {
                    while ((!(tv & T_HO) || (tv & T_H)) && j != 1) {
                        path[plen++] = 'H';
                        --j;
                        tv = T[IDX(i, j)];
                    }
                }
                path[plen++] = 'H';
                --j;
                tv = T[IDX(i, j)];
            } else if ((tv & T_MAXH) && (tv & T_HO)) {
                path[plen++] = 'H';
                --j;
                tv = T[IDX(i, j)];
            } else {
                break; /* NONE */
            }
        }
    }
    const int i0 = i, j0 = j;

    /* gapped rows: head + path + tail (S/align/dp_traceback_impl.h:523-545) */
    const int cap = n + l + 2;
    char *rr = (char *)malloc((size_t)cap);
    char *ar = (char *)malloc((size_t)cap);
    int len = 0;
    if (i0 != 0) {
        for (int k = 0; k < i0; ++k) { rr[len] = '-'; ar[len] = DNA5_CHARS[ac[k]]; ++len; }
    } else if (j0 != 0) {
        for (int k = 0; k < j0; ++k) { rr[len] = DNA5_CHARS[rc[k]]; ar[len] = '-'; ++len; }
    }
    {
        int ci = i0, cj = j0;
        for (int k = plen - 1; k >= 0; --k) {
            if (path[k] == 'D') { rr[len] = DNA5_CHARS[rc[cj]]; ar[len] = DNA5_CHARS[ac[ci]]; ++ci; ++cj; }
            else if (path[k] == 'V') { rr[len] = '-'; ar[len] = DNA5_CHARS[ac[ci]]; ++ci; }
            else { rr[len] = DNA5_CHARS[rc[cj]]; ar[len] = '-'; ++cj; }
            ++len;
        }
    }
    if (bi != l) {
        for (int k = bi; k < l; ++k) { rr[len] = '-'; ar[len] = DNA5_CHARS[ac[k]]; ++len; }
    }
    if (bj != n) {
        for (int k = bj; k < n; ++k) { rr[len] = DNA5_CHARS[rc[k]]; ar[len] = '-'; ++len; }
    }

    free(path);
    free(rc); free(ac);
#undef IDX
    *rr_out = rr;
    *ar_out = ar;
    return len;
}

void pcabi_oracle_align(const char *read, int n, const char *adapter, int l,
                        int ma, int mi, int go, int ge, pcabi_oracle_result *out) {
    memset(out, 0, sizeof(*out));
    out->rs = -1;
    out->re = -1;
    out->as = -1;
    out->ae = -1;
    char *rr, *ar;
    const int len = build_rows(read, n, adapter, l, ma, mi, go, ge, 0, &rr, &ar, &out->score);
    if (len == 0) return;
    /* ScoredAlignment (porechop_abi/src/alignment.cpp:27-109) */
    int st = -1, en = -1, a0 = -1, a1 = -1;
    { int r = 0, a = 0;
      for (int c = 0; c < len; ++c) { if (rr[c] != '-') r = 1; if (ar[c] != '-') a = 1; if (r && a) { st = c; break; } } }
    { int r = 0, a = 0;
      for (int c = len - 1; c >= 0; --c) { if (rr[c] != '-') r = 1; if (ar[c] != '-') a = 1; if (r && a) { en = c; break; } } }
    if (st >= 0 && en >= 0) {
        for (int c = 0; c < len; ++c) if (ar[c] != '-') { a0 = c; break; }
        for (int c = len - 1; c >= 0; --c) if (ar[c] != '-') { a1 = c; break; }
        int m1 = 0, m2 = 0;
        for (int c = st; c < en + 1; ++c) if (ar[c] == rr[c]) ++m1;
        for (int c = a0; c < a1 + 1; ++c) if (ar[c] == rr[c]) ++m2;
        int rb = 0, ab = 0;
        for (int c = 0; c < len; ++c) {
            if (c == st) { out->rs = rb; out->as = ab; }
            if (c == en) { out->re = rb; out->ae = ab; }
            if (rr[c] != '-') ++rb;
            if (ar[c] != '-') ++ab;
        }
        /* both identity numerators are the same set of D-match columns;
         * keep them separate here so the restatement stays literal. */
        out->m = m1;
        out->l1 = en - st + 1;
        out->l2 = a1 - a0 + 1;
        if (m1 != m2) out->m = -1000000 - m2; /* never happens; flags a broken assumption */
    }
    free(rr); free(ar);
}

/* check_compatibility (porechop_abi/ab_initio_src/compatibility.cpp:17-170), literally: the
 * longer sequence is row 0 (ties: seq1), String<Dna>, Score(2, -1, -1) linear, the aligned
 * region [st, en] of the gapped rows, distance = mismatching columns on [st, en), integer
 * identity (mapped - distance) * 100 / mapped >= 87.5, inclusion when row 0's region starts or
 * ends more than 3 bases inside it. Returns -1 where the reference divides by zero (no
 * overlap) or has no alignment (an empty sequence). */
int pcabi_oracle_compat(const char *s1, const char *s2) {
    const int n1 = (int)strlen(s1), n2 = (int)strlen(s2);
    const char *a = s1, *b = s2;
    int na = n1, nb = n2;
    if (n1 < n2) { a = s2; b = s1; na = n2; nb = n1; }
    char *rr, *ar;
    int score;
    const int len = build_rows(a, na, b, nb, 2, -1, -1, -1, 1, &rr, &ar, &score);
    if (len == 0) return -1;
    int st = -1, en = -1;
    { int r = 0, q = 0;
      for (int c = 0; c < len; ++c) { if (rr[c] != '-') r = 1; if (ar[c] != '-') q = 1; if (r && q) { st = c; break; } } }
    { int r = 0, q = 0;
      for (int c = len - 1; c >= 0; --c) { if (rr[c] != '-') r = 1; if (ar[c] != '-') q = 1; if (r && q) { en = c; break; } } }
    const int mapped = en - st + 1;
    int flag = -1;
    if (st >= 0 && en >= 0 && mapped > 0) {
        int dist = 0;
        for (int c = st; c < en; ++c) if (rr[c] != ar[c]) ++dist;
        int s1_start = 0, s1_end = 0, rb = 0;
        for (int c = 0; c < len; ++c) {
            if (c == st) s1_start = rb;
            if (c == en) s1_end = rb;
            if (rr[c] != '-') ++rb;
        }
        const float identity = (float)((mapped - dist) * 100 / mapped);
        const int included = s1_start > 3 || (na - s1_end) > 3;
        flag = identity >= 87.5f ? 1 : 0;
        if (included && flag == 1) flag = 2;
    }
    free(rr); free(ar);
    return flag;
}

static int fmt_pid(char *buf, size_t cap, int m, int l) {
    if (l == 0) return snprintf(buf, cap, "-nan"); /* 0.0/0 on x86-64 is the negative default NaN */
    double d = 100.0 * m / l;
    return snprintf(buf, cap, "%f", d);
}

char *pcabi_oracle_adapter_alignment(const char *read, const char *adapter,
                                     int ma, int mi, int go, int ge) {
    pcabi_oracle_result r;
    pcabi_oracle_align(read, (int)strlen(read), adapter, (int)strlen(adapter), ma, mi, go, ge, &r);
    char p1[64], p2[64];
    char *s = (char *)malloc(256);
    if (r.rs == -1) {
        /* reference leaves the remaining fields uninitialised; only field 0 is defined */
        snprintf(s, 256, "-1,0,-1,0,%d,0.000000,0.000000", r.score);
        return s;
    }
    fmt_pid(p1, sizeof p1, r.m, r.l1);
    fmt_pid(p2, sizeof p2, r.m, r.l2);
    snprintf(s, 256, "%d,%d,%d,%d,%d,%s,%s", r.rs, r.re, r.as, r.ae, r.score, p1, p2);
    return s;
}

void pcabi_oracle_free(char *p) { free(p); }

void pcabi_oracle_align_batch(const char *reads, const long long *read_off, const int *read_len,
                              const char *adapters, const int *adp_off, const int *adp_len,
                              const int *adp_idx, long long n_pairs,
                              int ma, int mi, int go, int ge, int *results) {
    for (long long p = 0; p < n_pairs; ++p) {
        pcabi_oracle_result r;
        int a = adp_idx[p];
        pcabi_oracle_align(reads + read_off[p], read_len[p], adapters + adp_off[a], adp_len[a],
                           ma, mi, go, ge, &r);
        int *o = results + 8 * p;
        o[0] = r.rs; o[1] = r.re; o[2] = r.as; o[3] = r.ae;
        o[4] = r.score; o[5] = r.m; o[6] = r.l1; o[7] = r.l2;
    }
}

/* find_middle_adapters' masked re-alignment loop (porechop_abi/nanopore_read.py:236-246), per
 * read: for each adapter in order, align the (masked) read; while the full-adapter identity
 * (the reference's "%f" text parsed back, nanopore_read.py:497-498) is not below the threshold,
 * record the hit and mask its aligned read bases with '-' (which SeqAn's Dna5 reads as N).
 * Reads are spread over n_threads threads. Hits come out per read in discovery order, reads in
 * order: rows (read, adapter, read_start, read_end_exclusive, m, l2), row-major out[6][cap].
 * Returns the number of hits (only the first cap are written). */
#include <pthread.h>
#include <stdlib.h>

typedef struct {
    int *v;
    long long n, cap;
} ivec;

static void ivec_push6(ivec *x, const int *six) {
    if (x->n + 6 > x->cap) {
        x->cap = x->cap ? 2 * x->cap : 64;
        x->v = (int *)realloc(x->v, sizeof(int) * (size_t)x->cap);
    }
    memcpy(x->v + x->n, six, 6 * sizeof(int));
    x->n += 6;
}

typedef struct {
    const char *reads, *adapters;
    const long long *read_off;
    const int *read_len, *adp_off, *adp_len;
    long long n_reads;
    int n_adp, ma, mi, go, ge, stride, first;
    double threshold;
    ivec *per_read;
} middle_job;

static double text_identity(int m, int l) {
    char buf[64];
    if (l == 0) return 0.0 / 0.0;
    snprintf(buf, sizeof buf, "%f", 100.0 * m / l);
    return strtod(buf, NULL);
}

static void *middle_worker(void *arg) {
    const middle_job *J = (const middle_job *)arg;
    for (long long w = J->first; w < J->n_reads; w += J->stride) {
        const int n = J->read_len[w];
        char *masked = (char *)malloc((size_t)n + 1);
        memcpy(masked, J->reads + J->read_off[w], (size_t)n);
        masked[n] = 0;
        for (int a = 0; a < J->n_adp; ++a) {
            for (;;) {
                pcabi_oracle_result r;
                pcabi_oracle_align(masked, n, J->adapters + J->adp_off[a], J->adp_len[a], J->ma, J->mi, J->go,
                                   J->ge, &r);
                const double full = r.rs == -1 ? 0.0 : text_identity(r.m, r.l2);
                if (!(full >= J->threshold)) break;   /* NaN never hits (l2 > 0 whenever rs >= 0) */
                const int rs = r.rs, rend = r.rs == -1 ? 0 : r.re + 1;
                for (int k = rs; k < rend; ++k) masked[k] = '-';
                const int six[6] = {(int)w, a, rs, rend, r.m, r.l2};
                ivec_push6(&J->per_read[w], six);
            }
        }
        free(masked);
    }
    return NULL;
}

long long pcabi_oracle_middle_scan(const char *reads, const long long *read_off, const int *read_len,
                                   long long n_reads, const char *adapters, const int *adp_off, const int *adp_len,
                                   int n_adp, int ma, int mi, int go, int ge, double threshold, int n_threads,
                                   int *out, long long cap) {
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 64) n_threads = 64;
    ivec *per_read = (ivec *)calloc((size_t)(n_reads > 0 ? n_reads : 1), sizeof(ivec));
    middle_job jobs[64];
    pthread_t th[64];
    for (int t = 0; t < n_threads; ++t) {
        jobs[t] = (middle_job){reads, adapters, read_off, read_len, adp_off, adp_len, n_reads, n_adp, ma, mi, go, ge,
                               n_threads, t, threshold, per_read};
        pthread_create(&th[t], NULL, middle_worker, &jobs[t]);
    }
    for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
    long long h = 0;
    for (long long w = 0; w < n_reads; ++w) {
        for (long long k = 0; k < per_read[w].n; k += 6, ++h)
            if (h < cap)
                for (int f = 0; f < 6; ++f) out[f * cap + h] = per_read[w].v[k + f];
        free(per_read[w].v);
    }
    free(per_read);
    return h;
}
