/*
 * pcabi.h -- C ABI of the MI355X adapter-alignment engine (libpcabi.so).
 *
 * Two layers:
 *
 *  1. Drop-in legacy symbols, byte-compatible with the reference's cpp_functions.so
 *     (porechop_abi/include/adapter_align.h:12-16, bound by ctypes in
 *     porechop_abi/cpp_function_wrappers.py:25-39):
 *        char *adapterAlignment(char *readSeq, char *adapterSeq,
 *                               int matchScore, int mismatchScore,
 *                               int gapOpenScore, int gapExtensionScore);
 *        void  freeCString(char *p);
 *     Same argument order (Python passes match, mismatch, gap_open, gap_extend:
 *     cpp_function_wrappers.py:46-51), same malloc'd "rs,re,as,ae,score,pid1,pid2" result
 *     (porechop_abi/src/alignment.cpp:113-120), caller frees with freeCString. Each call runs
 *     on the GPU (one lane); concurrent callers are serialised per device.
 *
 *  2. Batch ABI used by the batched phase drivers (replacing the per-read ThreadPool loops of
 *     porechop_abi/porechop_abi.py:200-245, 359-438, 457-522). Sequences are Dna5 codes
 *     (A=0 C=1 G=2 T/U=3 anything else=4, S/basic/alphabet_residue_tabs.h:113-140) packed in
 *     one byte buffer; a "window" is an (offset, length) view into it (any offset), the
 *     buffer padded with >= 16 readable bytes past the last window. Results are SoA int32,
 *     8 fields x n_results, field order PCABI_F_*.
 *
 * Errors: functions return 0 on success, a negative PCABI_E_* code otherwise;
 * pcabi_last_error() returns a thread-local message. No exceptions cross the ABI.
 * There is no CPU fallback: without a usable gfx950 device every compute entry point fails.
 * The two drop-in symbols have no error channel (the reference's never fail on valid input):
 * when the engine fails under them they print pcabi_last_error() to stderr and abort() rather
 * than return an answer the reference would not give (adapterAlignment's "-1" sentinel would read
 * as "no alignment" and silently change trimming decisions). Empty inputs keep the reference's
 * "-1" result.
 *
 * Lengths: windows / reads of any length up to pcabi_max_window_len(); adapters (and the
 * shorter sequence of a check_compatibility pair) up to pcabi_max_adapter_len() = 65535 bases.
 * Adapters up to 128 bases run register-resident cores; longer ones the striped core
 * (row stripes of 32, the boundary row in stream-ordered device scratch).
 */
#ifndef PCABI_H
#define PCABI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- result field order (SoA rows) -------------------------------------------------- */
enum {
    PCABI_F_RS = 0,     /* read start (ScoredAlignment::m_readStartPos), -1 = no alignment */
    PCABI_F_RE = 1,     /* read end, inclusive                                          */
    PCABI_F_AS = 2,     /* adapter start                                                */
    PCABI_F_AE = 3,     /* adapter end, inclusive                                       */
    PCABI_F_SCORE = 4,  /* raw DP score                                                 */
    PCABI_F_M = 5,      /* matching columns (numerator of both identities)              */
    PCABI_F_L1 = 6,     /* aligned-region length: pid1 = 100*m/l1 (NaN when l1 == 0)     */
    PCABI_F_L2 = 7,     /* full-adapter span length: pid2 = 100*m/l2                     */
    PCABI_NFIELDS = 8
};

enum {
    PCABI_OK = 0,
    PCABI_E_ARG = -1,      /* bad argument / unsupported size                   */
    PCABI_E_DEVICE = -2,   /* no usable gfx950 device / HIP runtime error       */
    PCABI_E_NOMEM = -3,
    PCABI_E_PARSE = -4     /* malformed FASTA / FASTQ input                     */
};

/* ---- legacy drop-in ------------------------------------------------------------------ */
char *adapterAlignment(char *readSeq, char *adapterSeq, int matchScore, int mismatchScore,
                       int gapOpenScore, int gapExtensionScore);
void freeCString(char *p);

/* ---- housekeeping -------------------------------------------------------------------- */
const char *pcabi_last_error(void);
int pcabi_version(void);                 /* ABI version, currently 1                     */
int pcabi_device_count(void);            /* visible HIP devices (0 if none)              */
int pcabi_max_adapter_len(void);         /* longest adapter the kernels accept (65535)   */
int pcabi_max_window_len(void);          /* longest window / read the kernels accept     */

/* ASCII -> Dna5 codes (host, table lookup). n bytes. */
void pcabi_encode_dna5(const char *ascii, uint8_t *codes, int64_t n);
/* Gathered ASCII -> Dna5 (host, up to 16 threads): codes[dst_off[i] .. + len[i]) = the codes of
 * the len[i] bytes at address src[i]; every byte of codes[0 .. codes_len) outside those segments
 * is set to N (4). dst_off ascending, segments disjoint. The Python drivers pass the addresses of
 * the reads' own str buffers, so windows of 10^5 reads are packed without a slice, a join or an
 * encode (replaces the per-read seq[:end_size] / seq[-end_size:] / trimmed-read slices that
 * nanopore_read.py:181, 203 and porechop_abi.py:495 hand to SeqAn's marshalling). */
void pcabi_encode_dna5_gather(const uint64_t *src, const int64_t *len, const int64_t *dst_off, int64_t n,
                              uint8_t *codes, int64_t codes_len);

/* Identity exactly as Python holds it after the reference's text round trip
 * (alignment.cpp:118-119 "%f", nanopore_read.py:497-498 float()): out[k] = pid6(m[k], l[k]),
 * NaN when l[k] == 0. Host-side formatting helper, same code as the device epilogues. */
void pcabi_pid6_host(const int32_t *m, const int32_t *l, int64_t n, double *out);

/* ---- batch alignment, host buffers ---------------------------------------------------- */
/*
 * Align windows against adapters on `device`.
 *   codes[codes_len]            : Dna5 codes holding every window (padding rules above)
 *   win_off[n_win], win_len[n_win]
 *   adp_codes, adp_off[n_adp], adp_len[n_adp] : adapters (Dna5 codes, any alignment)
 * Work:
 *   task_win == NULL  -> cross product: result (a, w) at index a*n_win + w
 *   task_win != NULL  -> n_task explicit pairs (task_win[t], task_adp[t]); result at index t
 * out: int32[PCABI_NFIELDS * n_results], row f holds field f for every result.
 */
int pcabi_align_host(int device,
                     const uint8_t *codes, int64_t codes_len,
                     const int64_t *win_off, const int32_t *win_len, int64_t n_win,
                     const uint8_t *adp_codes, const int32_t *adp_off, const int32_t *adp_len,
                     int32_t n_adp,
                     const int32_t *task_win, const int32_t *task_adp, int64_t n_task,
                     int match, int mismatch, int gap_open, int gap_extend,
                     int32_t *out);

/* ---- device-resident interface (bench / multi-GPU shards) ------------------------------ */
/* Thin HIP wrappers so hosts without a GPU framework can keep inputs resident in HBM. */
int pcabi_dev_set(int device);
int pcabi_dev_malloc(void **ptr, int64_t bytes);
int pcabi_dev_free(void *ptr);
int pcabi_dev_h2d(void *dst, const void *src, int64_t bytes);
int pcabi_dev_d2h(void *dst, const void *src, int64_t bytes);
int pcabi_dev_memset(void *dst, int value, int64_t bytes);
int pcabi_dev_sync(void);
/* ordered on `stream`; kind 0 = host->device, 1 = device->host, 2 = device->device */
int pcabi_dev_copy_async(void *dst, const void *src, int64_t bytes, int kind, void *stream);
int pcabi_stream_create(void **stream);
int pcabi_stream_destroy(void *stream);
int pcabi_stream_sync(void *stream);
int pcabi_event_create(void **ev);
int pcabi_event_destroy(void *ev);
int pcabi_event_record(void *ev, void *stream);
/* later work on `stream` waits for `ev` (recorded on another stream): fork / join of caller streams */
int pcabi_stream_wait_event(void *stream, void *ev);
int pcabi_event_elapsed_ms(float *ms, void *start, void *stop);

/*
 * Prepared adapter table: adapters re-laid out per register bucket (top-padded, packed codes).
 * Build once per adapter list; reuse across batches.
 */
typedef struct pcabi_adapters pcabi_adapters;
int pcabi_adapters_create(const uint8_t *adp_codes, const int32_t *adp_off, const int32_t *adp_len,
                          int32_t n_adp, pcabi_adapters **out);   /* uploads to current device */
/* Same, with small register buckets merged into larger ones for THIS scoring (fewer, fuller
 * launches; the packed core passes scores through the extra padding rows). The table then
 * serves that scoring only: pcabi_align_cross_dev rejects others. */
int pcabi_adapters_create_scored(const uint8_t *adp_codes, const int32_t *adp_off,
                                 const int32_t *adp_len, int32_t n_adp, int match, int mismatch,
                                 int gap_open, int gap_extend, pcabi_adapters **out);
void pcabi_adapters_destroy(pcabi_adapters *a);

/*
 * Tile layout of a window list, the form the cross-product kernels read:
 * windows [256t, 256t + 256) form tile t; dword (t, q, lane) holds codes 4q..4q+3 of window
 * 256t + lane at tiles[tile_off[t] + 256 q + lane], so a wavefront's load of one 4-column chunk
 * is 256 contiguous bytes. A tile holds ceil(longest window in it / 4) + 2 chunks; sort the
 * windows by length first when they vary (whole reads) to keep tiles dense.
 *   pcabi_tile_layout      : host; fills tile_off[ceil(n_win/256) + 1] (dword offsets) from the
 *                            host copy of win_len and returns the total dword count (< 0 on
 *                            error).
 *   pcabi_tile_windows_dev : device pointers, async on `stream`: writes `tiles` from windows
 *                            laid out as for pcabi_align_host (codes/win_off/win_len);
 *                            max_chunks = largest per-tile chunk count (a launch-shape hint).
 */
int64_t pcabi_tile_layout(const int32_t *win_len, int64_t n_win, int64_t *tile_off);
int pcabi_tile_windows_dev(const uint8_t *codes, const int64_t *win_off, const int32_t *win_len,
                           int64_t n_win, const int64_t *tile_off, int64_t max_chunks,
                           uint32_t *tiles, void *stream);

/*
 * Cross-product alignment, every pointer a DEVICE pointer, asynchronous on `stream`:
 * result (a, w) -> out[f * out_stride + a * n_win + w]. Windows come in tile layout (above);
 * win_len[n_win] is still passed per window. max_win_len (host value) bounds every win_len[w]
 * and must be honest: windows longer than 32k need negative gap costs (the start-column field
 * of the non-packed cores is kept mod 2^16).
 */
int pcabi_align_cross_dev(const uint32_t *tiles, const int64_t *tile_off, const int32_t *win_len,
                          int64_t n_win, int32_t max_win_len, const pcabi_adapters *adps,
                          int match, int mismatch, int gap_open, int gap_extend,
                          int32_t *out, int64_t out_stride, void *stream);
/* Same, and records ev_begin / ev_end (pcabi_event_create; either may be NULL) on `stream`
 * around the launch of the table's largest bucket (adapters x rows), which runs on `stream`
 * while the other buckets run beside it on the device's side streams: the events time that
 * kernel inside a full cross product (bench.py's roofline). */
int pcabi_align_cross_dev_marked(const uint32_t *tiles, const int64_t *tile_off, const int32_t *win_len,
                                 int64_t n_win, int32_t max_win_len, const pcabi_adapters *adps,
                                 int match, int mismatch, int gap_open, int gap_extend,
                                 int32_t *out, int64_t out_stride, void *stream, void *ev_begin,
                                 void *ev_end);
/* Several cross products in one call (r06): region k = (tiles, tile_off, win_len, n_win,
 * max_win_len, adps, out, out_stride) is aligned exactly as pcabi_align_cross_dev would align it
 * (same results, same layout), but the register buckets of ALL regions run as grouped launches: the
 * buckets of one core family -- the run-tagged core (affine, <= 32 rows) and the packed core (affine,
 * 36..64 rows) -- across every region share one launch each (pcabi_kern.h "grouped cross
 * launches"), the other buckets launch on their own. A bucket of one or two adapters (a 400-block
 * grid for 100k windows) is latency-bound alone; grouped with the others its waves fill the SIMDs.
 * The largest launch runs on `stream` (ev_begin / ev_end, either may be NULL, are recorded around
 * it), the others beside it on the side streams when they are on for `stream`. Replaces the
 * per-side calls of porechop_abi.py:359-438's end trim (both read ends in one call). */
typedef struct pcabi_cross_region {
    const uint32_t *tiles;
    const int64_t *tile_off;
    const int32_t *win_len;
    int64_t n_win;
    int32_t max_win_len;
    const pcabi_adapters *adps;
    int32_t *out;
    int64_t out_stride;
} pcabi_cross_region;
int pcabi_align_cross_multi_dev(const pcabi_cross_region *regions, int32_t n_regions, int match, int mismatch,
                                int gap_open, int gap_extend, void *stream, void *ev_begin, void *ev_end);
/* Side streams (process-wide): with on = 1 a cross product (and a middle-scan round) runs its
 * largest register bucket on the caller's stream and the others beside it on the device's side
 * streams; with on = 0 every bucket runs on the caller's stream, one after the other. Side by side
 * pays for ONE cross product at a time (the largest bucket's tail fills with the small ones);
 * callers that run cross products on several streams at once should turn it off: HIP maps the
 * process's streams onto GPU_MAX_HW_QUEUES hardware queues, and a side stream on the queue of
 * another caller stream's large launch waits for it (r04r: the reference job 4.95 -> 4.66 ms
 * off). Initially on. Returns the previous setting; on < 0 only reads it. */
int pcabi_set_side_streams(int on);
/* The same setting for one stream (r05): the cross products and middle-scan rounds queued on `stream`
 * use the side streams when on = 1 and run every bucket on `stream` when on = 0, whatever the
 * process-wide setting; on = -1 removes the stream's entry (it follows pcabi_set_side_streams again).
 * Returns the stream's previous entry (0 / 1) or -1 when it had none. Callers that run cross
 * products on several streams at once set 0 on those streams (r04r: the reference job 4.95 -> 4.66
 * ms), and no other caller of the library is affected. Destroying a stream does not remove its entry:
 * remove it first (a new stream may reuse the handle). */
int pcabi_stream_side_streams(void *stream, int on);

/*
 * End-trim decision epilogue (porechop_abi/nanopore_read.py:175-217), device pointers:
 *   start results: cross product of n_read start windows x n_sa start adapters (layout above)
 *   end results  : cross product of n_read end windows   x n_ea end adapters
 * Identities are compared exactly as the reference does after its text round trip
 * (alignment.cpp:118-119 prints "%f", nanopore_read.py:497-498 parses it back): the device
 * rounds 100*m/l to 6 decimals with round-half-even on the exact double, then to the nearest
 * double (pcabi::pid6, checked against Python's '%f' in tests/).
 * Writes start_trim[n_read], end_trim[n_read] (amounts, same integers as
 * NanoporeRead.start_trim_amount / end_trim_amount) and, when non-NULL, per-pair
 * "alignment recorded" flags (uint8, same layout as the results).
 */
int pcabi_end_trim_dev(const int32_t *start_res, int64_t start_stride, int32_t n_sa,
                       const int32_t *end_res, int64_t end_stride, int32_t n_ea,
                       int64_t n_read, int end_size, int extra_trim, double end_threshold, int min_trim_size,
                       int32_t *start_trim, int32_t *end_trim,
                       uint8_t *start_hit, uint8_t *end_hit, void *stream);

/*
 * The reads with their end adapters trimmed, on the device (nanopore_read.py:44-49,
 * get_seq_with_start_end_adapters_trimmed): view_off = read_off + start_trim, view_len =
 * max(read_len - start_trim - end_trim, 0) -- the middle scan's windows straight from
 * pcabi_end_trim_dev's amounts, with no host round trip. Async on `stream`.
 */
int pcabi_trim_views_dev(const int64_t *read_off, const int32_t *read_len, const int32_t *start_trim,
                         const int32_t *end_trim, int64_t n_read, int64_t *view_off, int32_t *view_len, void *stream);

/*
 * End-trim decisions with their alignment lists (porechop_abi/nanopore_read.py:175-217, the loop of
 * find_adapters_at_read_ends, porechop_abi.py:359-438) from HOST buffers, with only the decisions
 * coming back -- never the (read, adapter) result matrix:
 *   codes / s_off, s_len / e_off, e_len : start and end windows of n_read reads (layout of
 *                         pcabi_align_host: one buffer, any offsets, 16 bytes of padding)
 *   sa_* / ea_*         : start and end adapters (Dna5 codes)
 *   start_trim / end_trim[n_read] : NanoporeRead.start_trim_amount / end_trim_amount
 *   start_hits / end_hits : 7 rows x cap int32 -- every alignment find_start_trim / find_end_trim
 *                         record, read-major and in adapter order within a read (the order they
 *                         are appended): read, adapter, rs, re (inclusive), m, l1, l2 (full identity
 *                         = pid6(m, l2), partial = pid6(m, l1)); n_hits[2] receives the two counts,
 *                         and a side whose count exceeds cap is not written (call again, larger cap)
 *   bc_s[n_bc_s], bc_e[n_bc_e] : adapters whose full identity of every read the barcode dicts keep
 *                         (nanopore_read.py:193-195, 215-217); bc_full (double, (n_bc_s + n_bc_e) x
 *                         n_read, start adapters first) receives them when non-NULL
 * The prepared adapter tables are kept per device between calls with the same adapters and scoring.
 *   pcabi_flag_list_dev : the list of one side from device pointers (async on `stream`): flagged
 *                         pairs (k_end_trim's flags, layout of pcabi_end_trim_dev) of a result
 *                         block -> out (7 rows x cap, as above), *n_out (device uint64) = the count.
 */
int pcabi_end_decisions_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *s_off,
                             const int32_t *s_len, const int64_t *e_off, const int32_t *e_len, int64_t n_read,
                             const uint8_t *sa_codes, const int32_t *sa_off, const int32_t *sa_len, int32_t n_sa,
                             const uint8_t *ea_codes, const int32_t *ea_off, const int32_t *ea_len, int32_t n_ea,
                             int match, int mismatch, int gap_open, int gap_extend, int end_size, int extra_trim,
                             double end_threshold, int min_trim_size, int32_t *start_trim, int32_t *end_trim,
                             int32_t *start_hits, int32_t *end_hits, int64_t cap, int64_t *n_hits,
                             const int32_t *bc_s, int32_t n_bc_s, const int32_t *bc_e, int32_t n_bc_e,
                             double *bc_full);
/*
 * pcabi_end_decisions_seqs: the same decisions from the window STRINGS (the reference's
 * seq[:end_size] / seq[-end_size:] slices, nanopore_read.py:181, 203, never made): win[2 n_read]
 * the address of each window's first character (ASCII, one byte per base -- start windows, then
 * end windows), win_len[2 n_read] its length. The library lays them out as pcabi_end_decisions_host's
 * buffer and encodes them itself into pinned staging buffers while earlier chunks copy.
 */
int pcabi_end_decisions_seqs(int device, const char *const *win, const int32_t *win_len, int64_t n_read,
                             const uint8_t *sa_codes, const int32_t *sa_off, const int32_t *sa_len, int32_t n_sa,
                             const uint8_t *ea_codes, const int32_t *ea_off, const int32_t *ea_len, int32_t n_ea,
                             int match, int mismatch, int gap_open, int gap_extend, int end_size, int extra_trim,
                             double end_threshold, int min_trim_size, int32_t *start_trim, int32_t *end_trim,
                             int32_t *start_hits, int32_t *end_hits, int64_t cap, int64_t *n_hits,
                             const int32_t *bc_s, int32_t n_bc_s, const int32_t *bc_e, int32_t n_bc_e,
                             double *bc_full);
int pcabi_flag_list_dev(const uint8_t *flag, int32_t n_adp, int64_t n_read, const int32_t *res, int64_t stride,
                        int32_t *out, int64_t cap, unsigned long long *n_out, void *stream);

/*
 * Middle-adapter scan, round 1 (porechop_abi/nanopore_read.py:219-252): for every window
 * (whole end-trimmed read) the FIRST adapter in list order whose full-adapter identity
 * (pid2, compared after the "%f" round trip like the reference) is not below `threshold`.
 * The reference's masked re-alignment loop hits exactly that adapter first; later rounds
 * re-align the masked read against that adapter and the ones after it (pcabi_align_host pairs).
 * hits: int32 SoA, 5 rows x n_win: adapter index (-1 = none), rs, re (inclusive), m, l2.
 *   pcabi_first_hits_host : host buffers as pcabi_align_host (cross product, tiled on device);
 *                           only the 20 B/read of hits come back over PCIe.
 *   pcabi_first_hit_dev   : epilogue over a device cross-product result block (layout of
 *                           pcabi_align_cross_dev), async on `stream`.
 */
int pcabi_first_hits_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *win_off,
                          const int32_t *win_len, int64_t n_win, const uint8_t *adp_codes,
                          const int32_t *adp_off, const int32_t *adp_len, int32_t n_adp,
                          int match, int mismatch, int gap_open, int gap_extend, double threshold,
                          int32_t *hits);
int pcabi_first_hit_dev(const int32_t *res, int64_t stride, int64_t n_win, int32_t n_adp,
                        double threshold, int32_t *hits, int64_t hit_stride, void *stream);

/*
 * The whole middle-adapter scan (porechop_abi/nanopore_read.py:219-252, the masked re-alignment
 * loop of find_middle_adapters) for a batch of end-trimmed reads, in rounds on the device:
 * round 1 finds each read's first adapter whose best alignment reaches the threshold -- the pairs
 * that can hit are found first, by exact k-mer seeds (pcabi_seed.hip: seed scan, expansion, banded
 * bounds) or, where seeds do not apply, by a score-only filter, and only those candidates get the
 * attribute DP (in owned-column chunks, planned on the device); every later round masks the new
 * hits (N, the reference's '-') and re-aligns only the reads that just hit, from the adapter that
 * hit onwards, until no read hits (DESIGN.md §4 "Middle scan"). As the reference masks a copy
 * (nanopore_read.py:225,234), the caller's codes are never written: a read's first hit copies it
 * into a shadow arena the scan owns, and later hits mask that copy. Pairs where
 * neither way applies run the full cross product with k_first_hit. Hits are written to `hits`
 * (HOST int32, 6 rows x cap: read, adapter, read_start,
 * read_end (exclusive), m, l2 -- full identity = pid6(m, l2)) in discovery order, which per read
 * is the reference's order. Returns the number of hits (may exceed cap: only the first cap are
 * written) or a negative error. threshold must be > 0 (the reference never terminates otherwise).
 *   pcabi_scan_create / destroy : scratch for one adapter table (current device).
 *   pcabi_middle_scan_dev       : codes/win_off/win_len are DEVICE pointers (codes are read only:
 *                                 byte-identical after the call), h_win_len the host copy of the lengths or NULL (the call
 *                                 then copies them: e.g. views from pcabi_trim_views_dev). When the
 *                                 seeded plan covers the table and scoring, the rounds are queued on
 *                                 the device with their counts there (no host round trip between
 *                                 rounds; PCABI_MIDDLE_DEVROUNDS=0 keeps the host-driven loop).
 *   pcabi_middle_scan_host      : host buffers (as pcabi_align_host), copies in, scans.
 *   pcabi_middle_scan_seqs      : the windows as host strings, seqs[w] its first character and
 *                                 seq_len[w] its length (the char * the reference's ctypes wrapper
 *                                 passes per call, porechop_abi/cpp_function_wrappers.py:42-63):
 *                                 encoded (the Dna5 table of pcabi_encode_dna5) by host threads into
 *                                 pinned staging buffers while earlier chunks copy to the device,
 *                                 then scanned as pcabi_middle_scan_host. Same hits, same returns.
 *   pcabi_middle_seed_runs      : how many round-1 scans took their bounds from exact k-mer seeds
 *                                 (pcabi_seed.hip) instead of the score filter, process-wide.
 *                                 PCABI_MIDDLE_SEEDS=0 / 1 (default, cost model) / 2 (always when
 *                                 the seeds apply) selects; the hits are the same either way.
 *   pcabi_middle_requeues       : queued rounds that overflowed a buffer (raw-hit slabs, band task
 *                                 regions, candidate-DP task slots), were dropped and queued again,
 *                                 process-wide; *flags_seen (optional) = the OR of their flags
 *                                 (1 raw hits, 2 band tasks, 4 task slots, 8 shadow arena). Test knobs:
 *                                 PCABI_MIDDLE_INIT_CAPS="raw,task,slots[,arena]" sizes a new scan's buffers,
 *                                 PCABI_MIDDLE_FAULT="round:bits,..." shrinks one round's buffers.
 *   pcabi_scan_profile          : per-phase profile of this scan's device rounds (a diagnostic: with
 *                                 it on, every queued round is synchronised on its own). mode 1 =
 *                                 reset and on, 0 = off, 2 = read only; out[0..14] (n_out values at
 *                                 most): ms of k_seed_scan, k_seed_expand, the band classes, k_cands,
 *                                 the plan kernels, the candidate DP, the rest; then rounds, reads,
 *                                 bases scanned, raw seed hits, inside / edge band tasks, candidate-DP
 *                                 tasks and cells (columns x adapter rows); out[15] = ms of round 1
 *                                 (its runs, whole); out[16..23] per band class (2) the pinned bands'
 *                                 lane-rows issued, active lane-rows (x (2E + 1) = band cells), tasks
 *                                 and passes (counted by the profiled launches only); out[24..25]
 *                                 the classes' E. Returns 26 or < 0.
 */
typedef struct pcabi_scan pcabi_scan;
int pcabi_scan_create(const pcabi_adapters *adps, pcabi_scan **out);
void pcabi_scan_destroy(pcabi_scan *s);
int64_t pcabi_middle_scan_dev(pcabi_scan *s, const uint8_t *codes, const int64_t *win_off,
                              const int32_t *win_len, const int32_t *h_win_len, int64_t n_win,
                              int match, int mismatch, int gap_open, int gap_extend,
                              double threshold, int32_t *hits, int64_t cap, void *stream);
int64_t pcabi_middle_scan_host(int device, const uint8_t *codes, int64_t codes_len,
                               const int64_t *win_off, const int32_t *win_len, int64_t n_win,
                               const uint8_t *adp_codes, const int32_t *adp_off,
                               const int32_t *adp_len, int32_t n_adp, int match, int mismatch,
                               int gap_open, int gap_extend, double threshold, int32_t *hits,
                               int64_t cap);
/*
 * pcabi_stage_seqs_host: the staging the *_seqs entry points use, on its own -- the n strings
 * (addresses of their first characters, lengths) laid out as SeqPack does (4-aligned starts, N
 * between, 16 N after), carried to the device as 2-bit codes plus an N mask and unpacked there
 * into Dna5 bytes, then copied to out[out_len >= the layout's size] (a check of the staging).
 */
int pcabi_stage_seqs_host(int device, const char *const *seqs, const int32_t *seq_len, int64_t n, uint8_t *out,
                          int64_t out_len);
int64_t pcabi_middle_scan_seqs(int device, const char *const *seqs, const int32_t *seq_len, int64_t n,
                               const uint8_t *adp_codes, const int32_t *adp_off,
                               const int32_t *adp_len, int32_t n_adp, int match, int mismatch,
                               int gap_open, int gap_extend, double threshold, int32_t *hits,
                               int64_t cap);
int64_t pcabi_middle_seed_runs(void);
int64_t pcabi_middle_requeues(int32_t *flags_seen);
int32_t pcabi_scan_profile(pcabi_scan *s, int32_t mode, double *out, int32_t n_out);

/*
 * Adapter-set discovery reduction (porechop_abi/nanopore_read.py:158-173): for each adapter a
 * of a cross-product result block, best[a] = max(best[a], max_w pid2(a, w)).
 */
int pcabi_best_full_identity_dev(const int32_t *res, int64_t stride, int64_t n_win, int32_t n_adp,
                                 double *best, void *stream);
/* The same over windows in host buffers (layout of pcabi_align_host, cross product): the
 * (adapter, window) results stay on the device, only n_adp doubles move. best_on_device != 0:
 * `best` is a device pointer on `device` (e.g. the buffer a collective reduces next; it must be
 * ready when called and is updated when the call returns); else a host array. */
int pcabi_best_full_identity_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *win_off,
                                  const int32_t *win_len, int64_t n_win, const uint8_t *adp_codes,
                                  const int32_t *adp_off, const int32_t *adp_len, int32_t n_adp, int match,
                                  int mismatch, int gap_open, int gap_extend, double *best, int best_on_device);

/*
 * Middle-adapter trim ranges (porechop_abi/nanopore_read.py:233-250) of a scan's hits: hit k =
 * (read hits[k], adapter hits[stride + k], read_start hits[2 stride + k], read_end (exclusive)
 * hits[3 stride + k]) -- the layout pcabi_middle_scan_* return -- becomes the range
 * [read_start - (bad_start[a] ? bad_side : good_side), read_end + (bad_end[a] ? bad_side : good_side))
 * of NanoporeRead.middle_trim_positions; bad_start / bad_end flag the adapters whose name is a
 * start / end sequence name. Output grouped per read, each read's hits in discovery order:
 * ranges of read r at cuts[2 k], cuts[2 k + 1] for k in [cut_off[r], cut_off[r + 1]) (cut_off has
 * n_reads + 1 entries) -- the cut layout of pcabi_reads_write.
 *   pcabi_middle_cuts_dev  : device pointers, asynchronous on `stream`.
 *   pcabi_middle_cuts_host : host arrays (n_adp flags each).
 */
int pcabi_middle_cuts_dev(const int32_t *hits, int64_t hit_stride, int64_t n_hits, int64_t n_reads,
                          const uint8_t *bad_start, const uint8_t *bad_end, int good_side, int bad_side,
                          int64_t *cut_off, int64_t *cuts, void *stream);
int pcabi_middle_cuts_host(int device, const int32_t *hits, int64_t hit_stride, int64_t n_hits, int64_t n_reads,
                           const uint8_t *bad_start, const uint8_t *bad_end, int32_t n_adp, int good_side,
                           int bad_side, int64_t *cut_off, int64_t *cuts);

/*
 * Barcode demultiplexing call (porechop_abi/nanopore_read.py:408-482, determine_barcode) from
 * the barcode dicts find_start_trim / find_end_trim fill (nanopore_read.py:193-195, 215-217).
 * Replaces the per-read Python loop of porechop_abi.py:359-438 when -b is given.
 *   *_res            : cross-product result blocks (layout of pcabi_align_cross_dev), n_read
 *                      windows x the side's adapters
 *   *_slot_adp[k]    : slot k of the side's dict in insertion order = the adapter (index into the
 *                      side's table) whose full identity is the entry's value (the last adapter of
 *                      that barcode name in set order)
 *   *_slot_name[k]   : the entry's barcode id (ids >= 0, shared by both sides)
 * Identities are pid6(m, l2) (the reference's "%f" round trip), 0.0 for a failed alignment.
 * Writes call[n_read] = barcode id or -1 ('none'); scores (optional, double[4 * n_read]):
 * require_two -> best start, second start, best end, second end; else best, second overall.
 * The albacore cross-check (nanopore_read.py:479-482) stays with the caller.
 *   pcabi_barcode_call_dev  : device pointers, async on `stream`.
 *   pcabi_barcode_call_host : host result arrays int32[PCABI_NFIELDS][n_adp * n_read] per side.
 */
int pcabi_barcode_call_dev(const int32_t *start_res, int64_t start_stride, const int32_t *start_slot_adp,
                           const int32_t *start_slot_name, int32_t n_start_slots, const int32_t *end_res,
                           int64_t end_stride, const int32_t *end_slot_adp, const int32_t *end_slot_name,
                           int32_t n_end_slots, int64_t n_read, double barcode_threshold, double barcode_diff,
                           int require_two, int32_t *call, double *scores, void *stream);
int pcabi_barcode_call_host(int device, const int32_t *start_res, int32_t n_sa, const int32_t *start_slot_adp,
                            const int32_t *start_slot_name, int32_t n_start_slots, const int32_t *end_res,
                            int32_t n_ea, const int32_t *end_slot_adp, const int32_t *end_slot_name,
                            int32_t n_end_slots, int64_t n_read, double barcode_threshold, double barcode_diff,
                            int require_two, int32_t *call, double *scores);

/*
 * Ab-initio adapter clustering link test (porechop_abi/ab_initio_src/compatibility.cpp,
 * compatibility.h:58-60, called all-vs-all by consensus.py:72-100): semi-global alignment
 * (free end gaps, match 2 / mismatch -1 / linear gap -1, SeqAn String<Dna>: anything but
 * ACGTU is A) of the longer sequence against the shorter, then the reference's flag:
 * 0 not compatible, 1 compatible (integer identity of the aligned region >= 87.5), 2 compatible
 * and the shorter lies inside the longer (region more than 3 bases from an end).
 *   check_compatibility : the drop-in symbol of the reference's compatibility.so (current device;
 *       aborts with a message if the engine fails, see Errors above).
 *   pcabi_compat_host   : n_pairs (pair_i[t], pair_j[t]) of n_seq sequences given as Dna codes
 *       (0..3) in one buffer (seq_off / seq_len, 16 bytes of padding), flags[n_pairs]; the
 *       shorter sequence of a pair must be <= pcabi_max_adapter_len() bases. Empty -> 0.
 */
int check_compatibility(char *raw_seq1, char *raw_seq2);
int pcabi_compat_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *seq_off,
                      const int32_t *seq_len, int64_t n_seq, const int32_t *pair_i, const int32_t *pair_j,
                      int64_t n_pairs, int32_t *flags);
/* consensus.py:72-100 all_vs_all_matrix: mat[n_seq * n_seq] (row-major, -1 on the diagonal,
 * symmetric). Runs every sequence against every sequence in the tiled cross mode (sequences over
 * 128 bases as rows on the striped core) when all are 1..pcabi_max_adapter_len() bases, explicit
 * pairs otherwise. n_seq <= 46340. */
int pcabi_compat_all_vs_all_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *seq_off,
                                 const int32_t *seq_len, int64_t n_seq, int32_t *mat);

/*
 * Ab-initio k-mer counts (porechop_abi/ab_initio_src/approx_counter.cpp, csrc/pcabi_kmer.hip).
 * Sequences: Dna5 codes (0..4) in one buffer, seq_off / seq_len.
 *   pcabi_kmer_count_host : count_kmers (:487-519): every k-mer (2 <= k <= 32, 2-bit value,
 *       first base in the top bits) without N, not low-complexity (dimer score >= lc_threshold,
 *       :214-234) and not in forbidden_sorted (ascending); writes (k-mer, count) ascending by
 *       k-mer, returns the number of distinct k-mers (if > cap nothing is written: call again
 *       with cap >= the return value) or a negative PCABI_E_*.
 *   pcabi_kmer_approx_host : errorCount (:531-601): counts[q] = sum over sequences of
 *       3 - d for the best substring edit distance d <= 2 of kmers[q] (SeqAn's search at <= 2
 *       errors reports a sequence once at every level from d to 2). Sequences start at 4-aligned
 *       offsets of a buffer whose length is a multiple of 4 (N padding); n_kmers <= 65535 * 64.
 */
int64_t pcabi_kmer_count_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *seq_off,
                              const int32_t *seq_len, int64_t n_seq, int k, float lc_threshold,
                              const uint64_t *forbidden_sorted, int64_t n_forbidden, uint64_t *kmers,
                              uint32_t *counts, int64_t cap);
/*   pcabi_kmer_top_host : the same counts, sorted by count descending (equal counts k-mer
 *       ascending), only the entries with count >= max(min_count, the top-th largest count)
 *       (top <= 0: no rank cut) -- every k-mer get_most_frequent / get_solid_kmers can keep
 *       (:372-405). Returns the entries written, or the capacity needed when > cap. */
int64_t pcabi_kmer_top_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *seq_off,
                            const int32_t *seq_len, int64_t n_seq, int k, float lc_threshold,
                            const uint64_t *forbidden_sorted, int64_t n_forbidden, int64_t top, int64_t min_count,
                            uint64_t *kmers, uint32_t *counts, int64_t cap);
/* Host gather of byte segments: dst[dst_off[i] .. + len[i]) = src[src_off[i] .. + len[i]). */
void pcabi_gather_host(const uint8_t *src, const int64_t *src_off, const int32_t *len, int64_t n, uint8_t *dst,
                       const int64_t *dst_off);
int pcabi_kmer_approx_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *seq_off,
                           const int32_t *seq_len, int64_t n_seq, int k, const uint64_t *kmers, int64_t n_kmers,
                           uint64_t *counts);

/*
 * Sequence files (host code, csrc/pcabi_io.cpp; replaces porechop_abi/misc.py:60-168
 * load_fasta_or_fastq and NanoporeRead's normalisation, nanopore_read.py:31-44, for the batched
 * path, and NanoporeRead.get_fasta / get_fastq, nanopore_read.py:84-156, for output).
 *   pcabi_fastx_open / next / close : streaming reader, plain or gzip, FASTA or FASTQ (by the
 *       first character), the reference's parse rules; next() returns up to max_reads records
 *       (stopping once max_bases sequence bytes are in the batch) as a new pcabi_reads, or a
 *       negative PCABI_E_* (PCABI_E_PARSE for a malformed file); 0 records at end of file.
 *   pcabi_fastx_load : the whole file as one batch.
 *   raw != 0 : keep the file's text (no upper-casing, no U -> T, no quality padding; FASTQ '+'
 *       lines kept in spacer) -- the tuples of misc.load_fasta_or_fastq.
 *   pcabi_reads_views: borrowed pointers into a batch (valid until pcabi_reads_free):
 *       names   : full headers (text after '@' / '>'), name_off[n + 1]
 *       seq     : upper-cased sequences, U -> T for RNA reads (rna[i] = 1), seq_off[n + 1]
 *       qual    : qualities padded with '+' to the sequence length (FASTA: all '+'), qual_off[n + 1]
 *       codes   : Dna5 codes in the engine layout (4-aligned code_off[n], len[n], 16 bytes of
 *                 N padding at the end) -- ready for pcabi_align_host / the device ABI.
 *   pcabi_reads_write: the reference's trimmed output of every read (select[i] != 0 if given):
 *       start_trim / end_trim (NULL = untrimmed), middle cut ranges [cuts[2k], cuts[2k+1]) of the
 *       trimmed sequence for k in [cut_off[i], cut_off[i+1]) (NULL = none; a read with cuts is
 *       written as its split parts, or dropped with discard_middle), FASTA (70-column lines) or
 *       FASTQ, gzip when gz != 0, appended when append != 0, path "-" = stdout (plain only);
 *       untrimmed != 0 writes reads without cuts whole (split parts still come from the trimmed
 *       sequence, as in the reference). Returns the number of reads that produced output (the
 *       reference's non-empty read strings, porechop_abi.py:598-604), or a negative PCABI_E_*.
 */
enum { PCABI_FASTA = 0, PCABI_FASTQ = 1 };
typedef struct pcabi_fastx pcabi_fastx;
typedef struct pcabi_reads pcabi_reads;
typedef struct pcabi_reads_view {
    int64_t n;
    int32_t type;
    const char *names;
    const int64_t *name_off;
    const char *seq;
    const int64_t *seq_off;
    const char *qual;
    const int64_t *qual_off;
    const uint8_t *rna;
    const char *spacer;
    const int64_t *spacer_off;
    const uint8_t *codes;
    int64_t codes_len;
    const int64_t *code_off;
    const int32_t *len;
} pcabi_reads_view;
int pcabi_fastx_open(const char *path, int raw, pcabi_fastx **out);
int pcabi_fastx_type(const pcabi_fastx *r);
/* Byte-range reading of a plain (not gzip) file, for read shards split by position:
 *   pcabi_fastx_record_start : the first record start at or after `byte` (the file size if
 *       none): a FASTQ header line whose third line is the '+' line; a FASTA header with a name
 *       whose previous header has one too (an empty header's sequence runs on into the next
 *       record). Splitting at record starts gives every record to exactly one range.
 *   pcabi_fastx_set_range    : read only [begin, end) from now on (both record starts, or 0 / the
 *       file size); a fresh reader (no record read yet). */
int64_t pcabi_fastx_record_start(const pcabi_fastx *r, int64_t byte);
int pcabi_fastx_set_range(pcabi_fastx *r, int64_t begin, int64_t end);
/* Bytes of a plain file (or of its set range) not yet parsed; -1 for a gzip input, whose decoded
 * size is unknown. misc.read_batches sizes a pipeline's last batches from it (a ramp-down, so the
 * final write overlaps the trims before it). */
int64_t pcabi_fastx_remaining(const pcabi_fastx *r);
/* Streaming split of any input (gzip included) into spans of decoded text holding whole records,
 * for a distributor that hands spans to other readers (shards.trim_file_sharded): the next span,
 * at least max_bytes long unless the input ends (one record may overshoot), cut where a fresh
 * reader parses the same records as the continuous read -- FASTQ after a record whose successor's
 * first line starts with '@', FASTA before a header with a name whose preceding header has one.
 * *text is valid until the next call on r. Returns 1, 0 at the end of the input, or < 0. */
int pcabi_fastx_next_text(pcabi_fastx *r, int64_t max_bytes, const char **text, int64_t *len);
int64_t pcabi_fastx_next(pcabi_fastx *r, int64_t max_reads, int64_t max_bases, pcabi_reads **out);
void pcabi_fastx_close(pcabi_fastx *r);
int pcabi_fastx_load(const char *path, int raw, pcabi_reads **out);
int64_t pcabi_reads_count(const pcabi_reads *b);
int pcabi_reads_type(const pcabi_reads *b);
int pcabi_reads_views(const pcabi_reads *b, pcabi_reads_view *v);
void pcabi_reads_free(pcabi_reads *b);
int pcabi_reads_write(const pcabi_reads *b, const char *path, int append, int gz, int fasta,
                      const int32_t *start_trim, const int32_t *end_trim, const int64_t *cut_off,
                      const int64_t *cuts, int min_split_read_size, int discard_middle,
                      int untrimmed, const uint8_t *select);
/* Batches of 64 MB and more live in huge-page mappings that freed batches hand to a process-wide
 * cache (PCABI_IO_CACHE_MB, default min(4 GB, RAM / 8)) for the next batch to reuse; this
 * returns every cached mapping to the system. */
void pcabi_io_release_cache(void);

#ifdef __cplusplus
}
#endif
#endif /* PCABI_H */
