// pcabi_io.cpp -- native FASTA / FASTQ (plain or gzip) reader and trimmed-read writer for the
// adapter-alignment engine (host code, part of libpcabi.so; declared in include/pcabi.h).
//
// The reader turns a sequence file straight into the engine's input layout -- Dna5 codes packed
// back to back at 4-aligned offsets with 16 bytes of tail padding (engine.SeqPack) -- plus the
// read names, upper-cased sequence text and qualities, in batches, with the reference's parsing
// rules:
//   * file type from the first decoded character: '>' FASTA, '@' FASTQ, else an error
//     (porechop_abi/misc.py:84-105); gzip by its magic bytes, bzip2 / zip refused (:60-81);
//   * FASTQ: 4 lines per record, each stripped; name = line[1:] (the full header), sequence,
//     spacer, qualities (misc.py:148-165); a blank or truncated record is a parse error (the
//     reference dies on it too);
//   * FASTA: stripped lines, blank lines skipped, '>' starts a record whose sequence is the
//     concatenation of the following lines; a record with an empty name is not emitted and its
//     sequence carries over (misc.py:123-145, replicated exactly);
//   * lines end at \n, \r\n or \r (Python's universal newlines), strip() removes the ASCII
//     characters str.isspace() accepts;
//   * NanoporeRead's normalisation (porechop_abi/nanopore_read.py:31-44): sequence upper-cased,
//     U -> T when the read has more U than T (rna flag), qualities padded with '+' to the
//     sequence length.
// The writer reproduces NanoporeRead.get_fasta / get_fastq (nanopore_read.py:106-156) for a
// batch: start / end trims with Python slice semantics, middle split parts (positions given as
// [begin, end) ranges of the trimmed sequence, parts shorter than min_split_read_size dropped,
// names numbered like add_number_to_read_name, :503-509), 70-column FASTA lines, T -> U for RNA
// reads, optional gzip.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/uio.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <unordered_map>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pcabi.h"

namespace pcabi_internal {
int fail(int code, const std::string &msg);   // pcabi_engine.hip: pcabi_last_error()
}
using pcabi_internal::fail;

namespace {

inline bool py_space(unsigned char c) {   // str.isspace() on ASCII
    return (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x20);
}

uint8_t g_dna5[256];
const bool g_dna5_init = [] {
    for (int i = 0; i < 256; ++i) g_dna5[i] = 4;
    const char *s = "ACGTU", *l = "acgtu";
    const uint8_t v[5] = {0, 1, 2, 3, 3};
    for (int k = 0; k < 5; ++k) {
        g_dna5[(unsigned char)s[k]] = v[k];
        g_dna5[(unsigned char)l[k]] = v[k];
    }
    return true;
}();

}  // namespace

struct pcabi_fastx {
    gzFile f = nullptr;
    int type = -1;                 // PCABI_FASTA / PCABI_FASTQ
    std::vector<char> buf;         // gzip: decoded bytes [0, end)
    const char *base = nullptr;    // buf.data(), or the mapping of a plain file
    void *map = nullptr;           // plain files are memory-mapped whole
    size_t map_len = 0;
    size_t pin = (size_t)-1;       // refills keep the bytes from here on (a batch's records)
    size_t pos = 0, end = 0;
    bool eof = false;
    bool err = false;              // a read error (e.g. a truncated gzip stream): the next call fails
    int64_t line_no = 0;
    bool raw = false;              // keep the file's text (misc.load_fasta_or_fastq tuples)
    size_t size_hint = 0;          // decoded bytes expected (file size; x4 for gzip)
    size_t released = 0;           // mapped file bytes before this have had their page mappings dropped
    // populate-ahead (plain files): a helper thread maps the pages up to kAhead bytes past the
    // reader's published position, so the record scan finds them mapped (r05: the scan's own
    // faults were half a 200 MB batch's read time)
    std::thread ahead;
    std::atomic<bool> ahead_stop{false};
    std::atomic<size_t> reader_at{0};
    ~pcabi_fastx() {
        ahead_stop = true;
        if (ahead.joinable()) ahead.join();
    }
    // FASTA state that crosses batch boundaries
    bool fa_have_name = false;     // a header was seen (its name may be empty)
    std::string fa_name, fa_seq;
    int txt_named = -1;            // pcabi_fastx_next_text: the last header had a name (1), none (0), no header (-1)
};

// Large batch buffers (>= 8 MB, r05) come from anonymous mappings with transparent huge pages and
// go back to a small process-wide cache when a batch is freed, so the next batch reuses pages
// that are already faulted in: first-touch faults and the unmapping of gigabyte buffers cost
// about as much as the parse itself (4 KB pages: ~400 k faults per 1.6 GB batch).
namespace {
namespace bigmem {
constexpr size_t kBig = 8ull << 20;   // r05: 64 MB left the buffers of 6 k-read batches to malloc, which
                                      // maps and unmaps them per batch (e2e 3.5x slower at that size)
// Free blocks kept for reuse: PCABI_IO_CACHE_MB, default min(4 GB, physical memory / 8) -- enough
// for the batches a pipeline keeps in flight; pcabi_io_release_cache() returns them all.
size_t cache_max() {
    static const size_t v = [] {
        const char *e = std::getenv("PCABI_IO_CACHE_MB");
        if (e && e[0]) return (size_t)std::max(0LL, std::atoll(e)) << 20;
        const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGE_SIZE);
        const size_t ram = (pages > 0 && psz > 0) ? (size_t)pages * (size_t)psz : (8ull << 30);
        return std::min<size_t>(4ull << 30, ram / 8);
    }();
    return v;
}
std::mutex mu;
std::unordered_map<void *, size_t> mapped;          // live and cached blocks -> mapped bytes
std::vector<std::pair<void *, size_t>> cache;       // free blocks
size_t cached = 0;

inline size_t round2m(size_t b) { return (b + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1); }

void *get(size_t bytes) {
    if (bytes < kBig) return ::operator new(bytes);
    std::lock_guard<std::mutex> g(mu);
    size_t best = SIZE_MAX, bi = 0;
    for (size_t i = 0; i < cache.size(); ++i)
        if (cache[i].second >= bytes && cache[i].second < best) { best = cache[i].second; bi = i; }
    if (best != SIZE_MAX && best <= 2 * bytes + (256ull << 20)) {
        void *p = cache[bi].first;
        cached -= best;
        cache.erase(cache.begin() + (long)bi);
        return p;
    }
    // 1/8 headroom: the next batch's buffers, sized exactly and a little larger or smaller than
    // these, still fit a cached block (already faulted in) instead of a fresh mapping
    const size_t m = round2m(bytes + bytes / 8);
    void *p = mmap(nullptr, m, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) throw std::bad_alloc();
#ifdef MADV_HUGEPAGE
    madvise(p, m, MADV_HUGEPAGE);
#endif
    mapped[p] = m;
    return p;
}

void put(void *p, size_t bytes) {
    if (!p) return;
    if (bytes < kBig) {
        ::operator delete(p);
        return;
    }
    std::lock_guard<std::mutex> g(mu);
    const size_t m = mapped.at(p);
    cache.emplace_back(p, m);
    cached += m;
    while (cached > cache_max() && !cache.empty()) {   // drop the oldest
        munmap(cache.front().first, cache.front().second);
        mapped.erase(cache.front().first);
        cached -= cache.front().second;
        cache.erase(cache.begin());
    }
}
void release() {
    std::lock_guard<std::mutex> g(mu);
    for (auto &c : cache) {
        munmap(c.first, c.second);
        mapped.erase(c.first);
    }
    cache.clear();
    cached = 0;
}
}  // namespace bigmem
}  // namespace

extern "C" void pcabi_io_release_cache(void) { bigmem::release(); }

// vector whose resize() leaves new elements uninitialised (the batch buffers are written once,
// in parallel; zero-filling gigabytes first would cost as much as the parse)
template <typename T>
struct NoInit : std::allocator<T> {
    template <typename U>
    struct rebind { using other = NoInit<U>; };
    NoInit() = default;
    template <typename U>
    NoInit(const NoInit<U> &) {}
    T *allocate(size_t n) { return static_cast<T *>(bigmem::get(n * sizeof(T))); }
    void deallocate(T *p, size_t n) noexcept { bigmem::put(p, n * sizeof(T)); }
    template <typename U>
    void construct(U *p) noexcept { ::new ((void *)p) U; }
    template <typename U, typename... A>
    void construct(U *p, A &&...a) { ::new ((void *)p) U(std::forward<A>(a)...); }
};
template <typename T, typename U>
bool operator==(const NoInit<T> &, const NoInit<U> &) { return true; }
template <typename T, typename U>
bool operator!=(const NoInit<T> &, const NoInit<U> &) { return false; }
template <typename T>
using RawVec = std::vector<T, NoInit<T>>;

struct pcabi_reads {
    int type = -1;
    int64_t n = 0;
    RawVec<char> names;                      // full headers (after '@' / '>'), back to back
    std::vector<int64_t> name_off{0};
    RawVec<char> seq;                        // upper-cased, U->T for RNA reads
    std::vector<int64_t> seq_off{0};
    RawVec<char> qual;                       // padded with '+' to the sequence length
    std::vector<int64_t> qual_off{0};
    std::vector<uint8_t> rna;
    RawVec<char> spacer;                     // FASTQ '+' lines (stripped)
    std::vector<int64_t> spacer_off{0};
    RawVec<uint8_t> codes;                   // Dna5, 4-aligned starts, 16 B tail padding (N)
    std::vector<int64_t> code_off;
    std::vector<int32_t> len;
};

namespace {

// Next line (without its terminator) as [*p, *p + *n); false at end of file. Terminators are
// found with memchr: the first '\n', then any '\r' before it (CRLF, or a lone CR that ends the
// line earlier).
// The first '\n' or '\r' in [s, e), or nullptr: one pass over the line (r05; two memchr passes --
// '\n', then '\r' before it -- read every byte twice, the record scan's main cost once the pages are
// mapped ahead). AVX2 where the CPU has it.
#if defined(__x86_64__)
__attribute__((target("avx2"))) const char *find_eol_avx2(const char *s, const char *e) {
    const __m256i lf = _mm256_set1_epi8('\n'), cr = _mm256_set1_epi8('\r');
    for (; s + 32 <= e; s += 32) {
        const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s));
        const unsigned m = (unsigned)_mm256_movemask_epi8(_mm256_or_si256(_mm256_cmpeq_epi8(v, lf), _mm256_cmpeq_epi8(v, cr)));
        if (m) return s + __builtin_ctz(m);
    }
    for (; s < e; ++s)
        if (*s == '\n' || *s == '\r') return s;
    return nullptr;
}
#endif
const char *find_eol(const char *s, const char *e) {
#if defined(__x86_64__)
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2) return find_eol_avx2(s, e);
#endif
    const char *nl = (const char *)std::memchr(s, '\n', (size_t)(e - s));
    const char *cr = (const char *)std::memchr(s, '\r', (size_t)((nl ? nl : e) - s));
    return cr ? cr : nl;
}

bool next_line(pcabi_fastx *r, const char **p, size_t *n) {
    for (;;) {
        const char *base = r->base;
        const char *s0 = base + r->pos, *e0 = base + r->end;
        // the first line end of either kind: a '\r' before the first '\n' is the line's end
        const char *eol = find_eol(s0, e0);
        const char *nl = eol && *eol == '\n' ? eol : nullptr;
        const char *cr = eol && *eol == '\r' ? eol : nullptr;
        if (cr && (cr + 1 < e0 || r->eof)) {          // \r ends the line (a following \n is eaten)
            *p = s0;
            *n = (size_t)(cr - s0);
            r->pos = (size_t)(cr + 1 - base) + ((cr + 1 < e0 && cr[1] == '\n') ? 1 : 0);
            ++r->line_no;
            return true;
        }
        if (nl && !cr) {
            *p = s0;
            *n = (size_t)(nl - s0);
            r->pos = (size_t)(nl + 1 - base);
            ++r->line_no;
            return true;
        }
        if (r->eof) {
            if (r->pos < r->end) {   // last line without a terminator
                *p = s0;
                *n = r->end - r->pos;
                r->pos = r->end;
                ++r->line_no;
                return true;
            }
            return false;
        }
        // refill: keep the partial line (and a pinned batch), grow if it fills the buffer
        const size_t from = std::min(r->pos, r->pin);
        if (from > 0) {
            std::memmove(r->buf.data(), r->buf.data() + from, r->end - from);
            r->pos -= from;
            r->end -= from;
            if (r->pin != (size_t)-1) r->pin -= from;
        }
        if (r->buf.size() - r->end < (1u << 20)) r->buf.resize(std::max<size_t>(r->buf.size() * 2, 4u << 20));
        r->base = r->buf.data();
        const int got = gzread(r->f, r->buf.data() + r->end, (unsigned)std::min<size_t>(r->buf.size() - r->end, 1u << 30));
        int zerr = Z_OK;
        const char *zmsg = got < 0 || got == 0 ? gzerror(r->f, &zerr) : nullptr;
        if (got < 0 || (got == 0 && zerr != Z_OK && zerr != Z_STREAM_END)) {
            // a damaged or truncated gzip stream: the reference's gzip module raises too
            // (EOFError "Compressed file ended before the end-of-stream marker was reached")
            fail(PCABI_E_PARSE, std::string("read error: ") + (zmsg ? zmsg : "?"));
            r->err = true;
            r->eof = true;
            r->end = r->pos;   // drop the partial data
            return false;
        }
        if (got == 0) r->eof = true;
        r->end += (size_t)got;
    }
}

void strip(const char **p, size_t *n) {
    const char *a = *p;
    size_t m = *n;
    while (m && py_space((unsigned char)a[0])) { ++a; --m; }
    while (m && py_space((unsigned char)a[m - 1])) --m;
    *p = a;
    *n = m;
}

uint8_t g_upper[256];
const bool g_upper_init = [] {
    for (int i = 0; i < 256; ++i) g_upper[i] = (uint8_t)((i >= 'a' && i <= 'z') ? i - 32 : i);
    return true;
}();

// A record is appended in pieces (name, sequence, qualities) straight from the line buffer.
void add_name(pcabi_reads *b, const char *name, size_t nn) {
    b->names.insert(b->names.end(), name, name + nn);
    b->name_off.push_back((int64_t)b->names.size());
}

// Sequence with NanoporeRead's normalisation unless raw: upper case, U -> T when the read holds
// more U than T; Dna5 codes (U and T are both code 3) into the engine layout in the same pass.
void add_seq(pcabi_reads *b, const char *seq, size_t ns, bool raw) {
    const size_t s0 = b->seq.size();
    b->seq.resize(s0 + ns);
    char *d = b->seq.data() + s0;
    const int64_t off = (int64_t)b->codes.size();
    const size_t padded = (ns + 3) & ~(size_t)3;
    b->codes.resize((size_t)off + padded);
    uint8_t *c = b->codes.data() + off;
    int64_t nu = 0, nt = 0;
    if (raw) {
        std::memcpy(d, seq, ns);
        for (size_t i = 0; i < ns; ++i) c[i] = g_dna5[(unsigned char)seq[i]];
    } else {
        for (size_t i = 0; i < ns; ++i) {
            const uint8_t u = g_upper[(unsigned char)seq[i]];
            nu += (u == 'U');
            nt += (u == 'T');
            d[i] = (char)u;
            c[i] = g_dna5[u];
        }
    }
    for (size_t i = ns; i < padded; ++i) c[i] = 4;
    const bool rna = !raw && nu > nt;
    if (rna)
        for (size_t i = 0; i < ns; ++i)
            if (d[i] == 'U') d[i] = 'T';
    b->rna.push_back(rna ? 1 : 0);
    b->seq_off.push_back((int64_t)b->seq.size());
    b->code_off.push_back(off);
    b->len.push_back((int32_t)ns);
}

// Qualities padded with '+' to the sequence length unless raw; closes the record.
void add_qual(pcabi_reads *b, const char *q, size_t nq, size_t ns, bool raw, const char *sp = nullptr,
              size_t nsp = 0) {
    b->qual.insert(b->qual.end(), q, q + nq);
    if (!raw && nq < ns) b->qual.insert(b->qual.end(), ns - nq, '+');
    b->qual_off.push_back((int64_t)b->qual.size());
    b->spacer.insert(b->spacer.end(), sp, sp + nsp);
    b->spacer_off.push_back((int64_t)b->spacer.size());
    ++b->n;
}

void add_record(pcabi_reads *b, const char *name, size_t nn, const char *seq, size_t ns, const char *q, size_t nq,
                bool raw = false) {
    add_name(b, name, nn);
    add_seq(b, seq, ns, raw);
    add_qual(b, q, nq, ns, raw);
}

void finish_batch(pcabi_reads *b) { b->codes.resize(b->codes.size() + 16, 4); }

// A FASTQ record as spans of the batch's text (offsets from the batch start).
struct Span {
    size_t no, nn, so, sn, xo, xn, qo, qn;
};

#ifndef MADV_POPULATE_READ
#define MADV_POPULATE_READ 22
#endif
// The populate-ahead loop of a mapped file (pcabi_fastx::ahead): [at, end) in 8 MB steps, never more
// than kAhead bytes past the reader. MADV_POPULATE_READ (Linux >= 5.14) maps a step in one call;
// where it is refused the helper touches one byte per page instead (the faults then land here).
void populate_ahead(pcabi_fastx *r, size_t at, size_t end) {
    constexpr size_t kStep = 8u << 20, kAhead = 512u << 20;
    bool populate = true;
    volatile unsigned sink = 0;
    const char *m = (const char *)r->map;
    while (!r->ahead_stop.load(std::memory_order_relaxed) && at < end) {
        const size_t rd = r->reader_at.load(std::memory_order_relaxed);
        at = std::max(at, rd & ~(size_t)4095);        // never behind the reader (its pages are mapped)
        if (at >= end) break;
        const size_t lim = rd + kAhead;
        if (at >= lim) {
            std::this_thread::sleep_for(std::chrono::microseconds(200));
            continue;
        }
        const size_t n = std::min({kStep, end - at, lim - at});
        if (!populate || madvise((void *)(m + at), n, MADV_POPULATE_READ) != 0) {
            populate = false;
            unsigned x = 0;
            for (size_t q = at; q < at + n; q += 4096) x += (unsigned char)m[q];
            sink = sink + x;
        }
        at += n;
    }
}

int io_threads() {
    if (const char *e = std::getenv("PCABI_IO_THREADS")) {
        const int t = std::atoi(e);
        if (t > 0) return std::min(t, 256);
    }
    const unsigned hw = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hw ? hw : 1u, 16u));
}

// The records of one FASTQ batch, normalised into b in parallel: offsets first (prefix sums),
// then every thread fills a contiguous range of records (names, sequence + Dna5 codes + rna
// flag, qualities + padding, spacer lines).
void fill_fastq(pcabi_reads *b, const char *T, const std::vector<Span> &rec, bool raw) {
    const size_t n = rec.size();
    const size_t n0 = (size_t)b->n;
    b->name_off.resize(n0 + n + 1);
    b->seq_off.resize(n0 + n + 1);
    b->qual_off.resize(n0 + n + 1);
    b->spacer_off.resize(n0 + n + 1);
    b->code_off.resize(n0 + n);
    b->len.resize(n0 + n);
    b->rna.resize(n0 + n);
    int64_t code_end = (int64_t)b->codes.size();
    for (size_t i = 0; i < n; ++i) {
        const Span &r = rec[i];
        b->name_off[n0 + i + 1] = b->name_off[n0 + i] + (int64_t)r.nn;
        b->seq_off[n0 + i + 1] = b->seq_off[n0 + i] + (int64_t)r.sn;
        b->qual_off[n0 + i + 1] = b->qual_off[n0 + i] + (int64_t)(raw ? r.qn : std::max(r.qn, r.sn));
        b->spacer_off[n0 + i + 1] = b->spacer_off[n0 + i] + (int64_t)r.xn;
        b->code_off[n0 + i] = code_end;
        b->len[n0 + i] = (int32_t)r.sn;
        code_end += (int64_t)((r.sn + 3) & ~(size_t)3);
    }
    // exact sizes, known from the record scan (finish_batch's 16 bytes of padding included): the
    // blocks of one batch then match the next batch's, and the block cache hands them back already
    // faulted in (a file-sized reservation per batch made every free an unmapping, r05)
    b->names.reserve((size_t)b->name_off[n0 + n]);
    b->seq.reserve((size_t)b->seq_off[n0 + n]);
    b->qual.reserve((size_t)b->qual_off[n0 + n]);
    b->codes.reserve((size_t)code_end + 16);
    b->names.resize((size_t)b->name_off[n0 + n]);
    b->seq.resize((size_t)b->seq_off[n0 + n]);
    b->qual.resize((size_t)b->qual_off[n0 + n]);
    b->spacer.resize((size_t)b->spacer_off[n0 + n]);
    b->codes.resize((size_t)code_end);
    auto work = [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
            const Span &r = rec[i];
            const size_t k = n0 + i;
            std::memcpy(b->names.data() + b->name_off[k], T + r.no, r.nn);
            std::memcpy(b->spacer.data() + b->spacer_off[k], T + r.xo, r.xn);
            char *d = b->seq.data() + b->seq_off[k];
            uint8_t *c = b->codes.data() + b->code_off[k];
            const unsigned char *sq = (const unsigned char *)T + r.so;
            int64_t nu = 0, nt = 0;
            if (raw) {
                std::memcpy(d, sq, r.sn);
                for (size_t j = 0; j < r.sn; ++j) c[j] = g_dna5[sq[j]];
            } else {
                for (size_t j = 0; j < r.sn; ++j) {
                    const uint8_t u = g_upper[sq[j]];
                    nu += (u == 'U');
                    nt += (u == 'T');
                    d[j] = (char)u;
                    c[j] = g_dna5[u];
                }
            }
            for (size_t j = r.sn; j < ((r.sn + 3) & ~(size_t)3); ++j) c[j] = 4;
            const bool rna = !raw && nu > nt;
            if (rna)
                for (size_t j = 0; j < r.sn; ++j)
                    if (d[j] == 'U') d[j] = 'T';
            b->rna[k] = rna ? 1 : 0;
            char *q = b->qual.data() + b->qual_off[k];
            std::memcpy(q, T + r.qo, r.qn);
            if (!raw && r.qn < r.sn) std::memset(q + r.qn, '+', r.sn - r.qn);
        }
    };
    const int nt = (int)std::min<size_t>((size_t)io_threads(), std::max<size_t>(1, n / 256));
    if (nt <= 1) {
        work(0, n);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) th.emplace_back(work, n * t / nt, n * (t + 1) / nt);
        for (auto &x : th) x.join();
    }
    b->n = (int64_t)(n0 + n);
}

}  // namespace

extern "C" {

int pcabi_fastx_open(const char *path, int raw, pcabi_fastx **out) {
    if (!path || !out) return fail(PCABI_E_ARG, "bad arguments");
    *out = nullptr;
    FILE *fp = std::fopen(path, "rb");
    if (!fp) return fail(PCABI_E_ARG, std::string("could not find ") + path);
    unsigned char magic[4] = {0, 0, 0, 0};
    const size_t nm = std::fread(magic, 1, 4, fp);
    std::fclose(fp);
    if (nm >= 3 && magic[0] == 0x42 && magic[1] == 0x5a && magic[2] == 0x68)
        return fail(PCABI_E_ARG, "cannot use bzip2 format - use gzip instead");
    if (nm >= 4 && magic[0] == 0x50 && magic[1] == 0x4b && magic[2] == 0x03 && magic[3] == 0x04)
        return fail(PCABI_E_ARG, "cannot use zip format - use gzip instead");
    const bool gz = nm >= 2 && magic[0] == 0x1f && magic[1] == 0x8b;
    pcabi_fastx *r = new pcabi_fastx();
    r->raw = raw != 0;
    if (!gz) {
        // plain text: map the file, lines are read in place (no copies, no refills)
        const int fd = ::open(path, O_RDONLY);
        struct stat st;
        if (fd >= 0 && fstat(fd, &st) == 0 && st.st_size > 0) {
            // mapped lazily (r05): the record scan faults its batch in as it goes (fault-around maps
            // 16 pages a fault); MAP_POPULATE mapped the whole file before the first batch could be
            // parsed (~80 ms of a 1.6 GB file's first batch, nothing else overlapping it)
            void *m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
            if (m != MAP_FAILED) {
                madvise(m, (size_t)st.st_size, MADV_SEQUENTIAL);
                r->map = m;
                r->map_len = (size_t)st.st_size;
                r->base = (const char *)m;
                r->end = r->map_len;
                r->eof = true;
            }
        }
        if (fd >= 0) ::close(fd);
    }
    if (!r->map) {
        gzFile f = gzopen(path, "rb");
        if (!f) {
            delete r;
            return fail(PCABI_E_ARG, std::string("could not open ") + path);
        }
        gzbuffer(f, 1u << 20);
        r->f = f;
    }
    if (FILE *sf = std::fopen(path, "rb")) {
        std::fseek(sf, 0, SEEK_END);
        const long sz = std::ftell(sf);
        std::fclose(sf);
        if (sz > 0) r->size_hint = (size_t)sz * ((magic[0] == 0x1f && magic[1] == 0x8b) ? 4 : 1);
    }
    if (!r->map) {
        r->buf.resize(4u << 20);
        r->base = r->buf.data();
        // type from the first decoded character
        while (r->end == 0 && !r->eof) {
            const int got = gzread(r->f, r->buf.data(), (unsigned)r->buf.size());
            if (got <= 0) r->eof = true;
            else r->end = (size_t)got;
        }
    }
    const char c0 = r->end ? r->base[0] : 0;
    if (c0 == '>') r->type = PCABI_FASTA;
    else if (c0 == '@') r->type = PCABI_FASTQ;
    else {
        pcabi_fastx_close(r);
        return fail(PCABI_E_PARSE, std::string("File is neither FASTA or FASTQ: ") + path);
    }
    *out = r;
    return 0;
}

int pcabi_fastx_type(const pcabi_fastx *r) { return r ? r->type : -1; }

}  // extern "C"

namespace {
// Universal-newline line starts inside a memory-mapped file (the reader's line rules).
size_t line_after(const char *b, size_t n, size_t p) {
    while (p < n && b[p] != '\n' && b[p] != '\r') ++p;
    if (p < n && b[p] == '\r') {
        ++p;
        if (p < n && b[p] == '\n') ++p;
    } else if (p < n) {
        ++p;
    }
    return p;
}
size_t line_at_or_after(const char *b, size_t n, size_t p) {
    if (p == 0 || p >= n) return std::min(p, n);
    if (b[p - 1] == '\n' || (b[p - 1] == '\r' && b[p] != '\n')) return p;
    return line_after(b, n, p);
}
bool blank_after(const char *b, size_t n, size_t p) {   // only whitespace up to the line end
    for (; p < n && b[p] != '\n' && b[p] != '\r'; ++p)
        if (!std::isspace((unsigned char)b[p])) return false;
    return true;
}
// the nearest header ('>' at a line start) before position p, or n if none
size_t header_before(const char *b, size_t n, size_t p) {
    while (p > 0) {
        --p;
        if (b[p] == '>' && (p == 0 || b[p - 1] == '\n' || b[p - 1] == '\r')) return p;
    }
    return n;
}
}  // namespace

extern "C" {

int64_t pcabi_fastx_record_start(const pcabi_fastx *r, int64_t byte) {
    if (!r || !r->map) return fail(PCABI_E_ARG, "record starts need a plain (memory-mapped) file");
    const char *b = r->base;
    const size_t n = r->map_len;
    size_t p = line_at_or_after(b, n, byte < 0 ? 0 : (size_t)byte);
    for (; p < n; p = line_after(b, n, p)) {
        if (r->type == PCABI_FASTQ) {
            // a header line ('@') whose third line is the '+' line: a quality line may start
            // with '@', but two lines after it comes the next record's sequence, never '+'
            if (b[p] != '@') continue;
            const size_t q = line_after(b, n, line_after(b, n, p));
            if (q < n && b[q] == '+') return (int64_t)p;
        } else {
            // a header with a name, after a header with a name: an empty header's sequence runs
            // on into the next record (the reader's rule), so no record starts there
            if (b[p] != '>' || blank_after(b, n, p + 1)) continue;
            const size_t h = header_before(b, n, p);
            if (h == n || !blank_after(b, n, h + 1)) return (int64_t)p;
        }
    }
    return (int64_t)n;
}

int64_t pcabi_fastx_remaining(const pcabi_fastx *r) {
    if (!r || !r->map) return -1;
    return r->end > r->pos ? (int64_t)(r->end - r->pos) : 0;
}

int pcabi_fastx_set_range(pcabi_fastx *r, int64_t begin, int64_t end) {
    if (!r || !r->map) return fail(PCABI_E_ARG, "byte ranges need a plain (memory-mapped) file");
    if (begin < 0 || end < begin || (size_t)end > r->map_len) return fail(PCABI_E_ARG, "byte range outside the file");
    r->pos = (size_t)begin;
    r->end = (size_t)end;
    r->released = (size_t)begin & ~(size_t)4095;
    const size_t pg = (size_t)begin & ~(size_t)4095;
    if (end > begin) madvise((char *)r->map + pg, (size_t)end - pg, MADV_WILLNEED);
    r->eof = true;
    r->fa_have_name = false;
    r->fa_name.clear();
    r->fa_seq.clear();
    return 0;
}

void pcabi_fastx_close(pcabi_fastx *r) {
    if (!r) return;
    if (r->f) gzclose(r->f);
    r->ahead_stop = true;                 // the populate-ahead helper leaves the mapping first
    if (r->ahead.joinable()) r->ahead.join();
    if (r->map) {
        // tearing down a gigabyte mapping takes ~0.1 s: off the caller's path
        void *m = r->map;
        const size_t n = r->map_len;
        std::thread([m, n] { munmap(m, n); }).detach();
    }
    delete r;
}

int64_t pcabi_fastx_next(pcabi_fastx *r, int64_t max_reads, int64_t max_bases, pcabi_reads **out) {
    if (!r || !out || max_reads <= 0) return fail(PCABI_E_ARG, "bad arguments");
    if (r->map && !r->ahead.joinable() && r->end > r->pos + (64u << 20)) {
        // a large plain file read in batches: the helper maps pages ahead of the record scan
        r->reader_at.store(r->pos, std::memory_order_relaxed);
        r->ahead = std::thread(populate_ahead, r, r->pos & ~(size_t)4095, r->end);
    }
    pcabi_reads *b = new pcabi_reads();
    b->type = r->type;
    if (r->type != PCABI_FASTQ) {
        // FASTA appends record by record: sequence about the decoded bytes (FASTQ sizes its
        // buffers exactly from the record scan, fill_fastq)
        const size_t want = std::min<size_t>(r->size_hint / 2 + 4096, (size_t)std::min<int64_t>(max_bases, 1LL << 40));
        b->seq.reserve(want);
        b->codes.reserve(want + 4096);
    }
    int64_t bases = 0;
    const char *p;
    size_t n;
    // PCABI_IOPROF=1: per batch, the record scan's and the fill's milliseconds on stderr
    static const bool ioprof = [] {
        const char *e = std::getenv("PCABI_IOPROF");
        return e && e[0] == '1';
    }();
    const auto t_scan = std::chrono::steady_clock::now();
    if (r->type == PCABI_FASTQ) {
        std::vector<Span> rec;
        r->pin = r->pos;                 // the batch's bytes survive refills (shifted with the pin)
        auto rel = [&](const char *q) { return (size_t)(q - r->base) - r->pin; };
        while ((int64_t)rec.size() < max_reads && bases < max_bases) {
            if (!next_line(r, &p, &n)) break;
            strip(&p, &n);
            if (n == 0 || n == 1) {   // full_name.split()[0] fails in the reference (IndexError)
                delete b;
                r->pin = (size_t)-1;
                return fail(PCABI_E_PARSE, "could not be parsed - is it formatted correctly? (empty FASTQ header at line " +
                                               std::to_string(r->line_no) + ")");
            }
            Span sp{};
            sp.no = rel(p + 1);
            sp.nn = n - 1;
            const char *q;
            size_t qn;
            if (!next_line(r, &q, &qn)) { delete b; r->pin = (size_t)-1; return fail(PCABI_E_PARSE, "truncated FASTQ record"); }
            strip(&q, &qn);
            sp.so = rel(q);
            sp.sn = qn;
            if (!next_line(r, &q, &qn)) { delete b; r->pin = (size_t)-1; return fail(PCABI_E_PARSE, "truncated FASTQ record"); }
            if (r->raw) {
                strip(&q, &qn);
                sp.xo = rel(q);
                sp.xn = qn;
            }
            if (!next_line(r, &q, &qn)) { delete b; r->pin = (size_t)-1; return fail(PCABI_E_PARSE, "truncated FASTQ record"); }
            strip(&q, &qn);
            sp.qo = rel(q);
            sp.qn = qn;
            rec.push_back(sp);
            bases += (int64_t)sp.sn;
        }
        const auto t_fill = std::chrono::steady_clock::now();
        fill_fastq(b, r->base + r->pin, rec, r->raw);
        if (ioprof) {
            const auto t_end = std::chrono::steady_clock::now();
            std::fprintf(stderr, "[pcabi io] batch %zu reads: scan %.2f ms, fill %.2f ms\n", rec.size(),
                         std::chrono::duration<double, std::milli>(t_fill - t_scan).count(),
                         std::chrono::duration<double, std::milli>(t_end - t_fill).count());
        }
        r->pin = (size_t)-1;
    } else {
        while (b->n < max_reads && bases < max_bases) {
            if (!next_line(r, &p, &n)) {
                if (r->fa_have_name && !r->fa_name.empty()) {
                    add_record(b, r->fa_name.data(), r->fa_name.size(), r->fa_seq.data(), r->fa_seq.size(), "", 0, r->raw);
                    bases += (int64_t)r->fa_seq.size();
                }
                r->fa_have_name = false;
                r->fa_name.clear();
                r->fa_seq.clear();
                break;
            }
            strip(&p, &n);
            if (n == 0) continue;
            if (p[0] == '>') {
                if (!r->fa_name.empty()) {
                    add_record(b, r->fa_name.data(), r->fa_name.size(), r->fa_seq.data(), r->fa_seq.size(), "", 0, r->raw);
                    bases += (int64_t)r->fa_seq.size();
                    r->fa_seq.clear();
                }
                r->fa_name.assign(p + 1, n - 1);
                r->fa_have_name = true;
            } else {
                r->fa_seq.append(p, n);
            }
        }
    }
    if (r->err) {
        delete b;
        return PCABI_E_PARSE;   // the message is pcabi_last_error()'s (next_line)
    }
    if (r->map) r->reader_at.store(r->pos, std::memory_order_relaxed);
    if (r->map) {
        // the batch holds copies of its records: the page mappings of the file bytes it consumed
        // are dropped as the reader goes (madvise takes the address space's lock shared), so the
        // final munmap has nothing left to tear down -- a whole-file teardown held the lock
        // exclusively for ~50 ms and stalled every other thread's page faults (r05 e2e timeline).
        // The bytes stay in the page cache; a later read of them faults them back in.
        const size_t upto = r->pos & ~(size_t)4095;
        if (upto >= r->released + (32u << 20)) {
            madvise((char *)r->map + r->released, upto - r->released, MADV_DONTNEED);
            r->released = upto;
        }
    }
    finish_batch(b);
    *out = b;
    return b->n;
}

// The next span of the decoded text holding whole records, cut where a reader starting afresh
// parses the same records as the continuous read: FASTQ after a record whose successor's line
// starts with '@'; FASTA before a header with a name whose preceding header had one (an empty
// header's sequence runs on into the next record). At least max_bytes unless the input ends first
// (one record may overshoot). *text stays valid until the next call on r. Returns 1, 0 at the end.
int pcabi_fastx_next_text(pcabi_fastx *r, int64_t max_bytes, const char **text, int64_t *len) {
    if (!r || !text || !len || max_bytes <= 0) return fail(PCABI_E_ARG, "bad arguments");
    r->pin = r->pos;
    const char *p;
    size_t n;
    for (;;) {
        const size_t ls = r->pos - r->pin;           // this line's start, relative to the pin
        if (!next_line(r, &p, &n)) break;
        if (r->type == PCABI_FASTQ) {
            bool whole = true;
            for (int k = 0; k < 3 && whole; ++k) whole = next_line(r, &p, &n);
            if (!whole) break;                        // truncated: the chunk's reader reports it
            if ((int64_t)(r->pos - r->pin) >= max_bytes && r->pos < r->end && r->base[r->pos] == '@') break;
        } else {
            const char *q = p;
            size_t m = n;
            strip(&q, &m);
            if (m > 0 && q[0] == '>') {
                const int named = m > 1 ? 1 : 0;
                if ((int64_t)ls >= max_bytes && p[0] == '>' && named && r->txt_named == 1) {
                    r->pos = r->pin + ls;             // unread: the next span starts with this header
                    break;
                }
                r->txt_named = named;
            }
        }
    }
    *text = r->base + r->pin;
    *len = (int64_t)(r->pos - r->pin);
    r->pin = (size_t)-1;
    if (r->err) return PCABI_E_PARSE;
    return *len > 0 ? 1 : 0;
}

int pcabi_fastx_load(const char *path, int raw, pcabi_reads **out) {
    if (!out) return fail(PCABI_E_ARG, "bad arguments");
    *out = nullptr;
    pcabi_fastx *r = nullptr;
    if (int rc = pcabi_fastx_open(path, raw, &r)) return rc;
    pcabi_reads *all = nullptr;
    const int64_t got = pcabi_fastx_next(r, INT64_MAX, INT64_MAX, &all);
    pcabi_fastx_close(r);
    if (got < 0) return (int)got;
    *out = all;
    return 0;
}

void pcabi_reads_free(pcabi_reads *b) { delete b; }

void pcabi_gather_host(const uint8_t *src, const int64_t *src_off, const int32_t *len, int64_t n, uint8_t *dst,
                       const int64_t *dst_off) {
    for (int64_t i = 0; i < n; ++i)
        if (len[i] > 0) std::memcpy(dst + dst_off[i], src + src_off[i], (size_t)len[i]);
}

void pcabi_encode_dna5_gather(const uint64_t *src, const int64_t *len, const int64_t *dst_off, int64_t n,
                              uint8_t *codes, int64_t codes_len) {
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
    // segments [lo, hi) and the N gap after each (up to the next segment / codes_len)
    auto run = [&](int64_t lo, int64_t hi) {
        if (lo == 0 && n > 0) std::memset(codes, 4, (size_t)dst_off[0]);
        for (int64_t i = lo; i < hi; ++i) {
            const uint8_t *s = reinterpret_cast<const uint8_t *>(src[i]);
            uint8_t *d = codes + dst_off[i];
            for (int64_t k = 0; k < len[i]; ++k) d[k] = tab.t[s[k]];
            const int64_t end = i + 1 < n ? dst_off[i + 1] : codes_len;
            const int64_t gap = end - dst_off[i] - len[i];
            if (gap > 0) std::memset(d + len[i], 4, (size_t)gap);
        }
    };
    if (n <= 0) {
        if (codes_len > 0) std::memset(codes, 4, (size_t)codes_len);
        return;
    }
    // split by bytes, not by segments: chunk k starts at the first segment at or past k/nt of the total
    const int nt = (int)std::min<int64_t>(16, std::max<int64_t>(1, codes_len / (4 << 20)));
    if (nt <= 1) {
        run(0, n);
        return;
    }
    std::vector<int64_t> cut(nt + 1, n);
    cut[0] = 0;
    for (int k = 1; k < nt; ++k)
        cut[k] = std::lower_bound(dst_off, dst_off + n, codes_len * k / nt) - dst_off;
    std::vector<std::thread> th;
    for (int k = 0; k < nt; ++k)
        if (cut[k] < cut[k + 1]) th.emplace_back(run, cut[k], cut[k + 1]);
    for (auto &t : th) t.join();
}

int64_t pcabi_reads_count(const pcabi_reads *b) { return b ? b->n : 0; }
int pcabi_reads_type(const pcabi_reads *b) { return b ? b->type : -1; }

int pcabi_reads_views(const pcabi_reads *b, pcabi_reads_view *v) {
    if (!b || !v) return fail(PCABI_E_ARG, "bad arguments");
    v->n = b->n;
    v->type = b->type;
    v->names = b->names.data();
    v->name_off = b->name_off.data();
    v->seq = b->seq.data();
    v->seq_off = b->seq_off.data();
    v->qual = b->qual.data();
    v->qual_off = b->qual_off.data();
    v->rna = b->rna.data();
    v->spacer = b->spacer.data();
    v->spacer_off = b->spacer_off.data();
    v->codes = b->codes.data();
    v->codes_len = (int64_t)b->codes.size();
    v->code_off = b->code_off.data();
    v->len = b->len.data();
    return 0;
}

}  // extern "C"

// ---- writer ----------------------------------------------------------------------------------
namespace {

// Output sink. Plain files are written with writev straight from the batch's buffers (one
// copy, into the page cache); only text the writer makes itself (numbered names, U for T, FASTA
// line breaks) is staged in an arena first. gzip / stdout go through a buffer.
struct Sink {
    FILE *fp = nullptr;
    gzFile gz = nullptr;
    int fd = -1;
    std::string buf;
    std::vector<iovec> iov;
    std::vector<std::unique_ptr<char[]>> arena;
    size_t arena_left = 0;
    char *arena_p = nullptr;
    bool ok = true;
    void flush() {
        if (fd >= 0) {
            size_t k = 0;
            while (ok && k < iov.size()) {
                const int cnt = (int)std::min<size_t>(iov.size() - k, 1024);
                const ssize_t w = ::writev(fd, iov.data() + k, cnt);
                if (w < 0) {
                    if (errno == EINTR) continue;
                    ok = false;
                    break;
                }
                size_t left = (size_t)w;   // advance past what was written (partial writes)
                while (left > 0 && k < iov.size()) {
                    if (left >= iov[k].iov_len) {
                        left -= iov[k].iov_len;
                        ++k;
                    } else {
                        iov[k].iov_base = (char *)iov[k].iov_base + left;
                        iov[k].iov_len -= left;
                        left = 0;
                    }
                }
            }
            iov.clear();
            arena.clear();
            arena_left = 0;
            return;
        }
        if (buf.empty()) return;
        if (gz) ok = ok && gzwrite(gz, buf.data(), (unsigned)buf.size()) == (int)buf.size();
        else ok = ok && std::fwrite(buf.data(), 1, buf.size(), fp) == buf.size();
        buf.clear();
    }
    // bytes that stay valid until the next flush (the batch, string literals)
    void ref(const char *p, size_t n) {
        if (n == 0) return;
        if (fd < 0) {
            put(p, n);
            return;
        }
        iov.push_back(iovec{const_cast<char *>(p), n});
        if (iov.size() >= 8192) flush();
    }
    // bytes the caller may reuse: copied
    void put(const char *p, size_t n) {
        if (n == 0) return;
        if (fd >= 0) {
            if (n > arena_left) {
                const size_t sz = std::max<size_t>(n, 1 << 20);
                arena.emplace_back(new char[sz]);
                arena_p = arena.back().get();
                arena_left = sz;
            }
            std::memcpy(arena_p, p, n);
            iov.push_back(iovec{arena_p, n});
            arena_p += n;
            arena_left -= n;
            if (iov.size() >= 8192) flush();
            return;
        }
        buf.append(p, n);
        if (buf.size() > (8u << 20)) flush();
    }
    void put(const std::string &s) { put(s.data(), s.size()); }
    void put(char c) { put(&c, 1); }
};

// Python seq[start:end] with start >= 0 and end possibly negative (counts from the end).
inline void py_slice(int64_t len, int64_t start, int64_t end, int64_t *a, int64_t *b) {
    if (end < 0) end = std::max<int64_t>(0, len + end);
    if (end > len) end = len;
    if (start > len) start = len;
    *a = start;
    *b = std::max(start, end);
}

std::string numbered(const char *name, size_t nn, int k) {
    std::string s(name, nn);
    const std::string tag = "_" + std::to_string(k);
    size_t p = s.find('\t');
    if (p != std::string::npos) return s.substr(0, p) + tag + s.substr(p);
    p = s.find(' ');
    if (p != std::string::npos) return s.substr(0, p) + tag + s.substr(p);
    return s + tag;
}

// The parallel writer's two passes (pcabi_reads_write, plain files): CountSink sizes a range of
// records, MemSink copies them to their place in one contiguous output buffer.
struct CountSink {
    size_t n = 0;
    void ref(const char *, size_t k) { n += k; }
    void put(const char *, size_t k) { n += k; }
    void put(const std::string &x) { n += x.size(); }
    void put(char) { ++n; }
};
struct MemSink {
    char *p;
    void ref(const char *s, size_t k) {
        std::memcpy(p, s, k);
        p += k;
    }
    void put(const char *s, size_t k) { ref(s, k); }
    void put(const std::string &x) { ref(x.data(), x.size()); }
    void put(char c) { *p++ = c; }
};

template <class S>
void put_seq(S &o, const char *s, size_t n, bool rna, bool fasta) {
    std::string t;
    if (rna) {   // T -> U (a copy); otherwise the batch's bytes go out as they are
        t.assign(s, n);
        for (char &c : t)
            if (c == 'T') c = 'U';
        s = t.data();
    }
    if (!fasta) {
        if (rna) o.put(s, n);
        else o.ref(s, n);
        return;
    }
    for (size_t p = 0; p < n; p += 70) {   // add_line_breaks_to_sequence(seq, 70)
        if (rna) o.put(s + p, std::min<size_t>(70, n - p));
        else o.ref(s + p, std::min<size_t>(70, n - p));
        o.ref("\n", 1);
    }
}

// name: the batch's own header bytes (stable) or a numbered copy (own = true)
template <class S>
void put_record(S &o, bool fasta, const char *name, size_t nn, bool own, const char *s, size_t ns,
                const char *q, size_t nq, bool rna) {
    o.ref(fasta ? ">" : "@", 1);
    if (own) o.put(name, nn);
    else o.ref(name, nn);
    o.ref("\n", 1);
    if (fasta) {
        put_seq(o, s, ns, rna, true);
    } else {
        put_seq(o, s, ns, rna, false);
        o.ref("\n+\n", 3);
        o.ref(q, nq);
        o.ref("\n", 1);
    }
}

}  // namespace

extern "C" int pcabi_reads_write(const pcabi_reads *b, const char *path, int append, int gz, int fasta,
                                 const int32_t *start_trim, const int32_t *end_trim, const int64_t *cut_off,
                                 const int64_t *cuts, int min_split_read_size, int discard_middle,
                                 int untrimmed, const uint8_t *select) {
    if (!b || !path) return fail(PCABI_E_ARG, "bad arguments");
    Sink o;
    if (gz) {
        o.gz = gzopen(path, append ? "ab" : "wb");
        if (!o.gz) return fail(PCABI_E_ARG, std::string("could not write ") + path);
    } else if (std::strcmp(path, "-") == 0) {
        o.fp = stdout;
    } else {
        o.fd = ::open(path, O_WRONLY | O_CREAT | (append ? O_APPEND : O_TRUNC), 0666);
        if (o.fd < 0) return fail(PCABI_E_ARG, std::string("could not write ") + path);
    }
    // returns whether the read produced any output (the reference counts a read into its bin only
    // then, porechop_abi.py:598-604)
    auto format = [&](int64_t i, auto &o, std::vector<std::pair<int64_t, int64_t>> &rg) -> bool {
        if (select && !select[i]) return false;
        const char *name = b->names.data() + b->name_off[i];
        const size_t nn = (size_t)(b->name_off[i + 1] - b->name_off[i]);
        const char *seq = b->seq.data() + b->seq_off[i];
        const int64_t ns = b->seq_off[i + 1] - b->seq_off[i];
        const char *qual = b->qual.data() + b->qual_off[i];
        const int64_t nq = b->qual_off[i + 1] - b->qual_off[i];
        const bool rna = b->rna[i] != 0;
        const int64_t st = start_trim ? start_trim[i] : 0, et = end_trim ? end_trim[i] : 0;
        // get_seq_with_start_end_adapters_trimmed / get_quals_... (nanopore_read.py:66-82)
        int64_t sa = 0, sb = ns, qa = 0, qb = nq;
        if (st || et) {
            py_slice(ns, st, ns - et, &sa, &sb);
            py_slice(nq, st, nq - et, &qa, &qb);
        }
        bool split = false;
        if (cut_off)
            for (int64_t k = cut_off[i]; k < cut_off[i + 1] && !split; ++k) split = cuts[2 * k + 1] > cuts[2 * k];
        if (!split) {
            if (untrimmed) { sa = 0; sb = ns; qa = 0; qb = nq; }
            if (sb == sa) return false;   // no empty sequences
            put_record(o, fasta != 0, name, nn, false, seq + sa, (size_t)(sb - sa), qual + qa, (size_t)(qb - qa), rna);
            return true;
        }
        if (discard_middle) return false;
        // split parts (get_split_read_parts, nanopore_read.py:84-104): positions of the trimmed
        // sequence inside any cut range are dropped
        rg.clear();
        for (int64_t k = cut_off[i]; k < cut_off[i + 1]; ++k)
            if (cuts[2 * k + 1] > cuts[2 * k]) rg.emplace_back(cuts[2 * k], cuts[2 * k + 1]);
        std::sort(rg.begin(), rg.end());
        const int64_t tl = sb - sa;
        int part = 0;
        size_t ri = 0;
        int64_t run = 0;   // start of the current kept run
        auto emit = [&](int64_t a, int64_t e) {
            if (e - a <= 0 || e - a < min_split_read_size) return;
            ++part;
            const std::string nm = numbered(name, nn, part);
            put_record(o, fasta != 0, nm.data(), nm.size(), true, seq + sa + a, (size_t)(e - a), qual + qa + a,
                       (size_t)(e - a), rna);
        };
        int64_t pos = 0;
        while (pos < tl) {
            while (ri < rg.size() && rg[ri].second <= pos) ++ri;
            if (ri < rg.size() && rg[ri].first <= pos) {   // pos is cut
                emit(run, pos);
                int64_t e = rg[ri].second;
                for (size_t rj = ri; rj < rg.size() && rg[rj].first <= e; ++rj) e = std::max(e, rg[rj].second);
                pos = std::min(e, tl);
                run = pos;
            } else {
                const int64_t nxt = ri < rg.size() ? std::min(rg[ri].first, tl) : tl;
                pos = nxt;
            }
        }
        emit(run, tl);
        return part > 0;
    };
    // One stream: the page-cache copy is the cost, and writers of one file serialise on its
    // inode (measured: threads writing disjoint ranges with pwritev were no faster). r05: a plain
    // file's records are first laid out in one contiguous buffer by the io threads (a sizing pass,
    // then each thread copies its range of records to its offset), then written in large write()
    // calls -- a writev of ~7 small pieces per record spent more on the pieces than on the bytes
    // (e2e writer 8.1 GB/s against 11.9 for one contiguous buffer, bench write_probe).
    int64_t emitted = 0;
    const int nt = (int)std::min<int64_t>((int64_t)io_threads(), std::max<int64_t>(1, b->n / 512));
    if (o.fd >= 0 && b->n > 0) {
        std::vector<int64_t> lo((size_t)nt + 1), bytes((size_t)nt + 1, 0), emit((size_t)nt, 0);
        for (int t = 0; t <= nt; ++t) lo[(size_t)t] = b->n * t / nt;
        auto par = [&](auto &&fn) {
            if (nt <= 1) {
                fn(0);
                return;
            }
            std::vector<std::thread> th;
            for (int t = 0; t < nt; ++t) th.emplace_back(fn, t);
            for (auto &x : th) x.join();
        };
        par([&](int t) {
            std::vector<std::pair<int64_t, int64_t>> rg;
            CountSink c;
            for (int64_t i = lo[(size_t)t]; i < lo[(size_t)t + 1]; ++i) format(i, c, rg);
            bytes[(size_t)t + 1] = (int64_t)c.n;
        });
        for (int t = 0; t < nt; ++t) bytes[(size_t)t + 1] += bytes[(size_t)t];
        std::vector<char, NoInit<char>> out;
        out.resize((size_t)bytes[(size_t)nt]);
        par([&](int t) {
            std::vector<std::pair<int64_t, int64_t>> rg;
            MemSink m{out.data() + bytes[(size_t)t]};
            int64_t e = 0;
            for (int64_t i = lo[(size_t)t]; i < lo[(size_t)t + 1]; ++i) e += format(i, m, rg) ? 1 : 0;
            emit[(size_t)t] = e;
        });
        for (int t = 0; t < nt; ++t) emitted += emit[(size_t)t];
        size_t k = 0;
        while (o.ok && k < out.size()) {
            const ssize_t w = ::write(o.fd, out.data() + k, std::min<size_t>(out.size() - k, 256u << 20));
            if (w < 0) {
                if (errno == EINTR) continue;
                o.ok = false;
                break;
            }
            k += (size_t)w;
        }
    } else {
        std::vector<std::pair<int64_t, int64_t>> rg;
        for (int64_t i = 0; i < b->n; ++i) emitted += format(i, o, rg) ? 1 : 0;
    }
    o.flush();
    const bool ok = o.ok;
    if (o.gz) gzclose(o.gz);
    else if (o.fd >= 0) ::close(o.fd);
    else if (o.fp) std::fflush(o.fp);
    if (!ok) return fail(PCABI_E_ARG, std::string("write failed: ") + path);
    return (int)std::min<int64_t>(emitted, INT32_MAX);
}
