// pcabi_kmer.hip -- the ab-initio k-mer counts of approx_counter on the GPU (gfx950).
//
// Reference: porechop_abi/ab_initio_src/approx_counter.cpp
//   count_kmers (:487-519)  exact count of every k-mer of the sampled read ends that holds no N
//                           (is_DNA, :313-321), is not low-complexity (haveLowComplexity, DUST-like
//                           dimer score, :214-234) and not forbidden (:330-332);
//   errorCount (:531-601)   for each kept k-mer, SeqAn's FM-index search at edit distance <= 2
//                           over the sampled sequences, counting per sequence one hit for every
//                           error level it is found at. A sequence whose best substring is at edit
//                           distance d <= 2 is reported at d, d+1, ..., 2 errors, so the k-mer's
//                           count is sum over sequences of (3 - d) for d <= 2 (checked against the
//                           reference binary on every k-mer of its outputs: tests/golden/g5_kmer).
// Kernels (HBM / integer work, no MFMA):
//   k_kmer_keys   one block per sequence, one lane per position: 2-bit key (first base in the
//                 top bits, dna2int :55-62) or the sentinel ~0 for a skipped position;
//   hipcub radix sort + run-length encode -> (k-mer, count);
//   k_kmer_approx one lane per k-mer, the block's sequences walked with wave-uniform bases:
//                 Myers' bit-vector edit distance with a free text start (pattern <= 32 bases in
//                 one register), the minimum over text ends, summed per k-mer.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/pcabi.h"

namespace pcabi_internal {
int fail(int code, const std::string &msg);
}
using pcabi_internal::fail;

#define KM_TRY(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) return fail(PCABI_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

namespace {

constexpr uint64_t kSkip = ~0ull;

// haveLowComplexity (approx_counter.cpp:214-234): counts[16] of the k-1 dimers, sum of
// v (v - 1) over them == twice the number of equal dimer pairs; s = sum / float(2 (k - 2)).
__device__ __forceinline__ bool low_complexity(uint64_t kmer, int k, float thr) {
    uint32_t pairs = 0;
    for (int i = 0; i < k - 1; ++i) {
        const uint32_t a = (uint32_t)(kmer >> (2 * i)) & 15u;
        for (int j = i + 1; j < k - 1; ++j) pairs += ((uint32_t)(kmer >> (2 * j)) & 15u) == a;
    }
    const float s = (float)(2u * pairs) / (float)(2 * (k - 2));
    return s >= thr;
}

__global__ __launch_bounds__(256) void k_kmer_keys(const uint8_t *codes, const int64_t *seq_off, const int32_t *seq_len,
                                                   const int64_t *key_off, int k, float thr, const uint64_t *forb,
                                                   int64_t n_forb, uint64_t *keys) {
    const int64_t s = blockIdx.x;
    const int n = seq_len[s];
    const int n_pos = n - k + 1;
    const uint8_t *c = codes + seq_off[s];
    for (int p = threadIdx.x; p < n_pos; p += blockDim.x) {
        uint64_t v = 0;
        bool dna = true;
        for (int i = 0; i < k; ++i) {
            const uint32_t x = c[p + i];
            dna = dna && x < 4;
            v = (v << 2) | (x & 3u);
        }
        uint64_t key = kSkip;
        if (dna && !low_complexity(v, k, thr)) {
            int64_t lo = 0, hi = n_forb;   // isForbiddenKmer: sorted set lookup
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (forb[mid] < v) lo = mid + 1;
                else hi = mid;
            }
            if (!(lo < n_forb && forb[lo] == v)) key = v;
        }
        keys[key_off[s] + p] = key;
    }
}

// One wave per block: lane = k-mer (blockIdx.y picks a group of 64), the block walks
// kSeqPerBlock sequences whose bases are wave-uniform (scalar loads, no per-lane gather).
// Myers (1999) with D[0][j] = 0 (free text start): the score tracked is D[k][j]; the minimum over
// j is the best substring's edit distance.
constexpr int kSeqPerBlock = 32;

__global__ __launch_bounds__(64) void k_kmer_approx(const uint8_t *codes, const int64_t *seq_off,
                                                    const int32_t *seq_len, int64_t n_seq, const uint64_t *kmers,
                                                    int64_t n_kmers, int k, unsigned long long *counts) {
    const int64_t q = (int64_t)blockIdx.y * 64 + threadIdx.x;
    const uint64_t km = q < n_kmers ? kmers[q] : 0;
    uint32_t p0 = 0, p1 = 0, p2 = 0, p3 = 0;
    for (int i = 0; i < k; ++i) {                     // pattern base i = bits of position k-1-i
        const uint32_t b = (uint32_t)(km >> (2 * (k - 1 - i))) & 3u;
        const uint32_t bit = 1u << i;
        p0 |= b == 0 ? bit : 0u;
        p1 |= b == 1 ? bit : 0u;
        p2 |= b == 2 ? bit : 0u;
        p3 |= b == 3 ? bit : 0u;
    }
    const uint32_t mask = k == 32 ? 0xFFFFFFFFu : ((1u << k) - 1u);
    const uint32_t high = 1u << (k - 1);
    unsigned long long acc = 0;
    const int64_t s0 = (int64_t)blockIdx.x * kSeqPerBlock;
    const int64_t s1 = s0 + kSeqPerBlock < n_seq ? s0 + kSeqPerBlock : n_seq;
    for (int64_t s = s0; s < s1; ++s) {
        // sequences start 4-aligned (approx_counter.sample_sequences packs them): dword loads of
        // wave-uniform addresses, four bases each
        const uint32_t *c = reinterpret_cast<const uint32_t *>(codes + seq_off[s]);
        const int n = seq_len[s];
        uint32_t pv = mask, mv = 0;
        int score = k, best = k;
        for (int j0 = 0; j0 < n; j0 += 4) {
            const uint32_t w = c[j0 >> 2];
            const int nb = n - j0 < 4 ? n - j0 : 4;
            for (int b = 0; b < nb; ++b) {
                const uint32_t x = (w >> (8 * b)) & 0xFFu;   // wave-uniform
                const uint32_t eq = x == 0 ? p0 : (x == 1 ? p1 : (x == 2 ? p2 : (x == 3 ? p3 : 0u)));
                const uint32_t xv = eq | mv;
                const uint32_t xh = ((((eq & pv) + pv) & mask) ^ pv) | eq;
                uint32_t ph = mv | (~(xh | pv) & mask);
                uint32_t mh = pv & xh;
                score += (ph & high) ? 1 : ((mh & high) ? -1 : 0);
                ph = (ph << 1) & mask;
                mh = (mh << 1) & mask;
                pv = mh | (~(xv | ph) & mask);
                mv = ph & xv;
                best = score < best ? score : best;
            }
        }
        acc += best <= 2 ? (unsigned long long)(3 - best) : 0ull;
    }
    if (q < n_kmers && acc) atomicAdd(&counts[q], acc);
}

struct DevMem {
    std::vector<void *> ptrs;
    ~DevMem() {
        for (void *p : ptrs) (void)hipFree(p);
    }
    template <typename T>
    int alloc(T **p, size_t n) {
        void *q = nullptr;
        if (hipMalloc(&q, std::max<size_t>(n * sizeof(T), 16)) != hipSuccess) return fail(PCABI_E_NOMEM, "hipMalloc failed");
        ptrs.push_back(q);
        *p = (T *)q;
        return 0;
    }
};

int check_seqs(int64_t codes_len, const int64_t *seq_off, const int32_t *seq_len, int64_t n_seq, int k) {
    if (n_seq < 0 || k < 2 || k > 32) return fail(PCABI_E_ARG, "k-mer size must be between 2 and 32, n_seq >= 0");
    for (int64_t s = 0; s < n_seq; ++s)
        if (seq_len[s] < 0 || seq_off[s] < 0 || seq_off[s] + seq_len[s] > codes_len)
            return fail(PCABI_E_ARG, "sequence outside the code buffer");
    return 0;
}

}  // namespace

extern "C" {

int64_t pcabi_kmer_count_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *seq_off,
                              const int32_t *seq_len, int64_t n_seq, int k, float lc_threshold,
                              const uint64_t *forbidden_sorted, int64_t n_forbidden, uint64_t *kmers,
                              uint32_t *counts, int64_t cap) {
    return pcabi_kmer_top_host(device, codes, codes_len, seq_off, seq_len, n_seq, k, lc_threshold, forbidden_sorted,
                               n_forbidden, -1, 0, kmers, counts, cap);
}

int64_t pcabi_kmer_top_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *seq_off,
                            const int32_t *seq_len, int64_t n_seq, int k, float lc_threshold,
                            const uint64_t *forbidden_sorted, int64_t n_forbidden, int64_t top, int64_t min_count,
                            uint64_t *kmers, uint32_t *counts, int64_t cap) {
    if (int rc = check_seqs(codes_len, seq_off, seq_len, n_seq, k)) return rc;
    if (n_forbidden < 0 || cap < 0) return fail(PCABI_E_ARG, "negative count");
    KM_TRY(hipSetDevice(device));
    std::vector<int64_t> key_off((size_t)n_seq + 1, 0);
    for (int64_t s = 0; s < n_seq; ++s) key_off[s + 1] = key_off[s] + std::max(0, seq_len[s] - k + 1);
    const int64_t n_keys = key_off[n_seq];
    if (n_keys == 0) return 0;
    if (n_keys > INT32_MAX) return fail(PCABI_E_ARG, "too many k-mer positions for one call");
    DevMem m;
    uint8_t *d_codes;
    int64_t *d_off, *d_koff;
    int32_t *d_len;
    uint64_t *d_forb, *d_keys, *d_sorted, *d_unique;
    uint32_t *d_counts;
    int32_t *d_nruns;
    if (int rc = m.alloc(&d_codes, (size_t)codes_len)) return rc;
    if (int rc = m.alloc(&d_off, (size_t)n_seq)) return rc;
    if (int rc = m.alloc(&d_len, (size_t)n_seq)) return rc;
    if (int rc = m.alloc(&d_koff, (size_t)n_seq + 1)) return rc;
    if (int rc = m.alloc(&d_forb, (size_t)n_forbidden)) return rc;
    if (int rc = m.alloc(&d_keys, (size_t)n_keys)) return rc;
    if (int rc = m.alloc(&d_sorted, (size_t)n_keys)) return rc;
    if (int rc = m.alloc(&d_unique, (size_t)n_keys)) return rc;
    if (int rc = m.alloc(&d_counts, (size_t)n_keys)) return rc;
    if (int rc = m.alloc(&d_nruns, 1)) return rc;
    KM_TRY(hipMemcpy(d_codes, codes, (size_t)codes_len, hipMemcpyHostToDevice));
    KM_TRY(hipMemcpy(d_off, seq_off, sizeof(int64_t) * n_seq, hipMemcpyHostToDevice));
    KM_TRY(hipMemcpy(d_len, seq_len, sizeof(int32_t) * n_seq, hipMemcpyHostToDevice));
    KM_TRY(hipMemcpy(d_koff, key_off.data(), sizeof(int64_t) * (n_seq + 1), hipMemcpyHostToDevice));
    if (n_forbidden) KM_TRY(hipMemcpy(d_forb, forbidden_sorted, sizeof(uint64_t) * n_forbidden, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_kmer_keys, dim3((unsigned)n_seq), dim3(128), 0, 0, d_codes, d_off, d_len, d_koff, k,
                       lc_threshold, d_forb, n_forbidden, d_keys);
    KM_TRY(hipGetLastError());
    size_t tmp_sort = 0, tmp_rle = 0;
    // keys use 2k bits; the sentinel ~0 has bit 2k set, so it sorts last
    const int end_bit = 2 * k < 64 ? 2 * k + 1 : 64;
    KM_TRY(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp_sort, d_keys, d_sorted, (int)n_keys, 0, end_bit));
    KM_TRY(hipcub::DeviceRunLengthEncode::Encode(nullptr, tmp_rle, d_sorted, d_unique, d_counts, d_nruns, (int)n_keys));
    void *d_tmp = nullptr;
    if (int rc = m.alloc((char **)&d_tmp, std::max(tmp_sort, tmp_rle))) return rc;
    KM_TRY(hipcub::DeviceRadixSort::SortKeys(d_tmp, tmp_sort, d_keys, d_sorted, (int)n_keys, 0, end_bit));
    KM_TRY(hipcub::DeviceRunLengthEncode::Encode(d_tmp, tmp_rle, d_sorted, d_unique, d_counts, d_nruns, (int)n_keys));
    int32_t nruns = 0;
    KM_TRY(hipMemcpy(&nruns, d_nruns, sizeof(int32_t), hipMemcpyDeviceToHost));
    uint64_t last = 0;
    if (nruns > 0) KM_TRY(hipMemcpy(&last, d_unique + nruns - 1, sizeof(uint64_t), hipMemcpyDeviceToHost));
    int64_t n_unique = nruns;
    if (nruns > 0 && (last == kSkip || (2 * k < 64 && (last >> (2 * k)) != 0))) --n_unique;   // the skipped positions
    if (top < 0) {                                     // every k-mer, ascending
        if (n_unique > cap) return n_unique;
        if (n_unique) {
            KM_TRY(hipMemcpy(kmers, d_unique, sizeof(uint64_t) * n_unique, hipMemcpyDeviceToHost));
            KM_TRY(hipMemcpy(counts, d_counts, sizeof(uint32_t) * n_unique, hipMemcpyDeviceToHost));
        }
        return n_unique;
    }
    if (n_unique == 0) return 0;
    // count descending (a stable radix sort: equal counts stay k-mer ascending), then only the
    // prefix that can matter leaves the device
    uint32_t *d_cnt2;
    uint64_t *d_km2;
    if (int rc = m.alloc(&d_cnt2, (size_t)n_unique)) return rc;
    if (int rc = m.alloc(&d_km2, (size_t)n_unique)) return rc;
    size_t tmp_pairs = 0;
    KM_TRY(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp_pairs, d_counts, d_cnt2, d_unique, d_km2,
                                                        (int)n_unique, 0, 32));
    void *d_tmp2 = nullptr;
    if (int rc = m.alloc((char **)&d_tmp2, tmp_pairs)) return rc;
    KM_TRY(hipcub::DeviceRadixSort::SortPairsDescending(d_tmp2, tmp_pairs, d_counts, d_cnt2, d_unique, d_km2,
                                                        (int)n_unique, 0, 32));
    uint32_t thr = (uint32_t)std::max<int64_t>(min_count, 0);
    if (top > 0 && top <= n_unique) {
        uint32_t cut = 0;
        KM_TRY(hipMemcpy(&cut, d_cnt2 + top - 1, sizeof(uint32_t), hipMemcpyDeviceToHost));
        thr = std::max(thr, cut);
    }
    // entries with count >= thr: a binary search over the descending counts
    int64_t lo = 0, hi = n_unique;   // first index with count < thr lies in [lo, hi]
    while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        uint32_t c = 0;
        KM_TRY(hipMemcpy(&c, d_cnt2 + mid, sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (c >= thr) lo = mid + 1;
        else hi = mid;
    }
    const int64_t n_out = lo;
    if (n_out > cap) return n_out;
    if (n_out) {
        KM_TRY(hipMemcpy(kmers, d_km2, sizeof(uint64_t) * n_out, hipMemcpyDeviceToHost));
        KM_TRY(hipMemcpy(counts, d_cnt2, sizeof(uint32_t) * n_out, hipMemcpyDeviceToHost));
    }
    return n_out;
}

int pcabi_kmer_approx_host(int device, const uint8_t *codes, int64_t codes_len, const int64_t *seq_off,
                           const int32_t *seq_len, int64_t n_seq, int k, const uint64_t *kmers, int64_t n_kmers,
                           uint64_t *counts) {
    if (int rc = check_seqs(codes_len, seq_off, seq_len, n_seq, k)) return rc;
    if (n_kmers < 0 || n_kmers > 65535 * 64) return fail(PCABI_E_ARG, "too many k-mers for one call");
    for (int64_t s = 0; s < n_seq; ++s)
        if (seq_off[s] & 3) return fail(PCABI_E_ARG, "sequences must start at 4-aligned offsets");
    if (codes_len & 3) return fail(PCABI_E_ARG, "the code buffer must be a multiple of 4 bytes (N padding)");
    for (int64_t q = 0; q < n_kmers; ++q) counts[q] = 0;
    if (n_kmers == 0 || n_seq == 0) return 0;
    KM_TRY(hipSetDevice(device));
    DevMem m;
    uint8_t *d_codes;
    int64_t *d_off;
    int32_t *d_len;
    uint64_t *d_kmers;
    unsigned long long *d_counts;
    if (int rc = m.alloc(&d_codes, (size_t)codes_len)) return rc;
    if (int rc = m.alloc(&d_off, (size_t)n_seq)) return rc;
    if (int rc = m.alloc(&d_len, (size_t)n_seq)) return rc;
    if (int rc = m.alloc(&d_kmers, (size_t)n_kmers)) return rc;
    if (int rc = m.alloc(&d_counts, (size_t)n_kmers)) return rc;
    KM_TRY(hipMemcpy(d_codes, codes, (size_t)codes_len, hipMemcpyHostToDevice));
    KM_TRY(hipMemcpy(d_off, seq_off, sizeof(int64_t) * n_seq, hipMemcpyHostToDevice));
    KM_TRY(hipMemcpy(d_len, seq_len, sizeof(int32_t) * n_seq, hipMemcpyHostToDevice));
    KM_TRY(hipMemcpy(d_kmers, kmers, sizeof(uint64_t) * n_kmers, hipMemcpyHostToDevice));
    KM_TRY(hipMemset(d_counts, 0, sizeof(unsigned long long) * n_kmers));
    const dim3 grid((unsigned)((n_seq + kSeqPerBlock - 1) / kSeqPerBlock), (unsigned)((n_kmers + 63) / 64));
    hipLaunchKernelGGL(k_kmer_approx, grid, dim3(64), 0, 0, d_codes, d_off, d_len, n_seq, d_kmers, n_kmers, k,
                       d_counts);
    KM_TRY(hipGetLastError());
    KM_TRY(hipMemcpy(counts, d_counts, sizeof(uint64_t) * n_kmers, hipMemcpyDeviceToHost));
    return 0;
}

}  // extern "C"
