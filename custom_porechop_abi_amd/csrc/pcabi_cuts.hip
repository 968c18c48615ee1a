// pcabi_cuts.hip -- middle-adapter trim ranges on the device (porechop_abi/nanopore_read.py:233-250):
// every middle hit (read, adapter, read_start, read_end) becomes the range
//   [read_start - (adapter is a start sequence ? bad_side : good_side),
//    read_end   + (adapter is an end sequence   ? bad_side : good_side))
// of NanoporeRead.middle_trim_positions, grouped per read in discovery order (CSR: cut_off[r] ..
// cut_off[r + 1]), the layout pcabi_reads_write takes. The grouping is a stable radix sort of the
// hits by read, so each read keeps the reference's order of its own hits.
#include <hipcub/hipcub.hpp>

#include "pcabi_kern.h"

namespace pcabi_eng {
namespace {

__global__ __launch_bounds__(256) void k_hit_keys(const int32_t *hits, int64_t stride, int64_t n, int64_t n_reads,
                                                  uint32_t *key, uint32_t *idx, unsigned long long *count) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    const int32_t r = hits[k];
    key[k] = (uint32_t)r;
    idx[k] = (uint32_t)k;
    if (r >= 0 && r < n_reads) atomicAdd(&count[r], 1ull);
}

__global__ __launch_bounds__(256) void k_cut_ranges(const int32_t *hits, int64_t stride, const uint32_t *order,
                                                    int64_t n, const uint8_t *bad_start, const uint8_t *bad_end,
                                                    int good, int bad, int64_t *cuts) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t k = order[i];
    const int32_t a = hits[1 * stride + k];
    cuts[2 * i] = (int64_t)hits[2 * stride + k] - (bad_start[a] ? bad : good);
    cuts[2 * i + 1] = (int64_t)hits[3 * stride + k] + (bad_end[a] ? bad : good);
}

}  // namespace
}  // namespace pcabi_eng

using namespace pcabi_eng;

extern "C" int pcabi_middle_cuts_dev(const int32_t *hits, int64_t hit_stride, int64_t n_hits, int64_t n_reads,
                                     const uint8_t *bad_start, const uint8_t *bad_end, int good_side, int bad_side,
                                     int64_t *cut_off, int64_t *cuts, void *stream) {
    if (n_hits < 0 || n_reads < 0 || hit_stride < n_hits) return fail(PCABI_E_ARG, "bad hit counts");
    if (n_reads >= (1ll << 32)) return fail(PCABI_E_ARG, "too many reads");
    const hipStream_t st = (hipStream_t)stream;
    const size_t n = (size_t)n_hits, nr = (size_t)n_reads;
    // scratch: keys, values (in / out), per-read counts (+1 for the total), sort / scan temp
    size_t sort_tmp = 0, scan_tmp = 0;
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                               (uint32_t *)nullptr, (uint32_t *)nullptr, (int)std::max<size_t>(n, 1),
                                               0, 32, st));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, (unsigned long long *)nullptr,
                                             (unsigned long long *)nullptr, (int)(nr + 1), st));
    const size_t a4 = (4 * std::max<size_t>(n, 1) + 255) & ~(size_t)255;
    const size_t a8 = (8 * (nr + 1) + 255) & ~(size_t)255;
    const size_t tmp = std::max(sort_tmp, scan_tmp);
    char *buf = nullptr;
    HIP_TRY(hipMallocAsync((void **)&buf, 4 * a4 + a8 + tmp + 256, st));
    pcabi_poison_async(buf, 4 * a4 + a8 + tmp + 256, st);
    uint32_t *key = (uint32_t *)buf, *idx = (uint32_t *)(buf + a4), *key2 = (uint32_t *)(buf + 2 * a4),
             *order = (uint32_t *)(buf + 3 * a4);
    unsigned long long *count = (unsigned long long *)(buf + 4 * a4);
    void *t = buf + 4 * a4 + a8;
    int rc = 0;
    do {
        if (hipMemsetAsync(count, 0, 8 * (nr + 1), st) != hipSuccess) { rc = fail(PCABI_E_DEVICE, "memset"); break; }
        if (n) {
            hipLaunchKernelGGL(k_hit_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, hits, hit_stride,
                               n_hits, n_reads, key, idx, count);
            size_t ts = sort_tmp;
            if (hipcub::DeviceRadixSort::SortPairs(t, ts, key, key2, idx, order, (int)n, 0, 32, st) != hipSuccess) {
                rc = fail(PCABI_E_DEVICE, "radix sort of the middle hits");
                break;
            }
            hipLaunchKernelGGL(k_cut_ranges, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, hits, hit_stride,
                               order, n_hits, bad_start, bad_end, good_side, bad_side, cuts);
        }
        size_t ts = scan_tmp;
        if (hipcub::DeviceScan::ExclusiveSum(t, ts, count, (unsigned long long *)cut_off, (int)(nr + 1), st) !=
            hipSuccess) {
            rc = fail(PCABI_E_DEVICE, "scan of the per-read hit counts");
            break;
        }
        const hipError_t le = hipGetLastError();
        if (le != hipSuccess) rc = fail(PCABI_E_DEVICE, std::string("middle cuts: ") + hipGetErrorString(le));
    } while (0);
    HIP_TRY(hipFreeAsync(buf, st));
    return rc;
}
