// pcabi_decide.hip -- the end-trim decisions' alignment lists on the device
// (porechop_abi/nanopore_read.py:175-217): find_start_trim / find_end_trim append
// (adapter, full_id, partial_id, read_start, read_end) to a read's start / end_adapter_alignments for
// every alignment that trims (k_end_trim's per-pair flags). Instead of the whole result matrix
// (8 int32 per (read, adapter) pair), only those alignments leave the device: per side, read-major
// and in adapter order within a read -- the order the reference appends them in -- as 7 int32 rows
// (read, adapter, rs, re inclusive, m, l1, l2). Per-read counts, an exclusive scan (hipcub), then
// one thread per read writes its own alignments.
#include <hipcub/hipcub.hpp>

#include "pcabi_kern.h"

namespace pcabi_eng {
namespace {

__global__ __launch_bounds__(256) void k_flag_count(const uint8_t *flag, int32_t n_adp, int64_t n_read,
                                                    unsigned long long *count) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r > n_read) return;
    unsigned long long c = 0;
    if (r < n_read)
        for (int32_t a = 0; a < n_adp; ++a) c += flag[(int64_t)a * n_read + r];
    count[r] = c;                                  // count[n_read] = 0: the scan's total
}

__global__ __launch_bounds__(256) void k_flag_write(const uint8_t *flag, int32_t n_adp, int64_t n_read,
                                                    const int32_t *res, int64_t stride,
                                                    const unsigned long long *off, int32_t *out, int64_t cap) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n_read) return;
    int64_t k = (int64_t)off[r];
    for (int32_t a = 0; a < n_adp; ++a) {
        const int64_t i = (int64_t)a * n_read + r;
        if (!flag[i]) continue;
        if (k < cap) {
            out[0 * cap + k] = (int32_t)r;
            out[1 * cap + k] = a;
            out[2 * cap + k] = res[0 * stride + i];
            out[3 * cap + k] = res[1 * stride + i];
            out[4 * cap + k] = res[5 * stride + i];
            out[5 * cap + k] = res[6 * stride + i];
            out[6 * cap + k] = res[7 * stride + i];
        }
        ++k;
    }
}

}  // namespace
}  // namespace pcabi_eng

using namespace pcabi_eng;

// n_out (device, 1 x uint64): the side's alignment count; out (7 x cap int32) written when the
// count fits (the caller reads n_out, grows cap and calls again otherwise). Async on `stream`.
extern "C" int pcabi_flag_list_dev(const uint8_t *flag, int32_t n_adp, int64_t n_read, const int32_t *res,
                                   int64_t stride, int32_t *out, int64_t cap, unsigned long long *n_out,
                                   void *stream) {
    if (n_adp < 0 || n_read < 0 || cap < 0) return fail(PCABI_E_ARG, "bad counts");
    if (n_read >= (1ll << 31)) return fail(PCABI_E_ARG, "too many reads");
    const hipStream_t st = (hipStream_t)stream;
    const size_t nr = (size_t)n_read;
    size_t scan_tmp = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, (unsigned long long *)nullptr,
                                             (unsigned long long *)nullptr, (int)(nr + 1), st));
    const size_t a8 = (8 * (nr + 1) + 255) & ~(size_t)255;
    char *buf = nullptr;
    HIP_TRY(hipMallocAsync((void **)&buf, 2 * a8 + scan_tmp + 256, st));
    pcabi_poison_async(buf, 2 * a8 + scan_tmp + 256, st);
    unsigned long long *count = (unsigned long long *)buf, *off = (unsigned long long *)(buf + a8);
    void *t = buf + 2 * a8;
    int rc = 0;
    do {
        const unsigned grid = (unsigned)((nr + 1 + 255) / 256);
        hipLaunchKernelGGL(k_flag_count, dim3(grid), dim3(256), 0, st, flag, n_adp, n_read, count);
        size_t ts = scan_tmp;
        if (hipcub::DeviceScan::ExclusiveSum(t, ts, count, off, (int)(nr + 1), st) != hipSuccess) {
            rc = fail(PCABI_E_DEVICE, "scan of the per-read alignment counts");
            break;
        }
        if (hipMemcpyAsync(n_out, off + nr, 8, hipMemcpyDeviceToDevice, st) != hipSuccess) {
            rc = fail(PCABI_E_DEVICE, "alignment count copy");
            break;
        }
        if (nr)
            hipLaunchKernelGGL(k_flag_write, dim3((unsigned)((nr + 255) / 256)), dim3(256), 0, st, flag, n_adp, n_read,
                               res, stride, off, out, cap);
        const hipError_t le = hipGetLastError();
        if (le != hipSuccess) rc = fail(PCABI_E_DEVICE, std::string("alignment list: ") + hipGetErrorString(le));
    } while (0);
    HIP_TRY(hipFreeAsync(buf, st));
    return rc;
}
