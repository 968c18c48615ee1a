// pcabi_k_aux.hip -- the middle scan's packed-16 score filter (k_score_filter) and the striped
// bucket (k_align_striped, adapters over 128 bp).
#include "pcabi_kern.h"

namespace pcabi_eng {

template <int RPL>
void launch_filter(const FParams &p, bool affine, hipStream_t st) {
    const int64_t tiles8 = (p.n_win + 8 * 256 - 1) / (8 * 256) * 8;
    const dim3 grid((unsigned)(tiles8 * ((p.n_adp + 1) / 2)));
    if (affine) hipLaunchKernelGGL((k_score_filter<RPL, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((k_score_filter<RPL, false>), grid, dim3(256), 0, st, p);
}

void dispatch_filter(int rpl, const FParams &p, bool affine, hipStream_t st) {
    switch (rpl) {
#define C(R) case R: launch_filter<R>(p, affine, st); break;
    C(4) C(8) C(12) C(16) C(20) C(24) C(28) C(32) C(36) C(40) C(44) C(48) C(52) C(56) C(60) C(64)
    C(68) C(72) C(76) C(80) C(84) C(88)
#undef C
    }
}

// Scratch budget of one striped launch (PCABI_STRIPE_SCRATCH_MB, default 4096): it bounds the wave
// slots when windows are long (each slot holds a boundary row as long as the longest window).
const int64_t g_stripe_budget = [] {
    const char *e = std::getenv("PCABI_STRIPE_SCRATCH_MB");
    const int64_t mb = (e && e[0]) ? std::max<int64_t>(16, std::atoll(e)) : 4096;
    return mb << 20;
}();

// Launch the striped kernel for one bucket: p.rt, p.max_cols set by the caller; scratch is
// stream-ordered (hipMallocAsync / hipFreeAsync on `st`), so concurrent launches never share it.
int launch_striped(KParams p, bool affine, hipStream_t st) {
    p.n_items = p.task_win ? p.n_waves : (p.n_win + 63) / 64 * p.n_adp;
    if (p.n_items <= 0) return 0;
    const int64_t nf = affine ? 6 : 3;
    const int64_t per_slot = std::max<int64_t>(1, p.max_cols) * nf * 64 * 4;
    int64_t slots = std::min<int64_t>({(p.n_items + 3) / 4 * 4, (int64_t)2048, g_stripe_budget / per_slot / 4 * 4});
    slots = std::max<int64_t>(slots, 4);
    void *scr = nullptr;
    // slots past the last item never touch their scratch
    HIP_TRY(hipMallocAsync(&scr, (size_t)(std::min(slots, p.n_items) * per_slot), st));
    pcabi_poison_async(scr, (size_t)(std::min(slots, p.n_items) * per_slot), st);
    p.scratch = (int32_t *)scr;
    p.max_cols = std::max<int32_t>(1, p.max_cols);
    const dim3 grid((unsigned)(slots / 4));
    if (affine) hipLaunchKernelGGL((k_align_striped<kStripeRows, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((k_align_striped<kStripeRows, false>), grid, dim3(256), 0, st, p);
    const hipError_t le = hipGetLastError();
    HIP_TRY(hipFreeAsync(scr, st));
    if (le != hipSuccess) return fail(PCABI_E_DEVICE, std::string("k_align_striped: ") + hipGetErrorString(le));
    return 0;
}


}  // namespace pcabi_eng
