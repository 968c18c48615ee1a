// pcabi_k_split_chunk.hip -- k_align_split_chunk instantiations: the row-split core (pcabi_dp.h
// LaneSplit) on the middle scan's device-planned chunk tasks, K = 2 lanes per task (the candidate
// windows' rounds, pcabi_engine.hip; K = 4 measured slower in r05), run-tagged buckets of 8..32 rows
// (affine) and packed buckets of 8..64 rows (affine and linear).
#include "pcabi_kern.h"

namespace pcabi_eng {

namespace {
template <int RPL, int K>
bool go(const KParams &p, bool affine, bool tagged, dim3 grid, hipStream_t st) {
    if constexpr (RPL % K != 0 || RPL / K < 2) {
        return false;
    } else {
        if (tagged) {
            if constexpr (RPL <= 32) {
                if (!affine) return false;
                hipLaunchKernelGGL((k_align_split_chunk<RPL, K, true, TAGGED>), grid, dim3(256), 0, st, p);
                return true;
            }
            return false;
        }
        if (affine) hipLaunchKernelGGL((k_align_split_chunk<RPL, K, true, PACKED>), grid, dim3(256), 0, st, p);
        else hipLaunchKernelGGL((k_align_split_chunk<RPL, K, false, PACKED>), grid, dim3(256), 0, st, p);
        return true;
    }
}
}  // namespace

bool dispatch_split_chunk(int rpl, int K, const KParams &p, bool affine, bool tagged, hipStream_t st) {
    if (!p.dev_waves) return false;                      // device-planned launches only
    const dim3 grid((unsigned)p.n_waves);                // blocks striding over the planned waves
    switch (rpl) {
#define C(R) case R: return K == 2 ? go<R, 2>(p, affine, tagged, grid, st) : false;
    C(8) C(12) C(16) C(20) C(24) C(28) C(32) C(36) C(40) C(44) C(48) C(52) C(56) C(60) C(64)
#undef C
    default: return false;
    }
}

}  // namespace pcabi_eng
