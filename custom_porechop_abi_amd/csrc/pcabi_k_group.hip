// pcabi_k_group.hip -- grouped cross-mode launches (pcabi_kern.h "grouped cross launches"): the
// units of one core family, each a (window set, register bucket) cross product, in one launch.
// The block's unit is found by a scalar walk over the segment table in the kernel arguments; the
// unit's rows select the core (a wave-uniform switch), which then runs exactly as k_align's cross
// mode (cross_block). The kernel's register count is its largest case's: class 0 (run-tagged, <= 32
// rows) holds 5 waves per SIMD, class 1 (packed, 36..64 rows) 3.
#include "pcabi_kern.h"

namespace pcabi_eng {

template <int CLS>
__global__ __launch_bounds__(256) void k_align_group(GroupParams gp) {
    constexpr int MAXR = group_max_rpl(CLS);
    __shared__ __attribute__((aligned(16))) int32_t tab[4 * kTabW * MAXR];
    int32_t *wave_tab = tab + (threadIdx.x >> 6) * kTabW * MAXR;
    const int64_t b = blockIdx.x;
    int s = 0;
    while (s + 1 < gp.n_seg && b >= gp.seg[s + 1].block0) ++s;
    const GroupSeg &g = gp.seg[s];
    KParams p{};
    p.tiles = g.tiles;
    p.tile_off = g.tile_off;
    p.win_len = g.win_len;
    p.n_win = g.n_win;
    p.adp_pad = g.adp_pad;
    p.adp_len = g.adp_len;
    p.adp_id = g.adp_id;
    p.n_adp = g.n_adp;
    p.out = g.out;
    p.out_stride = g.out_stride;
    p.sc = gp.sc;
    const int64_t lb = b - g.block0;
    if constexpr (CLS == 0) {
        switch (g.rpl) {
#define T(R) case R: cross_block<R, true, TAGGED>(p, lb, wave_tab); break;
        T(4) T(8) T(12) T(16) T(20) T(24) T(28) T(32)
#undef T
        }
    } else {
        switch (g.rpl) {
#define P(R) case R: cross_block<R, true, PACKED>(p, lb, wave_tab); break;
        P(36) P(40) P(44) P(48) P(52) P(56) P(60) P(64)
#undef P
        }
    }
}

void dispatch_group(int cls, const GroupParams &p, int64_t blocks, hipStream_t st) {
    if (blocks <= 0) return;
    if (cls == 0) hipLaunchKernelGGL((k_align_group<0>), dim3((unsigned)blocks), dim3(256), 0, st, p);
    else hipLaunchKernelGGL((k_align_group<1>), dim3((unsigned)blocks), dim3(256), 0, st, p);
}

}  // namespace pcabi_eng
