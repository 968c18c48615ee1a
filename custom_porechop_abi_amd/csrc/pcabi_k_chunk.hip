// pcabi_k_chunk.hip -- k_align_chunk instantiations: the middle scan's candidate DP over
// owned-column chunks of long reads (pcabi_dp.h sf::chunk_plan), every core.
#include "pcabi_kern.h"

namespace pcabi_eng {

// pcabi_kern.h "grouped candidate-DP launches". PCABI_CG_WAVES (build macro, A/B variants): the
// launch's minimum waves per SIMD (5: <= 96 VGPRs, a few dwords spilled outside the column loop)
#ifndef PCABI_CG_WAVES
#define PCABI_CG_WAVES 5
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(PCABI_CG_WAVES))) void k_align_chunk_group(ChunkGroupParams gp) {
    __shared__ __attribute__((aligned(16))) int32_t tab[wave_tab_ints<TAGGED, kChunkGroupRpl>()];
    for (int64_t g = blockIdx.x;; g += gridDim.x) {     // block-uniform (one wave per block)
        int s = 0;
        int64_t base = 0;
        for (; s < gp.n_seg; ++s) {
            const int64_t nw = gp.seg[s].dev_waves[1];
            if (g < base + nw) break;
            base += nw;
        }
        if (s == gp.n_seg) return;
        const ChunkSeg &sg = gp.seg[s];
        KParams p = gp.p;
        p.adp_pad = sg.adp_pad;
        p.adp_len = sg.adp_len;
        p.adp_id = sg.adp_id;
        p.n_adp = sg.n_adp;
        const int64_t wave = sg.dev_waves[0] + (g - base);
        switch (sg.rpl) {
#define C(R) case R: chunk_wave<R, true, TAGGED>(p, wave, true, tab); break;
        C(4) C(8) C(12) C(16) C(20) C(24) C(28)
#undef C
        }
    }
}

void dispatch_chunk_group(const ChunkGroupParams &gp, unsigned blocks, hipStream_t st) {
    if (gp.n_seg > 0) hipLaunchKernelGGL(k_align_chunk_group, dim3(blocks), dim3(64), 0, st, gp);
}

int dispatch_chunk(int b, const KParams &p, bool affine, hipStream_t st, bool tagged) {
    // planned on the device: n_waves is the grid (blocks striding over the device wave count)
    const dim3 grid((unsigned)(p.dev_waves ? p.n_waves : (p.n_waves + 3) / 4));
    if (kBuckets[b].kind == STRIPED) return launch_striped(p, affine, st);
    {   // the row-split core, K lanes per chunk task: p.chunk_split, the caller's choice (r05: 2 for
        // the middle scan's certified-out whole reads, whose 32-column chunks behind a ~60-column
        // lead-in ran latency-bound one lane per chunk)
        const int ks = p.chunk_split;
        if ((ks == 2 || ks == 4) && kBuckets[b].kind == FAST && kBuckets[b].rpl <= 64 &&
            pcabi::split_ok(kBuckets[b].rpl, ks) &&
            dispatch_split_chunk(kBuckets[b].rpl, ks, p, affine, tagged && affine && kBuckets[b].rpl <= 32, st))
            return 0;
    }
    // one-wave blocks for the device-planned run-tagged / packed buckets, 4x the blocks (the same
    // wave slots): r04n, candidate DP 0.68 -> 0.62 ms per 8 kb step, the reference job's middle
    // 1.57-1.59 -> 1.52 ms.
    const bool wpb1 = p.dev_waves && kBuckets[b].kind == FAST && affine;
    const dim3 grid1(grid.x * 4);
    if (wpb1 && tagged && kBuckets[b].rpl <= 32) {
        switch (kBuckets[b].rpl) {
#define C(R) case R: hipLaunchKernelGGL((k_align_chunk<R, true, TAGGED, 1, 1>), grid1, dim3(64), 0, st, p); return 0;
        C(4) C(8) C(12) C(16) C(20) C(24) C(28) C(32)
#undef C
        }
    }
    if (wpb1 && !tagged) {
        switch (kBuckets[b].rpl) {
#define C(R) case R: hipLaunchKernelGGL((k_align_chunk<R, true, PACKED, 1, 1>), grid1, dim3(64), 0, st, p); return 0;
        C(4) C(8) C(12) C(16) C(20) C(24) C(28) C(32) C(36) C(40) C(44) C(48) C(52) C(56) C(60) C(64)
#undef C
        }
    }
    if (tagged && affine && kBuckets[b].kind == FAST && kBuckets[b].rpl <= 32) {
        // the run-tagged layout (9 VALU ops per cell instead of 10), as the end-window buckets
        switch (kBuckets[b].rpl) {
#define C(R) case R: hipLaunchKernelGGL((k_align_chunk<R, true, TAGGED>), grid, dim3(256), 0, st, p); return 0;
        C(4) C(8) C(12) C(16) C(20) C(24) C(28) C(32)
#undef C
        }
    }
    if (kBuckets[b].kind == GENERIC) {
        switch (kBuckets[b].rpl) {
#define C(R)                                                                                            \
    case R:                                                                                             \
        if (affine) hipLaunchKernelGGL((k_align_chunk<R, true, GENERIC>), grid, dim3(256), 0, st, p);   \
        else hipLaunchKernelGGL((k_align_chunk<R, false, GENERIC>), grid, dim3(256), 0, st, p);         \
        break;
        C(16) C(32) C(64) C(96) C(128)
#undef C
        }
        return 0;
    }
    if (kBuckets[b].kind == LONG) {
        switch (kBuckets[b].rpl) {
#define C(R)                                                                                         \
    case R:                                                                                          \
        if (affine) hipLaunchKernelGGL((k_align_chunk<R, true, LONG>), grid, dim3(256), 0, st, p);   \
        else hipLaunchKernelGGL((k_align_chunk<R, false, LONG>), grid, dim3(256), 0, st, p);         \
        break;
        C(96) C(112) C(128)
#undef C
        }
        return 0;
    }
    switch (kBuckets[b].rpl) {
#define C(R)                                                                                           \
    case R:                                                                                            \
        if (affine) hipLaunchKernelGGL((k_align_chunk<R, true, PACKED>), grid, dim3(256), 0, st, p);   \
        else hipLaunchKernelGGL((k_align_chunk<R, false, PACKED>), grid, dim3(256), 0, st, p);         \
        break;
    C(4) C(8) C(12) C(16) C(20) C(24) C(28) C(32) C(36) C(40) C(44) C(48) C(52) C(56) C(60) C(64)
    C(68) C(72) C(76) C(80) C(84) C(88)
#undef C
    }
    return 0;
}


}  // namespace pcabi_eng
