// pcabi_k_fast.hip -- k_align instantiations: the branch-free fast core (register buckets of
// 4..64 rows, scorings outside the packed ranges) and the guarded generic core (any scoring, <= 128).
#include "pcabi_kern.h"

namespace pcabi_eng {

void dispatch_fast(int rpl, bool generic, const KParams &p, bool affine, dim3 grid, hipStream_t st) {
    if (generic) {
        switch (rpl) {
        case 16: launch<16, GENERIC>(p, affine, grid, st); break;
        case 32: launch<32, GENERIC>(p, affine, grid, st); break;
        case 64: launch<64, GENERIC>(p, affine, grid, st); break;
        case 96: launch<96, GENERIC>(p, affine, grid, st); break;
        case 128: launch<128, GENERIC>(p, affine, grid, st); break;
        }
        return;
    }
    switch (rpl) {
#define C(R) case R: launch<R, FAST>(p, affine, grid, st); break;
    C(4) C(8) C(12) C(16) C(20) C(24) C(28) C(32) C(36) C(40) C(44) C(48) C(52) C(56) C(60) C(64)
#undef C
    }
}

}  // namespace pcabi_eng
