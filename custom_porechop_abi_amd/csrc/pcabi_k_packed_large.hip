// pcabi_k_packed_large.hip -- k_align instantiations: packed-key core, register buckets of 36..88
// rows (narrow and wide key layouts), and the long two-pass buckets of 96 / 112 / 128 rows.
#include "pcabi_kern.h"

namespace pcabi_eng {

void dispatch_packed_large(int rpl, bool long_kind, const KParams &p, bool affine, dim3 grid, hipStream_t st) {
    if (long_kind) {
        switch (rpl) {
        case 96: launch<96, LONG>(p, affine, grid, st); break;
        case 112: launch<112, LONG>(p, affine, grid, st); break;
        case 128: launch<128, LONG>(p, affine, grid, st); break;
        }
        return;
    }
    switch (rpl) {
#define C(R) case R: launch<R, PACKED>(p, affine, grid, st); break;
    C(36) C(40) C(44) C(48) C(52) C(56) C(60) C(64) C(68) C(72) C(76) C(80) C(84) C(88)
#undef C
    }
}

}  // namespace pcabi_eng
