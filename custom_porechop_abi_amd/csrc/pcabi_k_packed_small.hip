// pcabi_k_packed_small.hip -- k_align instantiations: packed-key core, register buckets of 4..32
// rows (the end-window adapters of the reference database).
#include "pcabi_kern.h"

namespace pcabi_eng {

void dispatch_packed_small(int rpl, const KParams &p, bool affine, dim3 grid, hipStream_t st) {
    switch (rpl) {
#define C(R) case R: launch<R, PACKED>(p, affine, grid, st); break;
    C(4) C(8) C(12) C(16) C(20) C(24) C(28) C(32)
#undef C
    }
}

}  // namespace pcabi_eng
