// pcabi_k_packed_small.hip -- k_align instantiations: packed-key core, register buckets of 4..32
// rows (the end-window adapters of the reference database), in the untagged and
// (affine) run-tagged key layouts.
#include "pcabi_kern.h"

namespace pcabi_eng {

void dispatch_packed_small(int rpl, const KParams &p, bool affine, dim3 grid, hipStream_t st, bool tagged) {
    if (tagged && affine) {
        switch (rpl) {
#define T(R) case R: hipLaunchKernelGGL((k_align<R, true, TAGGED>), grid, dim3(256), 0, st, p); return;
        T(4) T(8) T(12) T(16) T(20) T(24) T(28) T(32)
#undef T
        }
    }
    switch (rpl) {
#define C(R) case R: launch<R, PACKED>(p, affine, grid, st); break;
    C(4) C(8) C(12) C(16) C(20) C(24) C(28) C(32)
#undef C
    }
}

}  // namespace pcabi_eng
