#!/bin/bash
# perf_variants/r05bug.so: libpcabi with BOTH halves of the r05 fix c1b7048 reverted -- the plans'
# needs left as the fresh allocation holds them (no memset) and need2 taken in every round (not only
# the window rounds') -- for tests/test_gpu_middle_paths.py::test_poisoned_scratch's guard: the
# 0x7F poison must make tests/poisoned_middle.py fail against it (tools/gpu_r06_misc.sh).
set -e
cd "$(dirname "$0")/.."
src=custom_porechop_abi_amd/csrc
sed -e 's/    HIP_TRY(hipMemsetAsync(d_slots, 0, 4 \* sizeof(int64_t), st));/    \/\/ (r05bug variant: the plans'"'"' needs left unwritten)/' \
    -e 's/const int64_t most = std::max(need, windows ? need2 : (int64_t)0);/const int64_t most = std::max(need, need2);   \/\/ (r05bug variant)/' \
    $src/pcabi_engine.hip > $src/_engine_r05bug.hip
test "$(grep -c 'r05bug variant' $src/_engine_r05bug.hip)" = 2
mkdir -p build/vobj perf_variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -o build/vobj/engine_r05bug.o $src/_engine_r05bug.hip
rm -f $src/_engine_r05bug.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o perf_variants/r05bug.so build/vobj/engine_r05bug.o $(ls build/*.o | grep -v pcabi_engine.o) -lz
echo built perf_variants/r05bug.so
