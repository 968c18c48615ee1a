#!/bin/bash
# perf_variants/<name>.so = libpcabi with one kernel translation unit (TU, default the packed-core
# kernels for <= 32 rows: the headline's k_align<24>) rebuilt with extra -D flags; every other
# object as built by __graft_entry__. Perf experiments only:
#   [TU="pcabi_k_chunk ..."] tools/build_variant.sh <name> [-DFLAG=...]
set -e
name=$1; shift
mkdir -p perf_variants build/vobj
vo=""
skip="XXXX"
for tu in ${TU:-pcabi_k_packed_small}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -c "$@" -o build/vobj/${name}_$tu.o custom_porechop_abi_amd/csrc/$tu.hip
  vo="$vo build/vobj/${name}_$tu.o"
  skip="$skip|$tu.o"
done
objs=$(ls build/*.o | grep -Ev "$skip")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o perf_variants/$name.so $vo $objs -lz
echo built perf_variants/$name.so
