#!/bin/bash
# build/variants/<name>.so = libpcabi built with extra -D flags (perf experiments only)
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" -o build/variants/$name.so custom_porechop_abi_amd/csrc/pcabi_engine.hip
