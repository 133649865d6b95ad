#!/bin/bash
# Builds an experimental library zeebe_amd/libzbhip_<name>.so from kernels.hip with extra defines
# (A/B experiments only; the product is libzbhip.so):  scripts/variant.sh s16 -DZB_KSIMPLE_B=64 -DZB_KSIMPLE_R=16
set -e
cd "$(dirname "$0")/../zeebe_amd/csrc"
name=$1; shift
make -s -j4 >/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -O3 -fPIC -Wall -Wno-unused-function "$@" -c kernels.hip -o build/kernels_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libzbhip_$name.so build/kernels_$name.o build/logdev.o build/runtime.o build/compiler.o build/logwriter.o
