#!/bin/bash
# Builds an experimental library zeebe_amd/libzbhip_<name>.so with logdev.hip compiled with extra
# defines (A/B experiments only; the product is libzbhip.so):  scripts/logvariant.sh s3072 -DZB_LOGW_STAGE=3072
set -e
cd "$(dirname "$0")/../zeebe_amd/csrc"
name=$1; shift
make -s -j4 >/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -O3 -fPIC -Wall -Wno-unused-function "$@" -c logdev.hip -o build/logdev_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libzbhip_$name.so build/kernels.o build/logdev_$name.o build/runtime.o build/compiler.o build/logwriter.o
