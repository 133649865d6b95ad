#!/bin/bash
# The CPU suite under AddressSanitizer + UndefinedBehaviorSanitizer: host code of libzbhip (runtime,
# compiler, log writer) and the oracle, both built with clang so one sanitizer runtime serves them.
# CPU only (no GPU sanitizers).  Usage: bash scripts/sanitize.sh [pytest args]
set -eo pipefail
cd "$(dirname "$0")/.."
make -s -C zeebe_amd/csrc sanitize -j8
make -s -C oracle sanitize
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export ZBHIP_LIB=$PWD/zeebe_amd/csrc/build/libzbhip_asan.so ORACLE_LIB=$PWD/oracle/build/liboracle_asan.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD=$RT python -m pytest tests -q -x -m "not gpu" -p no:cacheprovider "$@"
