#!/bin/bash
# k_log_blocks with default-policy stores (product) against non-temporal stores
# (zeebe_amd/libzbhip_ntstores.so, built beforehand with -DZB_LOG_NT_STORES): kernel stats of the
# host-io bench.  Output: gpurun_out/ls/
set -e
cd "$(dirname "$0")/.."
O=gpurun_out/ls
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/plain -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-io > /dev/null 2>> $O/err.txt
cp zeebe_amd/libzbhip.so /tmp/libzbhip_plain.so
cp zeebe_amd/libzbhip_ntstores.so zeebe_amd/libzbhip.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/nt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-io > /dev/null 2>> $O/err.txt
cp /tmp/libzbhip_plain.so zeebe_amd/libzbhip.so
echo done > $O/done.txt
