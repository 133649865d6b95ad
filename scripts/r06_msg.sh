#!/bin/bash
# Config 5 evidence: msg bench lines (P = 8 partitions on one GPU, P = 1) and their rocprofv3 kernel
# traces.  Output under gpurun_out/r06/${TAG:-msg}.
set -e
cd "$(dirname "$0")/.."
O=gpurun_out/r06/${TAG:-msg}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config msg --virtual-partitions 8 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_msg8.json 2> $O/err.txt
timeout -k 10 300 python -u bench.py --config msg --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_msg.json 2>> $O/err.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_msg8 -o run --output-format csv -- python3 bench.py --config msg --virtual-partitions 8 --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>> $O/err.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_msg -o run --output-format csv -- python3 bench.py --config msg --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>> $O/err.txt
echo done > $O/done.txt
