#!/bin/bash
# Round-5 evidence on one box: the driver's default bench (timed), the host-io pass, every config's
# bench line and rocprofv3 kernel stats, the untrusted-window bench.  Output under gpurun_out/r05/.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
T0=$(date +%s)
timeout -k 10 300 python -u bench.py > gpurun_out/r05/bench_default.json 2> gpurun_out/r05/bench_default.err
echo "default bench $(( $(date +%s) - T0 )) s" > gpurun_out/r05/times.txt
T0=$(date +%s)
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-io > gpurun_out/r05/bench_hostio.json 2> gpurun_out/r05/bench_hostio.err
echo "host-io bench $(( $(date +%s) - T0 )) s" >> gpurun_out/r05/times.txt
for cfg in ${CFGS:-one_task xor forkjoin8 forkjoin8_tasks boundary10 linear10}; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05/bench_$cfg.json 2>> gpurun_out/r05/errs.txt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/prof_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>> gpurun_out/r05/errs.txt
done
timeout -k 10 300 python -u bench.py --config msg --virtual-partitions 8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05/bench_msg8.json 2>> gpurun_out/r05/errs.txt
timeout -k 10 300 python -u bench.py --config msg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05/bench_msg.json 2>> gpurun_out/r05/errs.txt
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --untrusted-windows > gpurun_out/r05/bench_untrusted.json 2>> gpurun_out/r05/errs.txt
echo done >> gpurun_out/r05/times.txt
