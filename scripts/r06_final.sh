#!/bin/bash
# Round-6 final evidence on one box: the driver's default bench, its rocprofv3 kernel stats, PMC traffic
# passes (FETCH_SIZE / WRITE_SIZE, one counter group per run) for linear10 (the headline) and
# forkjoin8_tasks (variant 4b), the 4b bench line and the untrusted-window bench.  Output under
# gpurun_out/r06/final; scripts/pmc_traffic.py summarises the PMC passes afterwards (on the CPU side).
set -e
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/r06/final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_default -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io > /dev/null 2>> $O/errs.txt
for cfg in linear10 forkjoin8_tasks; do
  i=0
  for group in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $group --output-format csv -d $O/pmc_$cfg/p$i -o p -- python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_${cfg}_p$i.log 2>&1
  done
done
timeout -k 10 300 python -u bench.py --config forkjoin8_tasks --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_forkjoin8_tasks.json 2>> $O/errs.txt
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --untrusted-windows > $O/bench_untrusted.json 2>> $O/errs.txt
echo done > $O/done.txt
