#!/bin/bash
# Round 3 probes: config 5 at 8 partitions (bench, kernel trace, per-dispatch PMC traffic) and the
# --host-io log-bytes path's kernel trace.  Every GPU step has its own limit, chained with &&.
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/probe}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
A="--config msg --virtual-partitions 8"
timeout -k 10 600 python -u bench.py $A --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_msg8.json 2> $O/bench_msg8.err || { tail -20 $O/bench_msg8.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_msg8.json'));print('%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_msg8 -o run -- python3 bench.py $A --steps 1 --warmup 1 --no-cpu-baseline > $O/prof_msg8.log 2>&1 || { tail -20 $O/prof_msg8.log; exit 1; }
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/pmc_msg8/p$i -o p -- python3 bench.py $A --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_msg8_p$i.log 2>&1 || { tail -5 $O/pmc_msg8_p$i.log; exit 1; }
done
python3 scripts/pmc_dispatch.py $O/pmc_msg8 400 > $O/pmc_msg8_dispatch.txt && tail -25 $O/pmc_msg8_dispatch.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_hostio -o run -- python3 bench.py --host-io --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_hostio.log 2>&1 || { tail -20 $O/prof_hostio.log; exit 1; }
cat $(find $O/prof_hostio -name "*kernel_stats.csv" | head -1) | cut -c1-200
echo "=== done"
