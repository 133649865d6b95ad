#!/bin/bash
# Round-4 refresh of the configs not re-measured elsewhere (one_task, xor, msg P=1) and the headline's
# PMC traffic (FETCH_SIZE / WRITE_SIZE passes of k_step).
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/refresh}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for cfg in one_task xor msg; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -20 $O/bench_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$cfg.json'));print('$cfg', '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
done
i=0
for group in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $group --output-format csv -d $O/pmc_linear10/p$i -o p -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline \
    > $O/pmc_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc_p$i.log; exit 1; }
done
python3 scripts/pmc_traffic.py $O/pmc_linear10 $O/pmc_linear10.json k_step || exit 1
python3 -c "import json;d=json.load(open('$O/pmc_linear10.json'));print('linear10 traffic %.1f MB/launch'%(d['traffic_bytes_per_launch']/1e6))"
echo "=== done"
