#!/bin/bash
# One GPU session refreshing every measurement under profiles/: GPU tests, the default bench (with
# the CPU baseline), rocprofv3 kernel stats, PMC passes, and the other BASELINE configs.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/all
export PYTHONUNBUFFERED=1
O=gpurun_out/all
echo "=== tests"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
echo "=== bench linear10"
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > $O/bench_linear10.json 2> $O/bench_linear10.err \
  || { tail -20 $O/bench_linear10.err; exit 1; }
cat $O/bench_linear10.json
echo "=== rocprof"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
  > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cat $(find $O/prof -name "*kernel_stats.csv" | head -1) | cut -c1-200
echo "=== pmc"
rm -rf gpurun_out/pmc && bash scripts/pmc.sh || exit 1
for cfg in one_task xor forkjoin8 boundary10 msg; do
  echo "=== bench $cfg"
  timeout -k 10 600 python -u bench.py --config $cfg --steps 3 --warmup 1 > $O/bench_$cfg.json 2> $O/bench_$cfg.err \
    || { tail -20 $O/bench_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$cfg.json'));print('%.4e'%d['value'], d['unit'], 'frac %.3f'%d['roofline']['frac'])"
done
echo "=== host boundary (--host-io) with kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_hio -o hio -- python3 bench.py --host-io --steps 2 --warmup 1 --no-cpu-baseline \
  > $O/bench_hostio.json 2> $O/bench_hostio.err || { tail -20 $O/bench_hostio.err; exit 1; }
cat $(find $O/prof_hio -name "*kernel_stats.csv" | head -1) | cut -c1-160 | head -8
echo "=== bench msg 8 virtual partitions"
timeout -k 10 600 python -u bench.py --config msg --virtual-partitions 8 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_msg_p8.json 2> $O/bench_msg_p8.err \
  || { tail -20 $O/bench_msg_p8.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_msg_p8.json'));print('%.4e'%d['value'], d['unit'])"
echo "=== done"
