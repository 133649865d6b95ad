#!/bin/bash
# The product with the straight-line batches on by default: the whole GPU suite, the headline line and
# its kernel trace, and the boundary10 / 4b / fork-join-8 / msg P=8 lines.
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/default}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench', '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep -h 'k_step' $O/prof/run_kernel_stats.csv | cut -d, -f2-4
for cfg in boundary10 forkjoin8_tasks forkjoin8; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -20 $O/bench_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$cfg.json'));print('$cfg', '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b10 -o run -- python3 bench.py --config boundary10 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_b10.log 2>&1 || { tail -20 $O/prof_b10.log; exit 1; }
grep -h 'k_step' $O/prof_b10/run_kernel_stats.csv | cut -d, -f2-4
echo "=== done"
