#!/bin/bash
# Round 3: the general (KGeneric / KSimple) path without CREATE templates, variant 4b, and the
# kernel trace of a templated run (first launch = recording).  Each GPU step has its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/gen}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for spec in "forkjoin8 --no-templates" "xor --no-templates" "forkjoin8_tasks" "forkjoin8" "xor"; do
  tag=$(echo $spec | tr ' ' '_' | tr -d '-')
  echo "=== bench $spec"
  timeout -k 10 600 python -u bench.py --config $spec --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$tag.json 2> $O/bench_$tag.err \
    || { tail -20 $O/bench_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$tag.json'));print('%.4e'%d['value'], d['unit'], 'frac %.3f'%d['roofline']['frac'], 'k_step %.3f ms'%d['roofline']['k_step_avg_ms'])"
  echo "=== trace $spec"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$tag -o run -- python3 bench.py --config $spec --steps 2 --warmup 1 --no-cpu-baseline \
    > $O/prof_$tag.log 2>&1 || { tail -20 $O/prof_$tag.log; exit 1; }
  f=$(find $O/prof_$tag -name "*kernel_trace.csv" | head -1)
  python3 scripts/launch_times.py "$f" | tail -25
done
echo "=== done"
