#!/bin/bash
# GPU test suite (+ optional bench configs in BENCH="xor forkjoin8 ..."), each step under its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
  > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for c in ${BENCH:-}; do
  timeout -k 10 600 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err \
    || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));print('$c', '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
done
echo "=== done"
