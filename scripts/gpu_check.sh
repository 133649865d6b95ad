#!/bin/bash
# One GPU session: tests, smoke, a short bench, a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STEPS=${STEPS:-tests,smoke,bench,prof}
run() { echo "=== $1"; }
if [[ $STEPS == *tests* ]]; then
  run tests
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
  tail -5 gpurun_out/pytest_gpu.log
fi
if [[ $STEPS == *smoke* ]]; then
  run smoke
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
if [[ $STEPS == *bench* ]]; then
  run bench
  timeout -k 10 600 python -u bench.py --steps ${BENCH_STEPS:-3} --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err \
    || { tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [[ $STEPS == *prof* ]]; then
  run prof
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} \
    > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*stats.csv" | head -5; cat $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) | cut -c1-220
fi
echo "=== done"
