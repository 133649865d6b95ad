#!/bin/bash
# Sub-process GPU check: the new tests first, then the whole GPU suite and a short default bench.
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/sub}
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "=== sub-process tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_subprocess.py -x -v -m gpu --timeout 120 --timeout-method thread \
  > $O/pytest_sub.log 2>&1 || { tail -80 $O/pytest_sub.log; exit 1; }
tail -3 $O/pytest_sub.log
if [[ -n "$FULL" ]]; then
echo "=== full GPU suite"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "=== bench"
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
fi
echo "=== done"
