#!/bin/bash
# Round-2 GPU check: the GPU suite, smoke, the default bench line and the config-5 line.
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/chk}
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "=== tests"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1 \
  || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "=== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
echo "=== bench"
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
echo "=== bench msg"
timeout -k 10 600 python -u bench.py --config msg --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_msg.json 2> $O/bench_msg.err || { tail -30 $O/bench_msg.err; exit 1; }
cat $O/bench_msg.json

if [[ -n "$MSG8" ]]; then
echo "=== bench msg 8 virtual partitions"
timeout -k 10 600 python -u bench.py --config msg --virtual-partitions 8 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_msg8.json 2> $O/bench_msg8.err || { tail -30 $O/bench_msg8.err; exit 1; }
cat $O/bench_msg8.json
fi
echo "=== done"
