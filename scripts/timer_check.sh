#!/bin/bash
# Timer / sub-process GPU check: the new tests first, then (FULL=1) the whole GPU suite and smoke.
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/tmr}
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "=== timer + sub-process tests"
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_timers.py tests/test_gpu_subprocess.py} -x -v -m gpu --timeout 120 \
  --timeout-method thread > $O/pytest_new.log 2>&1 || { tail -80 $O/pytest_new.log; exit 1; }
tail -3 $O/pytest_new.log
if [[ -n "$FULL" ]]; then
echo "=== full GPU suite"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "=== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
echo "=== done"
