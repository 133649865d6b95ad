#!/bin/bash
# A/B of library builds on the bench (no CPU baseline), alternating: LIBS="libzbhip_base.so libzbhip.so".
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
    || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
for r in $(seq ${ROUNDS:-3}); do
  for lib in ${LIBS:-libzbhip_base.so libzbhip.so}; do
    ZBHIP_LIB=$lib timeout -k 10 120 python3 bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab.json 2> gpurun_out/ab.err \
      || { tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('%-24s %.4e trans/s  k_step %.2f us  frac %.3f'%('$lib',d['value'],d['roofline'].get('k_step_avg_ms',d['roofline'].get('k_avg_ms',float('nan')))*1e3,d['roofline']['frac']))"
  done
done
