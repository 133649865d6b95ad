#!/bin/bash
# Quick perf iteration: GPU parity tests, the bench (no CPU baseline), the stamped build's phase cycles.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
  || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err \
  || { tail -20 gpurun_out/q_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/q_bench.json'));print('%.4e trans/s  k_step %.1f us  frac %.3f' % (d['value'], d['roofline']['k_step_avg_ms']*1e3, d['roofline']['frac']))"
if [ -f zeebe_amd/libzbhip_stamps.so ]; then
  ZBHIP_LIB=libzbhip_stamps.so ZBHIP_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} \
    > gpurun_out/q_stamps.json 2> gpurun_out/q_stamps.err || { tail -20 gpurun_out/q_stamps.err; exit 1; }
  grep stamps gpurun_out/q_stamps.err | tail -1
fi
