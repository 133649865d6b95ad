#!/bin/bash
# config-5 check: message GPU tests, then the msg bench at P=1 and with 8 virtual partitions
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_messages.py \
  tests/test_gpu_multiprocess.py $PYTEST_EXTRA > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for c in "--config msg --steps 5 --warmup 2" "--config msg --virtual-partitions 8 --steps 2 --warmup 1"; do
  timeout -k 10 300 python bench.py $c --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['device_ms_per_step'])" gpurun_out/b.log
done
