#!/bin/bash
# template path check: its GPU tests, then xor / forkjoin8 benches
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_templates.py \
  ${PYTEST_EXTRA:-} > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for c in ${CONFIGS:-xor forkjoin8}; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_$c.log 2>&1 || { tail -20 gpurun_out/b_$c.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('template_batches_per_step'))" gpurun_out/b_$c.log $c
done
