#!/bin/bash
# Kernel-configuration sweep for the small k_step variant (ZBHIP_KCFG, see kernels.hip).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in ${CFGS:--1 0 1 2 3 4}; do
  echo "=== cfg $v"
  ZBHIP_KCFG=$v timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/tune_$v.json 2> gpurun_out/tune_$v.err || { tail -5 gpurun_out/tune_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/tune_$v.json'));print('%.3e trans/s  ms/step %.3f  k_step %.1f us  frac %.3f'%(d['value'],d['ms_per_step'],d['roofline']['k_step_avg_ms']*1e3,d['roofline']['frac']))"
done
