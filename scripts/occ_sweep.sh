#!/bin/bash
# occupancy experiment: bench lines with the k_step grid sizing printed (ZBHIP_DEBUG) and forced (ZBHIP_WG_PER_CU)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
set -o pipefail
run() { ZBHIP_DEBUG=1 ZBHIP_LIB=$1 timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --config $2 > gpurun_out/o.json 2> gpurun_out/o.err || { tail -5 gpurun_out/o.err; exit 1; }; echo "$1 $2 WGPCU=${ZBHIP_WG_PER_CU:-auto} $(grep -m1 zbhip gpurun_out/o.err) $(python3 -c "import json;d=json.load(open('gpurun_out/o.json'));print('%.4e'%d['value'])")"; }
for lib in libzbhip_s20.so libzbhip_s8.so libzbhip_s4.so libzbhip.so; do run $lib xor; done
for lib in libzbhip_g6.so libzbhip_g4.so libzbhip_g2.so libzbhip.so; do run $lib forkjoin8; done
for c in linear10 one_task; do run libzbhip.so $c; for w in 15 16 17 18; do ZBHIP_WG_PER_CU=$w run libzbhip.so $c; done; done
