#!/bin/bash
# KScope / KGeneric configuration A/B on the straight-line workloads: the product, 4 waves per SIMD for
# KScope (-DZB_KSCOPE_W=4), 64-lane workgroups for KGeneric / KScope (-DZB_KGENERIC_B=64).
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/kab}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in ${VARIANTS:-product w4 b64}; do
  unset ZBHIP_LIB
  if [ $v != product ]; then [ -f zeebe_amd/libzbhip_$v.so ] || continue; export ZBHIP_LIB=$PWD/zeebe_amd/libzbhip_$v.so; fi
  for cfg in boundary10 forkjoin8_tasks forkjoin8; do
    timeout -k 10 300 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_${cfg}_$v.json 2> $O/bench_${cfg}_$v.err || { tail -20 $O/bench_${cfg}_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${cfg}_$v.json'));print('$cfg $v', '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
  done
done
echo "=== done"
