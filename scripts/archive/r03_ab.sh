#!/bin/bash
# Log writer check, then A/B bench lines on the same box: one_task twice, linear-10 with the
# product library and the KLinear 5-waves variant (scripts/variant.sh lw5 -DZB_KLINEAR_W=5).
set -o pipefail
cd "$(dirname "$0")/.."
bash scripts/r03_logcheck.sh || exit 1
O=gpurun_out/ab
mkdir -p $O
b() { timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }; python3 -c "import json;d=json.load(open('$O/b.json'));print('$*', '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'], 'k_step %.4f'%d['roofline']['k_step_avg_ms'])"; }
b --config one_task && b --config one_task && b --config linear10 && ZBHIP_LIB=$PWD/zeebe_amd/libzbhip_lw5.so b --config linear10 && b --config linear10
echo "=== ab done"
