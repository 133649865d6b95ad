#!/bin/bash
# Config 5 A/B: the product against the build before the message boundary work (libzbhip_preb.so:
# KMsg without its 24 B of scratch), P = 1 and P = 8 on one GPU, two runs each.
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/msgab}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for rep in 1 2; do
  for v in product preb; do
    unset ZBHIP_LIB
    [ $v = preb ] && export ZBHIP_LIB=$PWD/zeebe_amd/libzbhip_preb.so
    for P in 1 8; do
      timeout -k 10 300 python -u bench.py --config msg --virtual-partitions $P --steps 3 --warmup 1 --no-cpu-baseline > $O/msg${P}_${v}_$rep.json 2> $O/msg${P}_${v}_$rep.err || { tail -20 $O/msg${P}_${v}_$rep.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/msg${P}_${v}_$rep.json'));print('msg$P $v $rep', '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
    done
  done
done
echo "=== done"
