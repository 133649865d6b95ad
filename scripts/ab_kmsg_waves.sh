#!/bin/bash
# A/B of the KMsg register target (ZB_KMSG_W 2 / 3 / 4: 256 / 168 / 128 VGPRs, the latter two with spills) on config 5 at P = 8 and P = 1
set -e
cd "$(dirname "$0")/.."
O=gpurun_out/r06/kmsg_ab
mkdir -p $O
for v in default mw3 mw4; do
  if [ $v = default ]; then L=libzbhip.so; else L=libzbhip_$v.so; fi
  ZBHIP_LIB=$L timeout -k 10 300 python -u bench.py --config msg --virtual-partitions 8 --steps 3 --warmup 1 --no-cpu-baseline > $O/msg8_$v.json 2>> $O/err.txt
  ZBHIP_LIB=$L timeout -k 10 300 python -u bench.py --config msg --steps 3 --warmup 1 --no-cpu-baseline > $O/msg1_$v.json 2>> $O/err.txt
done
echo done > $O/done.txt
