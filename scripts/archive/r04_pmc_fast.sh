#!/bin/bash
# PMC traffic of k_step for the configs the round-4 straight-line batches run (boundary10, 4b): the
# FETCH_SIZE and WRITE_SIZE passes (one counter group per run), summarised per launch into
# profiles-style JSON (scripts/pmc_traffic.py), plus one SQ pass (VALU / SALU instructions per launch).
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/pmcfast}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for cfg in boundary10 forkjoin8_tasks; do
  i=0
  for group in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_WR"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $group --output-format csv -d $O/$cfg/p$i -o p -- python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline \
      > $O/${cfg}_p$i.log 2>&1 || { echo "pmc $cfg pass $i failed"; tail -5 $O/${cfg}_p$i.log; exit 1; }
  done
  python3 scripts/pmc_traffic.py $O/$cfg $O/pmc_$cfg.json k_step || exit 1
  python3 -c "import json;d=json.load(open('$O/pmc_$cfg.json'));print('$cfg', '%.1f MB/launch'%(d['traffic_bytes_per_launch']/1e6), 'VALU %.3g'%d['counters_per_launch'].get('SQ_INSTS_VALU',0))"
done
echo "=== done"
