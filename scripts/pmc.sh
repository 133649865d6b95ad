#!/bin/bash
# PMC passes (one rocprofv3 run per counter group; never combined with tracing domains).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc
ARGS=${BENCH_ARGS:---instances 1000000 --steps 1 --warmup 0 --no-cpu-baseline}
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  echo "=== pass $i: $group"
  timeout -s KILL 120 rocprofv3 --pmc $group --output-format csv -d gpurun_out/pmc/p$i -o p -- python3 bench.py $ARGS \
    > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done <<GROUPS
${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE}
GROUPS
echo "=== done"
