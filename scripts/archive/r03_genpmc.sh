#!/bin/bash
# PMC passes of the general (no-template) path: forkjoin8 and xor at 10^7 instances.
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/genpmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export PYTHONUNBUFFERED=1
for cfg in forkjoin8 xor; do
  i=0
  while read -r group; do
    [ -z "$group" ] && continue
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $group --output-format csv -d $O/$cfg/p$i -o p -- python3 bench.py --config $cfg --no-templates --steps 1 --warmup 1 --no-cpu-baseline \
      > $O/$cfg/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/$cfg/p$i.log; exit 1; }
  done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
GROUPS
  python3 scripts/pmc_traffic.py $O/$cfg $O/pmc_${cfg}_general.json || exit 1
done
echo "=== done"
