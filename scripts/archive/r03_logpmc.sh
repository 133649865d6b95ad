#!/bin/bash
# PMC passes of the device log writer (k_log_write / k_log_sizes) on the --host-io path.
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/logpmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export PYTHONUNBUFFERED=1
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $group --output-format csv -d $O/p$i -o p -- python3 bench.py --host-io --steps 1 --warmup 0 --no-cpu-baseline \
    > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
GROUPS
python3 scripts/pmc_traffic.py $O $O/k_log_write.json k_log_write && python3 scripts/pmc_traffic.py $O $O/k_log_sizes.json k_log_sizes
echo "=== done"
