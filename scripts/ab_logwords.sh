#!/bin/bash
# k_log_blocks (device log write: block loads + one lane per entry) against k_log_write: the
# device-log parity tests for each shape, then kernel stats of the host-io bench for each, then PMC
# passes of the default.  Output: gpurun_out/lw/
set -e
cd "$(dirname "$0")/.."
O=gpurun_out/lw
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
ZBHIP_LOG_BLOCKS=16 timeout -k 10 400 python -u -m pytest tests/test_gpu_logdev.py tests/test_gpu_logserial.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
#ZBHIP_LOG_BLOCKS=16 timeout -k 10 400 python -u -m pytest tests/test_gpu_logdev.py -x -q --timeout 120 --timeout-method thread > $O/tests16.log 2>&1
for b in ${BLOCKS:-16}; do
  ZBHIP_DEBUG=1 ZBHIP_LOG_BLOCKS=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b$b -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-io > $O/b$b.json 2>> $O/err.txt
done
#ZBHIP_LOG_HALFWAVE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_half -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-io > $O/half.json 2>> $O/err.txt
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  ZBHIP_LOG_BLOCKS=16 timeout -s KILL 300 rocprofv3 --pmc $group --output-format csv -d $O/p$i -o p -- python3 bench.py --host-io --steps 1 --warmup 0 --no-cpu-baseline \
    > $O/p$i.log 2>&1
done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
WRITE_SIZE
GROUPS
python3 scripts/pmc_traffic.py $O $O/k_log_blocks.json k_log_blocks
echo done > $O/done.txt
