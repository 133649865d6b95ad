#!/bin/bash
# Round-4 GPU evidence: the whole GPU suite (the opt-in paths switched on: ZBHIP_LOG_STREAM,
# ZBHIP_JOURNAL, ZBHIP_DEVICE_ACTIVATIONS), the default bench line, and the device log writer's PMC
# passes on the --host-io path.  Each step under its own time limit; the first failure ends it.
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/r04}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export ZBHIP_LOG_STREAM=1 ZBHIP_JOURNAL=1 ZBHIP_DEVICE_ACTIVATIONS=1
if [ -z "$NOTEST" ]; then
  timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
    > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench', '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
fi
if [ -n "$LOGPMC" ]; then
  i=0
  while read -r group; do
    [ -z "$group" ] && continue
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $group --output-format csv -d $O/logpmc/p$i -o p -- python3 bench.py --host-io --steps 1 --warmup 0 --no-cpu-baseline \
      > $O/logpmc_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/logpmc_p$i.log; exit 1; }
  done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
GROUPS
  python3 scripts/pmc_traffic.py $O/logpmc $O/k_log_stream.json k_log_stream || exit 1
fi
echo "=== done"
