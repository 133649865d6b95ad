#!/bin/bash
# Roofline evidence for every bench config: a bench line, a rocprofv3 kernel-trace summary and the
# PMC passes (one rocprofv3 run per counter group, never combined with tracing) per config.
# Usage: CONFIGS="linear10 xor" OUT=gpurun_out/ev bash scripts/evidence.sh
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/ev}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for spec in ${CONFIGS:-linear10 linear10@10000000 one_task xor forkjoin8 msg msg8}; do
  cfg=${spec%@*}
  args="--config $cfg"
  tag=$cfg
  if [[ $spec == *@* ]]; then args="$args --instances ${spec#*@}"; tag="${cfg}_${spec#*@}"; fi
  if [[ $spec == msg8 ]]; then args="--config msg --virtual-partitions 8"; fi
  echo "=== bench $tag"
  timeout -k 10 600 python -u bench.py $args --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err \
    || { tail -20 $OUT/bench_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$tag.json'));print('%.4e'%d['value'], d['unit'], 'frac %.3f'%d['roofline']['frac'])"
  # profiled runs: one warmup step (templates recorded), PS timed steps and the bench's timed pass
  PS=${PS:-2}
  echo "=== kernel trace $tag"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$tag -o run -- python3 bench.py $args --steps $PS --warmup 1 --no-cpu-baseline \
    > $OUT/prof_$tag.log 2>&1 || { tail -20 $OUT/prof_$tag.log; exit 1; }
  i=0
  while read -r group; do
    [ -z "$group" ] && continue
    i=$((i+1))
    echo "=== pmc $tag pass $i: $group"
    mkdir -p $OUT/pmc_$tag
    timeout -s KILL 200 rocprofv3 --pmc $group --output-format csv -d $OUT/pmc_$tag/p$i -o p -- python3 bench.py $args --steps $PS --warmup 1 --no-cpu-baseline \
      > $OUT/pmc_$tag/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/pmc_$tag/p$i.log; exit 1; }
  done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
GROUPS
  if [[ $cfg == msg* ]]; then
    python3 scripts/pmc_traffic.py $OUT/pmc_$tag $OUT/pmc_$tag.json "zb::" $((PS + 2)) || exit 1
  else
    python3 scripts/pmc_traffic.py $OUT/pmc_$tag $OUT/pmc_$tag.json || exit 1
  fi
done
echo "=== done"
