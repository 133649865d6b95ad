#!/bin/bash
# k_log_blocks variants, kernel stats of the host-io bench each: WAVES:PROBE:RANGE (ZBHIP_LOG_BLOCKS
# waves per workgroup; ZBHIP_LOG_PROBE 1 no template words, 2 no patches, 3 neither -- wrong bytes,
# timing only; ZBHIP_LOG_RANGE commands per round-robin range).  Output: gpurun_out/lp/
set -e
cd "$(dirname "$0")/.."
O=gpurun_out/lp
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in ${VARIANTS:-16:0:0 12:0:0 8:0:0 12:3:0}; do
  IFS=: read nw pr rg <<< "$v"
  ZBHIP_LOG_BLOCKS=$nw ZBHIP_LOG_PROBE=$pr ZBHIP_LOG_RANGE=$rg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/w${nw}_p${pr}_r$rg -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-io > /dev/null 2>> $O/err.txt
done
if [ -n "$TESTS" ]; then
  ZBHIP_LOG_BLOCKS=$TESTS timeout -k 10 400 python -u -m pytest tests/test_gpu_logdev.py tests/test_gpu_logserial.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
fi
echo done > $O/done.txt
