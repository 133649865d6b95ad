#!/bin/bash
# Device log writer A/B: parity tests with the product library, then a kernel trace of the
# --host-io bench per library (k_log_write average per 10^6-command window).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/logab
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
[ -n "$LOGAB_NOTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_logdev.py tests/test_gpu_logserial.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in "" $LOGAB_VARIANTS; do
  lib=$PWD/zeebe_amd/libzbhip${v:+_$v}.so
  ZBHIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${v:-product} -o run -- python3 bench.py --host-io --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_${v:-product}.log 2>&1 || { tail -20 $O/prof_${v:-product}.log; exit 1; }
  echo "${v:-product}: $(grep -E '"zb::k_log_write' $(find $O/prof_${v:-product} -name '*kernel_stats.csv' | head -1) | cut -d, -f2-4)"
done
echo "=== done"
