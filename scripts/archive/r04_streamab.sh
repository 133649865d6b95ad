#!/bin/bash
# k_log_stream A/B: kernel traces of the --host-io bench per library (product, then the variants in
# VARIANTS, built by scripts/logvariant.sh), after the device-log parity tests on each.
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/streamab}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export ZBHIP_LOG_STREAM=1 ZBHIP_JOURNAL=1 ZBHIP_DEVICE_ACTIVATIONS=1
for v in product ${VARIANTS:-}; do
  lib=$PWD/zeebe_amd/libzbhip.so
  [ $v != product ] && lib=$PWD/zeebe_amd/libzbhip_$v.so
  ZBHIP_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_logdev.py -x -q -m gpu --timeout 200 --timeout-method thread \
    > $O/pytest_$v.log 2>&1 || { echo "$v: parity FAILED"; tail -30 $O/pytest_$v.log; exit 1; }
  ZBHIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 bench.py --host-io --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log) | $(grep -E '"zb::k_log_(write|stream)' $(find $O/prof_$v -name '*kernel_stats.csv' | head -1) | cut -d, -f1-4 | tr '\n' ' ')"
done
echo "=== done"
