#!/bin/bash
# Device log writer A/B: parity tests, then a kernel trace of the --host-io bench with the streaming
# write pass (k_log_stream, the product) and with the half-wave pass (ZBHIP_LOG_HALFWAVE=1, k_log_write).
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/logab}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export ZBHIP_LOG_STREAM=1 ZBHIP_JOURNAL=1 ZBHIP_DEVICE_ACTIVATIONS=1
[ -n "$LOGAB_NOTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_logdev.py tests/test_gpu_logserial.py tests/test_gpu_journal.py tests/test_gpu_key_table.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in stream halfwave; do
  if [ $v = halfwave ]; then export ZBHIP_LOG_HALFWAVE=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 bench.py --host-io --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  echo "$v: $(grep -E '"zb::k_log_(write|stream|sizes)' $(find $O/prof_$v -name '*kernel_stats.csv' | head -1) | cut -d, -f1-4 | tr '\n' ' ')"
done

# the host side with two host threads (ZBHIP_DEBUG: per-call breakdown on stderr)
unset ZBHIP_LOG_HALFWAVE ZBHIP_LOG_STREAM
ZBHIP_HOST_THREADS=2 ZBHIP_DEBUG=1 timeout -k 10 300 python3 bench.py --host-io --steps 1 --warmup 0 --no-cpu-baseline > $O/t2.json 2> $O/t2.err || { tail -20 $O/t2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/t2.json'))['host_io']['log_bytes'];print('threads=2 hbm', json.dumps(d['hbm']))"
grep -m1 "log write pass" $O/t2.err; grep -E "submit n=1000000|serialize_log_device n=1000000|run n=1000000" $O/t2.err | tail -3 | cut -c1-220
echo "=== done"
