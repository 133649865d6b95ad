#!/bin/bash
# Device log path: parity tests, then the --host-io bench with the runtime's per-window timing lines.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/hostio
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_logdev.py tests/test_gpu_logserial.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ZBHIP_DEBUG=1 timeout -k 10 300 python -u bench.py --host-io --steps 3 --warmup 1 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b.json'));h=d['host_io']['log_bytes']['hbm'];print('log bytes in HBM %.3e tr/s'%h['value'], {k:round(v,1) for k,v in h.items() if k.endswith('_ms')})"
grep "serialize_log_device" $O/b.err | tail -12 | cut -c40-220
echo "=== done"
