#!/bin/bash
# Device log writer: parity tests, the --host-io bench and a kernel trace of it.
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/logcheck}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest tests/test_gpu_logdev.py tests/test_gpu_logserial.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
ZBHIP_DEBUG=1 timeout -k 10 600 python -u bench.py --host-io --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_hostio.json 2> $O/bench_hostio.err || { tail -20 $O/bench_hostio.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_hostio.json'));h=d['host_io']['log_bytes']['hbm'];print('log bytes in HBM %.3e tr/s'%h['value'], {k:round(v,1) for k,v in h.items() if k.endswith('_ms')})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --host-io --steps 1 --warmup 0 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep -E "k_log|k_table|k_ring" $(find $O/prof -name "*kernel_stats.csv" | head -1) | cut -c1-150
echo "=== done"
