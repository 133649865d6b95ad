#!/bin/bash
# Log writer check + the in-process exchange (message GPU tests, msg8 bench).
set -o pipefail
cd "$(dirname "$0")/.."
bash scripts/r03_logcheck.sh || exit 1
O=gpurun_out/check2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_messages.py tests/test_gpu_multiprocess.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_msg.log 2>&1 || { tail -40 $O/pytest_msg.log; exit 1; }
tail -2 $O/pytest_msg.log
timeout -k 10 600 python -u bench.py --config msg --virtual-partitions 8 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_msg8.json 2> $O/bench_msg8.err || { tail -20 $O/bench_msg8.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_msg8.json'));print('msg8 %.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
echo "=== done2"
