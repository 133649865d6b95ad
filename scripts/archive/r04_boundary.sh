#!/bin/bash
# Message boundary events: the new parity tests, the config-5 suites around them, and the msg P=8
# bench line (KMsg's register budget moved with the boundary paths).
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/boundary}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest tests/test_gpu_message_boundary.py tests/test_gpu_messages.py tests/test_gpu_psm_messages.py \
  tests/test_gpu_multiprocess.py tests/test_gpu_import.py -x -v -m gpu --timeout 200 --timeout-method thread \
  > $O/pytest.log 2>&1 || { grep -E "FAILED|Error|error" $O/pytest.log | head -20; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
if [ -z "$NOBENCH" ]; then
  timeout -k 10 300 python -u bench.py --config msg --virtual-partitions 8 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_msg8.json 2> $O/bench_msg8.err || { tail -20 $O/bench_msg8.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_msg8.json'));print('msg8', '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'], 'ms/step %.2f'%d['ms_per_step'])"
fi
echo "=== done"
