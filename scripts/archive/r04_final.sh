#!/bin/bash
# Round-4 closing evidence: the message boundary tests first (fail fast), the whole GPU suite, the
# straight-line batches' parity on their A/B build, the default bench line with a rocprofv3 kernel
# trace, the config-5 P=8 line, and the straight-line A/B bench lines.
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/final}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest tests/test_gpu_message_boundary.py tests/test_gpu_psm_messages.py -x -v -m gpu \
  --timeout 200 --timeout-method thread > $O/pytest_boundary.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_boundary.log | head -20; tail -40 $O/pytest_boundary.log; exit 1; }
tail -1 $O/pytest_boundary.log
if [ -z "$NOSUITE" ]; then
  timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
# the straight-line KScope / KGeneric batches (libzbhip_fast.so, ZBHIP_FAST_SCOPE=1): parity first
FASTOK=0
if [ -f zeebe_amd/libzbhip_fast.so ]; then
  ZBHIP_LIB=$PWD/zeebe_amd/libzbhip_fast.so ZBHIP_FAST_SCOPE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_boundary.py \
    tests/test_gpu_timers.py tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_batch_limit.py tests/test_gpu_subprocess.py \
    tests/test_gpu_multi_instance.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_fast.log 2>&1 && FASTOK=1
  echo "fast parity: $FASTOK $(tail -1 $O/pytest_fast.log)"
  [ $FASTOK = 1 ] || grep -E "FAILED|Error" $O/pytest_fast.log | head -10
fi
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench', '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep -h '"zb::k_step' $(find $O/prof -name '*kernel_stats.csv' | head -1) | cut -d, -f1-4
timeout -k 10 300 python -u bench.py --config msg --virtual-partitions 8 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_msg8.json 2> $O/bench_msg8.err || { tail -20 $O/bench_msg8.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_msg8.json'));print('msg8', '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'], 'ms/step %.2f'%d['ms_per_step'])"
# straight-line A/B: the product (general path), the fast build with the batches on, the build before
# round 4's straight-line work (libzbhip_prev.so)
for cfg in boundary10 forkjoin8_tasks forkjoin8; do
  for v in product fast prev; do
    unset ZBHIP_FAST_SCOPE ZBHIP_LIB
    if [ $v = fast ]; then [ $FASTOK = 1 ] || continue; export ZBHIP_LIB=$PWD/zeebe_amd/libzbhip_fast.so ZBHIP_FAST_SCOPE=1; fi
    if [ $v = prev ]; then [ -f zeebe_amd/libzbhip_prev.so ] || continue; export ZBHIP_LIB=$PWD/zeebe_amd/libzbhip_prev.so; fi
    timeout -k 10 300 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_${cfg}_$v.json 2> $O/bench_${cfg}_$v.err || { tail -20 $O/bench_${cfg}_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${cfg}_$v.json'));print('$cfg $v', '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
  done
done
unset ZBHIP_FAST_SCOPE ZBHIP_LIB
echo "=== done"
