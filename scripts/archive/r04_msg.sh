#!/bin/bash
# Config 5 at 8 partitions on one GPU, with and without the subject-sorted device windows
# (ZBHIP_SUBJECT_SORT): parity test, bench line, and the FETCH/WRITE PMC passes over all zb:: kernels.
set -o pipefail
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/msg}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_messages.py -x -q -m gpu -k "subject_sorted or device_exchange" --timeout 200 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ARGS="--config msg --virtual-partitions 8 --steps 2 --warmup 1 --no-cpu-baseline"
for v in arrival sorted; do
  if [ $v = sorted ]; then export ZBHIP_SUBJECT_SORT=4096; fi
  timeout -k 10 300 python -u bench.py $ARGS > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v', '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'], 'ms/step %.2f'%d['ms_per_step'])"
  i=0
  for group in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $group --output-format csv -d $O/pmc_$v/p$i -o p -- python3 bench.py $ARGS \
      > $O/pmc_${v}_p$i.log 2>&1 || { echo "pmc $v $group failed"; tail -5 $O/pmc_${v}_p$i.log; exit 1; }
  done
  python3 scripts/pmc_traffic.py $O/pmc_$v $O/pmc_$v.json "zb::" 4 || exit 1
done
echo "=== done"
