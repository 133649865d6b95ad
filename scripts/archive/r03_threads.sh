#!/bin/bash
# Host-io path vs the number of host worker threads (ZBHIP_HOST_THREADS; default: the cgroup quota).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/threads
mkdir -p $O
echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null) affinity: $(python3 -c 'import os;print(len(os.sched_getaffinity(0)))')"
for t in 16 default 8 4; do
  if [ $t = default ]; then unset ZBHIP_HOST_THREADS; else export ZBHIP_HOST_THREADS=$t; fi
  timeout -k 10 300 python -u bench.py --host-io --steps 3 --warmup 1 --no-cpu-baseline > $O/b_$t.json 2> $O/b_$t.err || { tail -5 $O/b_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$t.json'));h=d['host_io'];print('$t', {k:('%.3e'%v['hbm']['value'], {x:round(y,1) for x,y in v['hbm'].items() if x.endswith('_ms')}) if k=='log_bytes' else '%.3e'%v['value'] for k,v in h.items() if isinstance(v,dict) and ('value' in v or 'hbm' in v)})"
done
echo "=== done"
