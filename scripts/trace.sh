#!/bin/bash
# rocprofv3 kernel-trace summary of one bench configuration: OUT=dir ARGS="bench args" bash scripts/trace.sh
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/trace}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py $ARGS --no-cpu-baseline \
  > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("%-60s calls %6s avg %10.1f us total %8.3f ms %5.1f%%" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3,
          float(r["TotalDurationNs"]) / 1e6, 100 * float(r["TotalDurationNs"]) / tot))
PY
