# scripts/debug/debug_mi_random.py over the seeds the wider campaign (scripts/fuzz_random.py) failed:
# SEEDS="mode:seed ..." (mode boundary or mi)
mkdir -p gpurun_out/dbg
for a in ${SEEDS:-boundary:141 boundary:312 mi:140 mi:144 mi:228 mi:242 mi:222}; do
  timeout -k 10 120 python -u scripts/debug/debug_mi_random.py ${a%%:*} ${a##*:} > gpurun_out/dbg/${a%%:*}_${a##*:}.txt 2>&1 || true
done
