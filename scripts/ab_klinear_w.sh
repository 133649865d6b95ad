set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for i in 1 2; do
for v in libzbhip.so libzbhip_w3.so libzbhip_w5.so libzbhip_w6.so; do
  ZBHIP_LIB=$v timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-io > gpurun_out/ab/$v.$i.json 2>/dev/null
done
done
