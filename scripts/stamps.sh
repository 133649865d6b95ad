cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export ZBHIP_LIB=libzbhip_stamps.so ZBHIP_STAMPS=1 &&
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/st1.json 2> gpurun_out/st1.err &&
ZBHIP_CHUNKS_PER_WG=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/st2.json 2> gpurun_out/st2.err &&
ZBHIP_LIB=libzbhip.so ZBHIP_CHUNKS_PER_WG=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/st3.json 2> gpurun_out/st3.err &&
ZBHIP_LIB=libzbhip.so ZBHIP_CHUNKS_PER_WG=12 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/st4.json 2> gpurun_out/st4.err
