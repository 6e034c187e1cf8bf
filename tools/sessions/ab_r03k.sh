# round-3: LL128 unroll A/B (2 ranks sharing the GPU), then the GPU suite
export LAT_COLLS=ar,rs LAT_SIZES=262144,1048576,4194304 LAT_ALGOS=ll128 LAT_STEPS=30
bash tools/ab_lib.sh r03k_ll 2 3 vccl_amd/lib/libvccl.so vccl_amd/lib/libvccl_llu4.so &&
unset LAT_COLLS LAT_SIZES LAT_ALGOS LAT_STEPS &&
bash tools/gpu_run.sh r03k test
