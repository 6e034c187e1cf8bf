# round-3 A/B: ring RS / AG store policy and AG unroll; LL128 unroll (2 ranks sharing the GPU)
export LAT_COLLS=rs,ag LAT_SIZES=536870912 LAT_ALGOS=ring LAT_STEPS=10
bash tools/ab_lib.sh r03j 2 3 vccl_amd/lib/libvccl.so vccl_amd/lib/libvccl_outnt.so vccl_amd/lib/libvccl_agu8.so &&
export LAT_COLLS=ar,rs LAT_SIZES=262144,1048576,4194304 LAT_ALGOS=ll128 LAT_STEPS=30
bash tools/ab_lib.sh r03j_ll 2 3 vccl_amd/lib/libvccl.so vccl_amd/lib/libvccl_llu4.so &&
bash tools/gpu_run.sh r03j n2
