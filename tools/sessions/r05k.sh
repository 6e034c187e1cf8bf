#!/bin/bash
# round 5: ring latency 256 KiB - 64 MiB (ring forced), per-wave vs workgroup hand-off, 2 and 4 ranks sharing the GPU
export LAT_ALGOS=ring LAT_SIZES=262144,1048576,8388608,67108864 LAT_COLLS=ar,rs,ag LAT_STEPS=30
bash tools/ab_lib.sh r05k_n2 2 2 vccl_amd/lib/libvccl.so vccl_amd/lib/libvccl_wg.so && \
VCCL_CHANNELS_PER_RING=8 bash tools/ab_lib.sh r05k_n4 4 2 vccl_amd/lib/libvccl.so vccl_amd/lib/libvccl_wg.so
echo rc=$?
for f in gpurun_out/r05k_n*/lat_*.log; do echo "== $f"; cat $f; done
