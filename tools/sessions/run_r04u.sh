#!/bin/bash
# r04u: nccl-tests-style C-API latency sweep (tools/coll_perf.hip, no Python
# in the loop), 2 ranks sharing the GPU, ordering event bound (default) vs
# marker; fp16 all-reduce 8 B - 1 MiB, fp32 8 B - 64 MiB
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04u; mkdir -p $O; cd $R; export TMPDIR=/tmp
export VCCL_ALLOW_SHARED_DEVICE=1 VCCL_SPIN_TIMEOUT_S=20
for le in 1 0; do
  VCCL_LAUNCH_EVENT=$le timeout -k 10 200 vccl_amd/lib/coll_perf -C allreduce -r 2 -b 8 -e 1048576 -f 4 -n 500 -w 50 -d half \
    > $O/ar_half_le$le.txt 2>&1 || exit 1
  VCCL_LAUNCH_EVENT=$le timeout -k 10 200 vccl_amd/lib/coll_perf -C allreduce -r 2 -b 8 -e 67108864 -f 8 -n 100 -w 10 -d float \
    > $O/ar_float_le$le.txt 2>&1 || exit 1
done
echo done
