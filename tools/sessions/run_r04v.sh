#!/bin/bash
# r04v: kernel durations of the eager LL all-reduce (coll_perf, 2 ranks
# sharing the GPU, every rank under rocprofv3 --kernel-trace --stats)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04v; mkdir -p $O; cd $R; export TMPDIR=/tmp
export VCCL_ALLOW_SHARED_DEVICE=1 VCCL_SPIN_TIMEOUT_S=20
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  $R/vccl_amd/lib/coll_perf -C allreduce -r 2 -b 8 -e 2048 -f 16 -n 500 -w 50 -d half > $O/ar_half.txt 2>&1
echo rc=$?
