#!/bin/bash
# r04p: host enqueue cost vs device time of eager small all-reduces
# (tools/ll_host_driver.py), 2 ranks sharing the GPU; then rank 0 under the
# HIP runtime trace for the per-API split.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04p; mkdir -p $O; cd $R; export TMPDIR=/tmp
run() {  # $1 tag, $2.. driver args
  tag=$1; shift
  timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29600 + RANDOM % 300)) tools/ll_host_driver.py "$@" > $O/$tag.json 2> $O/$tag.err
}
run ll8 8 2000 f16
run ll16k 16384 2000 f16
run ring1m 1048576 500 f32
# rank 1 plain, rank 0 under the runtime trace
P=$((29900 + RANDOM % 50))
env RANK=1 LOCAL_RANK=1 WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$P timeout -k 10 120 python tools/ll_host_driver.py 8 2000 f16 > /dev/null 2> $O/trace_r1.err &
(cd /tmp && RANK=0 LOCAL_RANK=0 WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$P timeout -k 10 120 rocprofv3 --hip-runtime-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/ll_host_driver.py 8 2000 f16 > $O/trace_r0.json 2> $O/trace_r0.err)
wait
echo done
