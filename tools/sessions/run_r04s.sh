#!/bin/bash
# r04s: ordering event bound to the kernel (VCCL_LAUNCH_EVENT=1, default) vs
# a recorded marker (0), eager small all-reduces, interleaved, 2 ranks
# sharing the GPU; then the cross-stream ordering tests
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04s; mkdir -p $O; cd $R; export TMPDIR=/tmp
run() {  # $1 tag, $2 launch-event mode, $3.. driver args
  tag=$1; le=$2; shift 2
  VCCL_LAUNCH_EVENT=$le timeout -k 10 120 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) \
    tools/ll_host_driver.py "$@" > $O/$tag.json 2> $O/$tag.err
}
for rep in 1 2; do
  for le in 0 1; do
    run ll8_le${le}_$rep $le 8 2000 f16
    run ll64k_le${le}_$rep $le 65536 2000 f16
    run ring1m_le${le}_$rep $le 1048576 500 f32
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_collectives.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "alternating or group_fusion or graph" > $O/pytest_streams.log 2>&1
echo done
