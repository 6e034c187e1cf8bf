#!/bin/bash
# r04r: the ordering event's release scope (VCCL_EVENT_FENCE 0 system /
# 1 device / 2 none) vs no event (VCCL_DEBUG_NO_MARK=1) on eager small
# all-reduces, interleaved, 2 ranks sharing the GPU
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04r; mkdir -p $O; cd $R; export TMPDIR=/tmp
run() {  # $1 tag, $2 fence mode, $3 nomark, $4.. driver args
  tag=$1; fm=$2; nm=$3; shift 3
  VCCL_EVENT_FENCE=$fm VCCL_DEBUG_NO_MARK=$nm timeout -k 10 120 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) \
    tools/ll_host_driver.py "$@" > $O/$tag.json 2> $O/$tag.err
}
for rep in 1 2; do
  for v in "0 0" "1 0" "2 0" "0 1"; do
    set -- $v
    run ll8_f$1_nm$2_$rep $1 $2 8 2000 f16
    run ring1m_f$1_nm$2_$rep $1 $2 1048576 500 f32
  done
done
echo done
