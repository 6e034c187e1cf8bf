#!/bin/bash
# r04q: cost of the per-call ordering event (VCCL_DEBUG_NO_MARK=1, one
# stream) on eager small all-reduces, interleaved A/B, 2 ranks sharing the GPU
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04q; mkdir -p $O; cd $R; export TMPDIR=/tmp
run() {  # $1 tag, $2 nomark, $3.. driver args
  tag=$1; nm=$2; shift 2
  VCCL_DEBUG_NO_MARK=$nm timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) tools/ll_host_driver.py "$@" \
    > $O/$tag.json 2> $O/$tag.err
}
for rep in 1 2; do
  for nm in 0 1; do
    run ll8_nm${nm}_$rep $nm 8 2000 f16
    run ll64k_nm${nm}_$rep $nm 65536 2000 f16
    run ring1m_nm${nm}_$rep $nm 1048576 500 f32
  done
done
echo done
