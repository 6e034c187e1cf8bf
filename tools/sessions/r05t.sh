#!/bin/bash
# round 5: where the 2-rank ring loses HBM rate — FIFO memory type (0 uncached, 1 fine-grained,
# 2 coarse) at 96 channels, 1 GiB fp32 all-reduce, ring forced, output checked
O=gpurun_out/r05t; mkdir -p $O
stop() { case $1 in 124|137|134|139) echo "fault/timeout rc=$1 at $2"; exit $1;; esac; }
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
export VCCL_SPIN_TIMEOUT_S=10
for rep in 1 2; do for m in 0 1 2; do
  VCCL_FIFO_ALLOC=$m NCCL_NCHANNELS=96 timeout -k 10 120 $TR --master-port $((29500 + RANDOM % 400)) \
    tools/ring_ar_driver.py $((1<<30)) 6 >> $O/ar_alloc$m.jsonl 2>> $O/err.log; r=$?; echo "alloc $m rep $rep rc=$r"; stop $r ar
done; done
echo done
