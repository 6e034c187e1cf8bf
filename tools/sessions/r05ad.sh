#!/bin/bash
# round 5: ring hand-off A/B at 4 ranks sharing the GPU (library default channels: 48), 1 GiB fp32
# all-reduce, ring forced, output checked; VCCL_RING_WAVE 0 / 1 interleaved, 3 reps
O=gpurun_out/r05ad; mkdir -p $O
stop() { case $1 in 124|137|134|139) echo "fault/timeout rc=$1 at $2"; exit $1;; esac; }
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1"
for rep in 1 2 3; do for w in 0 1; do
  VCCL_RING_WAVE=$w VCCL_ALLOW_SHARED_DEVICE=1 timeout -k 10 180 $TR --master-port $((29500 + RANDOM % 400)) \
    tools/ring_ar_driver.py $((1<<30)) 6 >> $O/ar_n4_wave$w.jsonl 2>> $O/err.log; r=$?; echo "wave $w rep $rep rc=$r"; stop $r ar
  [ $r -ne 0 ] && exit $r
done; done
echo done
