#!/bin/bash
# round 5: the SIMPLE ring's HBM fraction in the 2-rank rehearsal against its channel count (96 vs the
# co-residency cap of 112 per rank), 1 GiB fp32 all-reduce, ring forced
O=gpurun_out/r05s; mkdir -p $O
stop() { case $1 in 124|137|134|139) echo "fault/timeout rc=$1 at $2"; exit $1;; esac; }
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
for rep in 1 2; do for ch in 64 96 112; do
  NCCL_NCHANNELS=$ch timeout -k 10 120 $TR --master-port $((29500 + RANDOM % 400)) \
    tools/ring_ar_driver.py $((1<<30)) 6 >> $O/ar_ch$ch.jsonl 2>> $O/err.log; r=$?; stop $r ar; [ $r -ne 0 ] && exit $r
done; done
echo done
