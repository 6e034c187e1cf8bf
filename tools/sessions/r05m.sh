#!/bin/bash
# round 5: slot timeline at 1 MiB (latency regime), per-wave vs workgroup hand-off
O=gpurun_out/r05m; mkdir -p $O
for lib in libvccl libvccl_wg; do
  VCCL_LIB=$PWD/vccl_amd/lib/$lib.so TRACE_BYTES=$((1<<20)) timeout -k 10 120 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29700 + RANDOM % 200)) tools/ring_trace.py \
    > $O/trace_${lib}_1m.jsonl 2> $O/trace_${lib}_1m.err || exit 1
done
echo ok
