#!/bin/bash
# Ring geometry sweep, ranks sharing the GPU (measurement tool): channels per
# ring x FIFO slot (VCCL_SLICE_BYTES; VCCL's step and partition unchanged)
# for RS / AG / AR of a 512 MiB bucket.
# tools/ring_geom_sweep.sh <label> [nranks]
set -e
O=gpurun_out/$1; N=${2:-2}; mkdir -p $O
export LAT_COLLS=${LAT_COLLS:-rs,ag,ar} LAT_SIZES=${LAT_SIZES:-536870912} LAT_ALGOS=ring LAT_STEPS=${LAT_STEPS:-10}
i=0
for ch in ${SWEEP_CH:-48 64}; do
  for slice in ${SWEEP_SLICE:-131072 262144 524288}; do
    i=$((i + 1))
    VCCL_CHANNELS_PER_RING=$ch VCCL_SLICE_BYTES=$slice timeout -k 10 200 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29600 + i)) tools/coll_latency.py \
      > $O/geom_n${N}_ch${ch}_slice${slice}.log 2> $O/geom_n${N}_ch${ch}_slice${slice}.err
  done
done
