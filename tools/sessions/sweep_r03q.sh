# round 3: channels beyond MAXCHANNELS 64 (2 ranks sharing the GPU), 512 MiB RS / AG / AR, ring
set -e
O=gpurun_out/r03q; mkdir -p $O
export LAT_COLLS=rs,ag,ar LAT_SIZES=536870912 LAT_ALGOS=ring LAT_STEPS=10
i=0
for ch in 64 96 128; do
  i=$((i + 1))
  VCCL_LIB=$PWD/vccl_amd/lib/libvccl_ch128.so VCCL_CHANNELS_PER_RING=$ch timeout -k 10 200 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29620 + i)) tools/coll_latency.py \
    > $O/ch${ch}.log 2> $O/ch${ch}.err
done
