# Net-forced ring all-reduce (2 ranks sharing the GPU, loopback TCP): channels x slot size
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r01p; mkdir -p $O
cd $R
export VCCL_SPIN_TIMEOUT_S=20 VCCL_NET_FORCE=1 VCCL_NTHREADS=512
for CH in 4 8 16; do for SLOT in 524288 2097152; do
VCCL_NET_NCHANNELS=$CH VCCL_SLOT_BYTES=$SLOT timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 2 --bytes 268435456 --no-peer --no-extras > $O/net_${CH}_${SLOT}.json 2> $O/net_${CH}_${SLOT}.err
python -c "import json; d=json.load(open('$O/net_${CH}_${SLOT}.json')); c=d['config']; print('channels $CH slot $SLOT', c['busbw_per_rank'], 'GB/s busbw', c['correct'])" | tee -a $O/sweep.log
done; done
