set -e
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r02e; mkdir -p $O
bash tools/gpu_run.sh r02e test:collectives
SWEEP_MODE=misaligned SWEEP_ROUNDS=6 timeout -k 10 200 python -u tools/sweep_rc.py > $O/sweep_misaligned.log 2>&1
export VCCL_SPIN_TIMEOUT_S=20 VCCL_CHANNELS_PER_RING=2 VCCL_NTHREADS=256 VCCL_LL_MAX_BLOCKS=32 VCCL_DIRECT_MAX_BLOCKS=16
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 tools/coll_latency.py > $O/lat_n4.log 2> $O/lat_n4.err
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29542 tools/coll_latency.py > $O/lat_n8.log 2> $O/lat_n8.err
