set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r01n; mkdir -p $O
cd $R
export VCCL_SPIN_TIMEOUT_S=20
timeout -k 10 300 python -u -m pytest tests/test_gpu_collectives.py -x -v --timeout 250 --timeout-method thread -k "net" > $O/pytest_net.log 2>&1
# net-forced ring all-reduce rate: 2 ranks sharing the GPU, loopback TCP
for B in 1048576 67108864 268435456; do
VCCL_NET_FORCE=1 VCCL_NTHREADS=512 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 2 --bytes $B --no-peer --no-extras > $O/bench_net_$B.json 2> $O/bench_net_$B.err
done
