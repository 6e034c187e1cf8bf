set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r02b; mkdir -p $O; cd $R
timeout -k 10 300 python -u tools/rc_offsets.py > $O/rc_offsets.log 2>&1
NCCL_ALGO=Ring SWEEP_BYTES=1073741824 SWEEP_STEPS=5 SWEEP_THREADS=1024 SWEEP_CPR=32 SWEEP_SLOT=131072,262144,524288,1048576,2097152 SWEEP_FENCES=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 tools/sweep_ring.py > $O/sweep_ring_1g.log 2>&1
NCCL_ALGO=Ring SWEEP_BYTES=67108864 SWEEP_STEPS=10 SWEEP_THREADS=1024 SWEEP_CPR=32 SWEEP_SLOT=131072,262144,524288,1048576 SWEEP_FENCES=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 tools/sweep_ring.py > $O/sweep_ring_64m.log 2>&1
bash tools/gpu_run.sh r02b n2
