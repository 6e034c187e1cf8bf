set -e
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r02g; mkdir -p $O
bash tools/gpu_run.sh r02g test bench n2
SWEEP_MODE=misaligned SWEEP_ROUNDS=6 timeout -k 10 200 python -u tools/sweep_rc.py > $O/sweep_misaligned.log 2>&1
NCCL_ALGO=Ring SWEEP_BYTES=1073741824 SWEEP_STEPS=5 SWEEP_THREADS=512 SWEEP_CPR=16,32,48 SWEEP_SLOT=262144,524288,1048576 SWEEP_FENCES=0 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 tools/sweep_ring.py > $O/sweep_ring_1g.log 2>&1
