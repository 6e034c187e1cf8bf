# GPU tests + a 2-rank shared-GPU rehearsal of the N>1 bench line (extras incl.).
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-coll}; mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
VCCL_SPIN_TIMEOUT_S=20 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 2 \
  --rs-ag-bytes 1073741824 > $O/bench_n2.json 2> $O/bench_n2.err
timeout -k 10 300 python -u bench.py > $O/bench_n1.json 2> $O/bench_n1.err
