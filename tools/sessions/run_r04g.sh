# round-4 session g: the GPU suite with fine-grained FIFOs; FIFO allocation
# latency A/B; graph-mode LL rows on fresh vs one shared capture stream
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04g; mkdir -p $O
export TMPDIR=/tmp
echo "== graph probe fresh $(date +%T)"
PROBE_SIZES=8,8,8,8,8,1024,1024 PROBE_DTYPES=f16 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29537 tools/ll_graph_probe.py > $O/ll_graph_fresh.log 2> $O/ll_graph_fresh.err
echo "== graph probe shared $(date +%T)"
PROBE_STREAM=shared PROBE_SIZES=8,8,8,8,8,1024,1024 PROBE_DTYPES=f16 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29538 tools/ll_graph_probe.py > $O/ll_graph_shared.log 2> $O/ll_graph_shared.err
echo "== fifo alloc A/B $(date +%T)"
LAT_SIZES=8,8192,65536,1048576,8388608,67108864 LAT_ALGOS=auto,ring,direct,ll128 LAT_COLLS=ar,rs,ag bash tools/ab_env.sh r04g/ab_fifo 2 2 VCCL_FIFO_ALLOC=0 VCCL_FIFO_ALLOC=1
echo "== suite fine-grained $(date +%T)"
VCCL_FIFO_ALLOC=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_fifo1.log 2>&1
echo "== done $(date +%T)"
