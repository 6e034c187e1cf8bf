# round-4 session h: FIFO slot = 1 / 2 MiB (VCCL's 2-step slices) vs the
# 512 KiB step, ring timing at 96 and 16 channels; latency A/B; the LL chain
# geometry; N=2 line
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04h; mkdir -p $O
export TMPDIR=/tmp
echo "== chain tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_collectives.py -m gpu -x -q --timeout 300 --timeout-method thread -k "chain or 4-test or net_ll128" > $O/pytest_chain.log 2>&1
echo "== ring timing $(date +%T)"
PMC_RING_TIMING_ONLY=1 PMC_RING_OUT=ring_slices.json PMC_RING_VARIANTS=alloc0_ch96,slice1m_ch96,slice2m_ch96,alloc0_ch16,slice1m_ch16 timeout -k 10 600 python -u tools/pmc_ring.py > $O/ring_slices.log 2>&1
cp gpurun_out/ring_slices.json $O/
echo "== slice latency A/B $(date +%T)"
LAT_SIZES=262144,1048576,8388608,67108864,268435456 LAT_ALGOS=ring LAT_COLLS=ar,rs,ag LAT_STEPS=20 bash tools/ab_env.sh r04h/ab_slice 2 2 - VCCL_SLICE_BYTES=1048576
echo "== n2 $(date +%T)"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_n2.json 2> $O/bench_n2.err
echo "== done $(date +%T)"
