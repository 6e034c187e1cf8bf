set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04e; mkdir -p $O
export TMPDIR=/tmp
echo "== mixed $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_collectives.py -m gpu -x -q --timeout 240 --timeout-method thread -k "mixed_direct or zero_pattern" > $O/pytest_mixed.log 2>&1
echo "== n2 $(date +%T)"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_n2.json 2> $O/bench_n2.err
echo "== ab2 $(date +%T)"
LAT_SIZES=262144,1048576,8388608 LAT_ALGOS=ll128,ring LAT_COLLS=ar,rs,ag bash tools/ab_lib.sh r04e/ab2 2 2 vccl_amd/lib/libvccl.so vccl_amd/lib/libvccl_l128.so
echo "== ab4 $(date +%T)"
LAT_SIZES=262144,1048576,8388608 LAT_ALGOS=ll128,ring LAT_COLLS=ar,rs,ag bash tools/ab_lib.sh r04e/ab4 4 2 vccl_amd/lib/libvccl.so vccl_amd/lib/libvccl_l128.so
echo "== done $(date +%T)"
