set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r01z; mkdir -p $O
cd $R
VCCL_LIB=$R/vccl_amd/lib/libvccl_e5c.so timeout -k 10 300 python -u -m pytest tests/test_gpu_reduce_copy.py -x -q --timeout 200 --timeout-method thread > $O/pytest_e5c.log 2>&1
timeout -k 10 600 python -u tools/ab_fp8.py vccl_amd/lib/libvccl.so vccl_amd/lib/libvccl_e5c.so 3 > $O/ab_fp8.log 2>&1
