set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r01r; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_c_api.py -x -v --timeout 200 --timeout-method thread > $O/pytest_c_api.log 2>&1
VCCL_ALLOW_SHARED_DEVICE=1 timeout -k 10 120 vccl_amd/lib/coll_perf -C allreduce -r 2 -b 8 -e 1073741824 -f 4 -n 10 -w 3 > $O/coll_perf_ar2.log 2>&1
