set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r01v; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_reduce_copy.py tests/test_gpu_api.py -x -q --timeout 200 --timeout-method thread > $O/pytest_rc.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err
