set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r01t; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
