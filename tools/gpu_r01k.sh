set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r01k; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k beyond_2gib > $O/pytest_2gib.log 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_n1.json 2> $O/bench_n1.err
