set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r01q; mkdir -p $O
cd $R
SWEEP_MODE=lds SWEEP_ROUNDS=12 timeout -k 10 300 python -u tools/sweep_rc.py > $O/sweep_lds.log 2> $O/sweep_lds.err
timeout -k 10 300 python -u -m pytest tests/test_gpu_reduce_copy.py -x -q --timeout 200 --timeout-method thread > $O/pytest_rc.log 2>&1
