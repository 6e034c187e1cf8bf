# Reduce-copy parity tests + collective tests + misaligned / fine sweeps.
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-rcc}; mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
SWEEP_MODE=misaligned SWEEP_ROUNDS=10 timeout -k 10 200 python -u tools/sweep_rc.py > $O/sweep_misaligned.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_n1.json 2> $O/bench_n1.err
