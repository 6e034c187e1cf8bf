set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r01p; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_collectives.py -x -v --timeout 250 --timeout-method thread -k "net" > $O/pytest_net.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash tools/gpu_net_sweep.sh
