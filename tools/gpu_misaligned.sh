set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-mis}; mkdir -p $O
cd $R
SWEEP_MODE=misaligned SWEEP_ROUNDS=10 timeout -k 10 200 python -u tools/sweep_rc.py > $O/sweep_misaligned.log 2>&1
SWEEP_MODE=fine SWEEP_ROUNDS=8 timeout -k 10 300 python -u tools/sweep_rc.py > $O/sweep_fine.log 2>&1
