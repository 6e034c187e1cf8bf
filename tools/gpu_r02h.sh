set -e
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r02h; mkdir -p $O
bash tools/gpu_run.sh r02h test bench n2
SWEEP_MODE=misaligned SWEEP_ROUNDS=6 timeout -k 10 200 python -u tools/sweep_rc.py > $O/sweep_misaligned.log 2>&1
