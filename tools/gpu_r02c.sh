set -e
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_run.sh r02c test:collectives n2
timeout -k 10 300 python -u tools/rc_offsets.py > gpurun_out/r02c/rc_offsets.log 2>&1
