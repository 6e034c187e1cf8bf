# round-4 session i: the GPU suite on the current tree, smoke, the N=1 line
# and its rocprofv3 kernel stats, the 4-rank rehearsal line
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_run.sh r04i test smoke bench prof nr:4
