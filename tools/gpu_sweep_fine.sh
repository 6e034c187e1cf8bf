set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r01c; mkdir -p $O
cd $R
SWEEP_MODE=fine SWEEP_ROUNDS=12 timeout -k 10 300 python -u tools/sweep_rc.py > $O/sweep_fine.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu > $O/bench_prof.json 2> $O/bench_prof.err
