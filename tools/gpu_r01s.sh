set -e
R=$GRAFT_REPO_ROOT; RUN=${RUN:-r01s}; O=$R/gpurun_out/$RUN; mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_n1.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu > $O/bench_prof.json 2> $O/bench_prof.err
