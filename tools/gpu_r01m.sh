set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r01m; mkdir -p $O
cd $R
timeout -k 10 120 python -u tools/host_cost.py > $O/host_cost.json 2> $O/host_cost.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/tools/pmc_traffic.py > $O/pmc.log 2>&1
cp $R/gpurun_out/pmc_traffic.json $O/ || true
