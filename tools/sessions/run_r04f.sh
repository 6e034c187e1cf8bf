# round-4 session f: LL128 (128-byte lines) parity, graph-mode LL probe,
# ring kernel counters (tools/pmc_ring.py)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04f; mkdir -p $O
export TMPDIR=/tmp
echo "== ll128 tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ll128" > $O/pytest_ll128.log 2>&1
echo "== ll graph probe $(date +%T)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29537 tools/ll_graph_probe.py > $O/ll_graph_probe.log 2> $O/ll_graph_probe.err
echo "== pmc ring $(date +%T)"
timeout -k 10 900 python -u tools/pmc_ring.py > $O/pmc_ring.log 2>&1
cp gpurun_out/pmc_ring.json $O/
echo "== done $(date +%T)"
