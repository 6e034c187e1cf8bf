#!/bin/bash
# round 5: the whole GPU suite on the current library, then the spawned N=4 rehearsal line
O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1; rc=$?; echo "suite rc=$rc: $(tail -1 $O/pytest_gpu.log)"
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 600 python bench.py --gpus 4 --steps 5 --warmup 2 > $O/bench_spawn_n4.json 2> $O/bench_spawn_n4.err
echo "spawn4 rc=$?"; head -c 400 $O/bench_spawn_n4.json
exit $rc
