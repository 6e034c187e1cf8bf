#!/bin/bash
# round 5: net cases x3 on the per-wave hand-off (sizes ordered before the tail), then r05b's parity + A/B
O=gpurun_out/r05d; mkdir -p $O
stop() { case $1 in 124|137|134|139) echo "fault/timeout rc=$1 at $2"; exit $1;; esac; }
for i in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_collectives.py -q --timeout 240 --timeout-method thread \
    -k "multi_process_ranks and net" > $O/net_$i.log 2>&1; r=$?; echo "net $i rc=$r: $(tail -1 $O/net_$i.log)"; stop $r net
done
bash tools/sessions/r05b.sh
# item 5: two-destination reduce-copy geometry sweep
SWEEP_MODE=twodst_geom SWEEP_ROUNDS=8 timeout -k 10 300 python tools/sweep_rc.py > gpurun_out/r05d/twodst_geom.jsonl 2> gpurun_out/r05d/twodst_geom.err
echo "sweep rc=$?"; head -12 gpurun_out/r05d/twodst_geom.jsonl
