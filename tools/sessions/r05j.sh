#!/bin/bash
# round 5: soak of the per-wave ring hand-off — the multi-process parity rows three times
O=gpurun_out/r05j; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 600 python -u -m pytest tests/test_gpu_collectives.py -q --maxfail 3 --timeout 240 --timeout-method thread \
    -k "multi_process_ranks or group_plan_stress or alternating_streams or group_zero or graph" > $O/soak_$i.log 2>&1; rc=$?
  echo "soak $i rc=$rc: $(tail -1 $O/soak_$i.log)"
  case $rc in 124|137|134|139) exit $rc;; esac
done
