#!/bin/bash
# round 5: isolate the 3-net failure of the per-wave hand-off
O=gpurun_out/r05c; mkdir -p $O
stop() { case $1 in 124|137|134|139) echo "fault/timeout rc=$1 at $2"; exit $1;; esac; }
t() { local label=$1; shift; env "$@" timeout -k 10 300 python -u -m pytest tests/test_gpu_collectives.py -q \
  --timeout 240 --timeout-method thread -k "multi_process_ranks and ($K)" > $O/$label.log 2>&1; local r=$?
  echo "$label rc=$r: $(tail -1 $O/$label.log)"; stop $r $label; }
K="3-net or 2-net"; t net_ws_1 X=1
K="3-net"; t net_ws_2 X=1
K="3-net"; t net_wg VCCL_LIB=$PWD/vccl_amd/lib/libvccl_wg.so
K="3-test or 2-test or 4-test"; t fences_ws VCCL_FENCES=1
