#!/bin/bash
# n=3 reduce-scatter regression triage (coll_perf, ranks as processes)
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r03e; mkdir -p $O
P=vccl_amd/lib/coll_perf
export VCCL_ALLOW_SHARED_DEVICE=1 VCCL_SPIN_TIMEOUT_S=8 VCCL_NTHREADS=512 VCCL_LL_MAX_BLOCKS=32 VCCL_DIRECT_MAX_BLOCKS=16 VCCL_CHANNELS_PER_RING=8
for v in "default" "NCCL_PROTO=LL" "NCCL_ALGO=Ring" "VCCL_NCHANNELS=1" "VCCL_LL_THRESHOLD=8"; do
  echo "== $v"
  if [ "$v" = default ]; then
    timeout -k 5 60 $P -C reducescatter -r 3 -b 131040 -e 131040 -n 2 -w 1 -d int32 -o min > $O/rs3_default.log 2>&1; echo rc=$?
  else
    env $v timeout -k 5 60 $P -C reducescatter -r 3 -b 131040 -e 131040 -n 2 -w 1 -d int32 -o min > "$O/rs3_$v.log" 2>&1; echo rc=$?
  fi
done
VCCL_DEBUG=INFO timeout -k 5 60 $P -C reducescatter -r 3 -b 131040 -e 131040 -n 1 -w 0 -d int32 -o min > $O/rs3_debug.log 2>&1; echo rc=$?
