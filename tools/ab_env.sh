#!/bin/bash
# Interleaved A/B of environment settings on tools/coll_latency.py (ranks
# sharing the GPU):  tools/ab_env.sh <label> <nranks> <reps> <VAR=val[,VAR=val]> ...
# ("-" = no extra setting).  LAT_* env as coll_latency.py.
# Outputs gpurun_out/<label>/lat_<k>_<rep>.log, k = index of the setting.
set -e
O=gpurun_out/$1; N=$2; REPS=$3; shift 3
mkdir -p $O
for rep in $(seq 1 $REPS); do
  k=0
  for spec in "$@"; do
    E=""; [ "$spec" != "-" ] && E=$(echo "$spec" | tr ',' ' ')
    echo "$k $spec" > $O/setting_$k.txt
    env $E timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
      --master-addr 127.0.0.1 --master-port $((29570 + rep * 8 + k)) tools/coll_latency.py > $O/lat_${k}_$rep.log 2> $O/lat_${k}_$rep.err
    k=$((k + 1))
  done
done
