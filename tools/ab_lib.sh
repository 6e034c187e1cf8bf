#!/bin/bash
# Interleaved A/B of library builds on tools/coll_latency.py (ranks sharing
# the GPU):  tools/ab_lib.sh <label> <nranks> <reps> <lib.so> [<lib.so> ...]
# LAT_* env as coll_latency.py.  Outputs gpurun_out/<label>/lat_<lib>_<rep>.log
set -e
O=gpurun_out/$1; N=$2; REPS=$3; shift 3
mkdir -p $O
for rep in $(seq 1 $REPS); do
  for lib in "$@"; do
    b=$(basename $lib .so)
    VCCL_LIB=$PWD/$lib timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
      --master-addr 127.0.0.1 --master-port $((29550 + rep)) tools/coll_latency.py > $O/lat_${b}_$rep.log 2> $O/lat_${b}_$rep.err
  done
done
