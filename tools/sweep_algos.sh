#!/bin/bash
# All-reduce size sweep per algorithm (auto / forced Ring / forced Direct with a
# raised direct threshold), N ranks sharing the box's GPUs: rehearsal of the
# LL / direct / ring crossovers.  Usage: tools/sweep_algos.sh N OUTDIR
set -e
N=${1:-8}
OUT=${2:-gpurun_out}
export VCCL_SPIN_TIMEOUT_S=20
if [ "$N" -gt 2 ]; then  # N ranks share one GPU: shrink grids so all are co-resident
  export VCCL_LL_MAX_BLOCKS=32 VCCL_DIRECT_MAX_BLOCKS=16 VCCL_NTHREADS=256 VCCL_CHANNELS_PER_RING=2
fi
port=29600
for algo in auto Ring Direct; do
  port=$((port + 1))
  if [ "$algo" = auto ]; then unset NCCL_ALGO; else export NCCL_ALGO=$algo; fi
  if [ "$algo" = Direct ]; then export VCCL_DIRECT_THRESHOLD=$((1 << 30)); else unset VCCL_DIRECT_THRESHOLD; fi
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus "$N" --sweep --no-peer \
    --steps 5 --warmup 2 > "$OUT/sweep_${N}rank_$algo.json" 2> "$OUT/sweep_${N}rank_$algo.log"
done
