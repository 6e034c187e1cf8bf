#!/bin/bash
# round 5: per-wave ring hand-off — parity, then A/B against the workgroup hand-off (libvccl_wg.so)
O=gpurun_out/r05b; mkdir -p $O
stop() { case $1 in 124|137|134|139) echo "fault/timeout rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_collectives.py tests/test_gpu_failure.py -q -x \
  --timeout 300 --timeout-method thread > $O/pytest_coll.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -3 $O/pytest_coll.log
stop $rc parity; [ $rc -ne 0 ] && exit $rc
run() {  # label lib env...
  local label=$1 lib=$2; shift 2
  env VCCL_LIB=$PWD/$lib "$@" timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 200)) tools/ring_ar_driver.py $((1<<30)) 6 \
    >> $O/ab_$label.jsonl 2>> $O/ab_$label.err
  local r=$?; stop $r $label; return 0
}
for rep in 1 2; do
  for lib in libvccl.so libvccl_wg.so; do
    run ${lib%.so}_ch96 vccl_amd/lib/$lib NCCL_NCHANNELS=96
    run ${lib%.so}_ch16 vccl_amd/lib/$lib
  done
done
for lib in libvccl.so libvccl_wg.so; do
  for ch in 96 16; do
    env VCCL_LIB=$PWD/vccl_amd/lib/$lib NCCL_NCHANNELS=$ch TRACE_BYTES=$((512<<20)) timeout -k 10 120 \
      python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $((29700 + RANDOM % 200)) tools/ring_trace.py > $O/trace_${lib%.so}_ch$ch.jsonl 2> $O/trace_${lib%.so}_ch$ch.err
    stop $? trace
  done
done
for f in $O/ab_*.jsonl; do echo "$f"; cat $f; done
