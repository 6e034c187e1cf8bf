#!/bin/bash
# round 5: one credit poller per workgroup — parity subset, ring latency A/B, 1 GiB throughput A/B
O=gpurun_out/r05o; mkdir -p $O
stop() { case $1 in 124|137|134|139) echo "fault/timeout rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_collectives.py tests/test_gpu_failure.py -q -x --timeout 240 \
  --timeout-method thread -k "multi_process_ranks or failure or trace or alternating or stress" > $O/pytest.log 2>&1; rc=$?
echo "parity rc=$rc: $(tail -1 $O/pytest.log)"; stop $rc parity; [ $rc -ne 0 ] && exit $rc
export LAT_ALGOS=ring LAT_SIZES=262144,1048576,8388608,67108864 LAT_COLLS=ar,rs,ag LAT_STEPS=30
bash tools/ab_lib.sh r05o/n2 2 2 vccl_amd/lib/libvccl.so vccl_amd/lib/libvccl_wg.so || exit 1
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
for rep in 1 2; do for lib in libvccl libvccl_wg; do for ch in 16 96; do
  VCCL_LIB=$PWD/vccl_amd/lib/$lib.so NCCL_NCHANNELS=$ch timeout -k 10 120 $TR --master-port $((29500 + RANDOM % 400)) \
    tools/ring_ar_driver.py $((1<<30)) 6 >> $O/ar_${lib}_ch$ch.jsonl 2>> $O/err.log; stop $? ar
done; done; done
echo done
