#!/bin/bash
# round 5: interleaved A/B, per-wave (libvccl) vs workgroup (libvccl_wg) ring hand-off, 2 ranks sharing the GPU
O=gpurun_out/r05f; mkdir -p $O
stop() { case $1 in 124|137|134|139) echo "fault/timeout rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_collectives.py tests/test_gpu_failure.py -q -x \
  --timeout 240 --timeout-method thread -k "multi_process_ranks or failure or split or trace" > $O/pytest.log 2>&1; rc=$?
echo "parity rc=$rc: $(tail -1 $O/pytest.log)"; stop $rc parity; [ $rc -ne 0 ] && exit $rc
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
for rep in 1 2 3; do
  for lib in libvccl libvccl_ns libvccl_wg; do
    for ch in 16 48 96; do
      VCCL_LIB=$PWD/vccl_amd/lib/$lib.so NCCL_NCHANNELS=$ch timeout -k 10 120 $TR --master-port $((29500 + RANDOM % 400)) tools/ring_ar_driver.py $((1<<30)) 6 \
        >> $O/ar_${lib}_ch$ch.jsonl 2>> $O/err.log; stop $? ar
    done
    for ch in 16 96; do
      VCCL_LIB=$PWD/vccl_amd/lib/$lib.so NCCL_NCHANNELS=$ch timeout -k 10 180 $TR --master-port $((29500 + RANDOM % 400)) bench.py --workload rs_ag --steps 10 \
        --warmup 2 --no-cpu --no-extras >> $O/rsag_${lib}_ch$ch.jsonl 2>> $O/err.log; stop $? rsag
    done
  done
done
python - <<'PY'
import glob, json, statistics as st
for f in sorted(glob.glob("gpurun_out/r05f/*.jsonl")):
    rows = [json.loads(l) for l in open(f) if l.startswith("{")]
    if "ar_" in f:
        med = [st.median(r["us"]) for r in rows]
        print(f.split("/")[-1], "AR us per rep", med, "correct", all(r["correct"] for r in rows))
    else:
        print(f.split("/")[-1], "RS", [r["config"]["rs_busbw"] for r in rows], "AG", [r["config"]["ag_busbw"] for r in rows],
              "ok", [r["config"]["correct"] for r in rows])
PY
