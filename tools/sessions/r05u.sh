#!/bin/bash
# round 5: the per-wave SIMPLE ring as its own kernels (PART 4), chosen per comm — parity rows that run it
# (TEST_GEOM sets VCCL_RING_WAVE=1), the failure tests on both hand-offs, config 3/4 windows, then the
# spawned N=2 line with its ring_handoff rows
O=gpurun_out/r05u; mkdir -p $O
stop() { case $1 in 124|137|134|139) echo "fault/timeout rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_collectives.py tests/test_gpu_failure.py -x -v --timeout 300 \
  --timeout-method thread -k "multi_process_ranks or failure or lost_peer or abort_from" > $O/pytest_coll.log 2>&1; r=$?
echo "coll rc=$r: $(tail -1 $O/pytest_coll.log)"; stop $r coll; [ $r -ne 0 ] && exit $r
timeout -k 10 900 python -u -m pytest tests/test_gpu_workloads.py -x -v --timeout 600 --timeout-method thread \
  -k "4-test" > $O/pytest_work.log 2>&1; r=$?
echo "work rc=$r: $(tail -1 $O/pytest_work.log)"; stop $r work; [ $r -ne 0 ] && exit $r
timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_spawn_n2.json 2> $O/bench_spawn_n2.err; r=$?
echo "n2 rc=$r"; stop $r n2
echo done
