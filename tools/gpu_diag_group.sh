# Which ring-only multi-process group cases time out, with 2 streams vs 1.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-diag}; mkdir -p $O
cd $R
timeout -k 10 200 python -u -m pytest tests/test_gpu_collectives.py -m gpu -v --timeout 150 --timeout-method thread -k "ring_only" > $O/ring_only_2streams.log 2>&1
echo "rc=$?" >> $O/ring_only_2streams.log
VCCL_TEST_GROUP_STREAMS=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_collectives.py -m gpu -v --timeout 150 --timeout-method thread -k "ring_only" > $O/ring_only_1stream.log 2>&1
echo "rc=$?" >> $O/ring_only_1stream.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_collectives.py -m gpu -v --timeout 150 --timeout-method thread -k "group_fusion_single" > $O/group_single.log 2>&1
echo "rc=$?" >> $O/group_single.log
