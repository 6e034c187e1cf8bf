set -e
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r02i; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_run.sh r02i test bench prof n2
timeout -k 10 400 python -u tools/pmc_traffic.py > $O/pmc_traffic.log 2>&1
cp gpurun_out/pmc_traffic.json $O/ 2>/dev/null || true
LAT_COLLS=ar,rs,ag LAT_SIZES=65536,1048576,8388608,67108864 LAT_ALGOS=auto,ring,direct LAT_STEPS=20 VCCL_SPIN_TIMEOUT_S=20 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29551 tools/coll_latency.py > $O/lat_n2.log 2> $O/lat_n2.err
timeout -k 10 200 python -u tools/rc_dtypes.py > $O/dtypes_default.log 2>&1
VCCL_LIB=$R/vccl_amd/lib/libvccl_e5.so timeout -k 10 200 python -u tools/rc_dtypes.py > $O/dtypes_e5cvt.log 2>&1
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $R/$O/pmc_valu_default -o run -- python3 $R/tools/rc_dtypes.py > $R/$O/pmc_valu_default.log 2>&1)
(cd /tmp && VCCL_LIB=$R/vccl_amd/lib/libvccl_e5.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $R/$O/pmc_valu_e5 -o run -- python3 $R/tools/rc_dtypes.py > $R/$O/pmc_valu_e5.log 2>&1)
