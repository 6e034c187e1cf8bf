set -e
O=gpurun_out/r04ar; mkdir -p $O
for rep in 1 2; do
for v in base op; do
  if [ $v = base ]; then LIBV=vccl_amd/lib/libvccl.so; else LIBV=vccl_amd/lib/libvccl_$v.so; fi
  VCCL_LIB=$PWD/$LIBV TRACE_BYTES=$((1<<30)) timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2955$rep tools/ring_trace.py > $O/trace_${v}_$rep.log 2>&1
  echo "$v $rep done"
done
done
