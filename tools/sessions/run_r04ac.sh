#!/bin/bash
# r04ac: kernel durations of the eager LL all-reduce (8 B / 64 KiB fp16) and
# the 1 MiB ring, 2 ranks sharing the GPU, both under rocprofv3 --kernel-trace
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04ac; mkdir -p $O; cd $R; export TMPDIR=/tmp
prof() {  # $1 tag, $2.. driver args
  tag=$1; shift
  P=$((29700 + RANDOM % 200))
  for r in 0 1; do
    (cd /tmp && RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$P timeout -k 10 120 \
      rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag/rank$r -o run -- \
      python3 $R/tools/ll_host_driver.py "$@" > $O/$tag/rank$r.json 2> $O/$tag/rank$r.err) &
  done
  wait
}
mkdir -p $O/ll8 $O/ll64k $O/ring1m
prof ll8 8 2000 f16
prof ll64k 65536 2000 f16
prof ring1m 1048576 500 f32
echo done
