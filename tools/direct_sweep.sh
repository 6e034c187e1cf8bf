set -e
export LAT_COLLS=ar,rs,ag LAT_SIZES=8388608,67108864,268435456 LAT_ALGOS=ring,direct LAT_STEPS=10
for n in 4 2; do
 for v in "64 16777216" "128 16777216" "64 67108864" "128 67108864"; do
  set -- $v
  VCCL_DIRECT_MAX_BLOCKS=$1 VCCL_DIRECT_CHUNK_BYTES=$2 bash tools/gpu_run.sh r03i_n${n}_b$1_c$(($2>>20)) lat:$n
 done
done
