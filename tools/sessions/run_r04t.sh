#!/bin/bash
# r04t: (1) the cross-stream ordering worker with the ordering removed
# (VCCL_DEBUG_NO_MARK=1) — the test must be able to fail; (2) the N>1 bench
# line at 2 ranks sharing the GPU with the bound ordering event
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04t; mkdir -p $O; cd $R; export TMPDIR=/tmp
UID_HEX=$(python -c "from vccl_amd import nccl; print(nccl.unique_id_to_bytes(nccl.get_unique_id()).hex())" 2>/dev/null)
echo "no-mark run (expected to fail):"
python - > $O/nomark.log 2>&1 <<'PY'
import os, subprocess, sys
from vccl_amd import nccl
uid = nccl.get_unique_id()
hexid = nccl.unique_id_to_bytes(uid).hex()
env = dict(os.environ, VCCL_DEBUG_NO_MARK="1", VCCL_SPIN_TIMEOUT_S="10", VCCL_ALLOW_SHARED_DEVICE="1",
           VCCL_NCHANNELS="14", VCCL_SLOT_BYTES=str(256 << 10), VCCL_LL_THRESHOLD=str(1 << 20),
           VCCL_LL_MAX_BLOCKS="32", VCCL_DIRECT_THRESHOLD=str(4 << 20), VCCL_DIRECT_MAX_BLOCKS="16",
           VCCL_DIRECT_CHUNK_BYTES=str(1 << 20))
ps = [subprocess.Popen(["timeout", "-k", "5", "90", sys.executable, "tests/mp_stream_worker.py", str(r), "2", hexid],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(2)]
outs = [p.communicate()[0].decode(errors="replace")[-1500:] for p in ps]
print("exit codes", [p.returncode for p in ps])
print("\n".join(outs))
PY
tail -5 $O/nomark.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_n2.json 2> $O/bench_n2.err
echo done
