"""Print the algorithm choice around the LL / ring boundaries at 2 ranks on one GPU."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"
os.environ["VCCL_DEBUG"] = "INFO"
from vccl_amd import nccl  # noqa: E402
comms = nccl.Comm.init_all([0, 0])
for coll, count in ((0, 16 << 10), (0, 17 << 10), (1, 16 << 10), (1, 17 << 10), (2, 17 << 10)):
    print(coll, count, comms[0].coll_algo(coll, count, 7), flush=True)
for c in comms:
    c.destroy()
