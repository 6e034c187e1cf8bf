"""A/B of two library builds on the per-dtype reduce-copy rates (bench.py
extras), alternating in separate processes: python tools/ab_fp8.py LIB_A LIB_B ROUNDS."""
import json
import os
import subprocess
import sys

libs, rounds = sys.argv[1:3], int(sys.argv[3])
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = ("import sys,json; sys.path.insert(0, %r); import bench; "
        "print(json.dumps(bench.bench_rc_dtypes(256 << 20)))" % root)
for r in range(rounds):
    for lib in libs:
        env = dict(os.environ, VCCL_LIB=os.path.abspath(lib))
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                             timeout=300, check=True).stdout.strip().splitlines()[-1]
        rows = {x["dtype"]: x["GB/s"] for x in json.loads(out)}
        print(json.dumps({"round": r, "lib": os.path.basename(lib), **rows}), flush=True)
