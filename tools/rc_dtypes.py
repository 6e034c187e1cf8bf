"""Run bench.py's per-dtype reduce-copy leg alone (for rocprofv3 PMC passes)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

print(json.dumps(bench.bench_rc_dtypes(256 << 20, steps=5, warmup=1)))
