#!/usr/bin/env python3
"""Per-dtype reduce-copy PMC (tools/rc_dtypes.py under rocprofv3): issue and
stall cycles, VALU instructions and the GPU clock per launch, for one or more
library builds (PMC_LIBS = comma-separated .so paths; default the in-tree
build).  One --pmc pass per library (7 SQ + 2 GRBM counters fit one pass on
gfx950); rocprofv3 runs as a child with the program directly after `--`.
Prints one JSON line per (library, kernel).  Measurement tool."""
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
COUNTERS = ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU",
            "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "GRBM_GUI_ACTIVE", "GRBM_COUNT"]


def main():
    libs = os.environ.get("PMC_LIBS", os.path.join(ROOT, "vccl_amd", "lib", "libvccl.so")).split(",")
    for li, lib in enumerate(libs):
        d = os.path.join(OUT, f"pmc_dtypes_{li}")
        cmd = ["rocprofv3", "--pmc", *COUNTERS, "--kernel-trace", "--output-format", "csv", "-d", d,
               "-o", "run", "--", sys.executable, os.path.join(ROOT, "tools", "rc_dtypes.py")]
        subprocess.run(cmd, check=True, timeout=240, cwd=ROOT,
                       env={**os.environ, "VCCL_LIB": os.path.abspath(lib)})
        vals = defaultdict(lambda: defaultdict(list))
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = row.get("Kernel_Name", "")
                if "k_reduce_copy" in k:
                    vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
        for k, cs in vals.items():
            avg = {c: sum(v) / len(v) for c, v in cs.items()}
            print(json.dumps({"lib": os.path.basename(lib), "kernel": k.split("(")[0][-80:],
                              "launches": len(next(iter(cs.values()))), **{c: round(v) for c, v in avg.items()}}),
                  flush=True)


if __name__ == "__main__":
    main()
