#!/usr/bin/env python3
"""PMC counters per reduce-copy shape (tools/rc_shape_driver.py), one
rocprofv3 `--pmc` pass per counter group (kernel trace only, no sys/runtime
trace), each under its own hard time limit.  Per MI355X_MICROARCH.md §HBM:
FETCH_SIZE is doubled on gfx950 (wide streaming reads tallied at half),
WRITE_SIZE is exact for 16-B-per-lane stores; both in KiB.

Launches are attributed to shapes in issue order (13 per shape, the first 3
dropped).  Writes gpurun_out/pmc_shapes.json.  This script never touches the
GPU itself: rocprofv3 runs as a child with python3 directly after `--`.
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
SHAPES = ["2to2", "2to2_o3", "2to2_plain1", "copy", "2to1"]
PASSES = [["FETCH_SIZE"], ["WRITE_SIZE"],
          ["SQ_INSTS_VMEM_WR", "SQ_INSTS_VMEM_RD", "SQ_WAVES", "SQ_BUSY_CYCLES"],
          ["TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"]]
ALGO = {"2to2": 4, "2to2_o3": 4, "2to2_plain1": 4, "copy": 2, "2to1": 3}


def run_pass(counters):
    d = os.path.join(OUT, "pmc_shapes", "_".join(c.lower() for c in counters))
    cmd = ["timeout", "-s", "KILL", "90", "rocprofv3", "--pmc", *counters, "--output-format", "csv",
           "-d", d, "-o", "run", "--", sys.executable, os.path.join(ROOT, "tools", "rc_shape_driver.py"),
           *SHAPES]
    subprocess.run(cmd, check=True, cwd="/tmp")
    return d


def parse(d):
    """{counter: [value per dispatch, in dispatch order]} for k_reduce_copy."""
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "k_reduce_copy" in row.get("Kernel_Name", ""):
                rows.append(row)
    out = {}
    for row in sorted(rows, key=lambda r: int(r.get("Dispatch_Id", 0))):
        out.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return out


def main():
    res = {s: {} for s in SHAPES}
    errors = {}
    for counters in PASSES:
        try:
            vals = parse(run_pass(counters))
        except subprocess.CalledProcessError as e:  # an unknown counter name: record, go on
            errors["+".join(counters)] = f"rc {e.returncode}"
            if e.returncode in (-9, 137, 124):  # killed at its limit: stop here
                break
            continue
        for c, v in vals.items():
            for i, s in enumerate(SHAPES):
                per = v[13 * i + 3:13 * (i + 1)]
                res[s][c] = sum(per) / len(per) if per else None
    for s in SHAPES:
        r = res[s]
        algo = ALGO[s] * (1 << 28)
        if r.get("FETCH_SIZE") is not None and r.get("WRITE_SIZE") is not None:
            hbm = (2 * r["FETCH_SIZE"] + r["WRITE_SIZE"]) * 1024
            r["read_bytes_corrected"] = int(2 * r["FETCH_SIZE"] * 1024)
            r["write_bytes"] = int(r["WRITE_SIZE"] * 1024)
            r["traffic_over_algorithmic"] = round(hbm / algo, 4)
        r["algorithmic_bytes"] = algo
    out = {"shapes": res, "errors": errors, "method": "rocprofv3 --pmc, one pass per counter group; FETCH_SIZE x2 (gfx950)"}
    json.dump(out, open(os.path.join(OUT, "pmc_shapes.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
