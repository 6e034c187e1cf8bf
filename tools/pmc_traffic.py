#!/usr/bin/env python3
"""HBM traffic per launch of the reduce-copy kernel from rocprofv3 PMC counters.

Two separate `--pmc` passes (FETCH_SIZE and WRITE_SIZE do not fit one pass on
gfx950, MI355X_MICROARCH.md §rocprofv3 PMC slots), kernel-trace only, of
`bench.py --no-cpu`.  Per MI355X_MICROARCH.md §HBM: FETCH_SIZE reports exactly
half of the bytes of a wide coalesced streaming read on gfx950, so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores; both in KiB.

Writes gpurun_out/pmc_traffic.json (copy it to profiles/pmc_traffic.json).
This script itself never touches the GPU: rocprofv3 runs as a child process
with the program directly after `--`.
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
KERNEL = "k_reduce_copy<vccl::FnSum<float>, 2, 1,"


def run_pass(counter):
    d = os.path.join(OUT, f"pmc_{counter.lower()}")
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "run", "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2", "--no-cpu"]
    subprocess.run(cmd, check=True, timeout=180, cwd=ROOT)
    return d


def parse(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = []
    for f in files:
        for row in csv.DictReader(open(f)):
            if KERNEL in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    res = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = run_pass(counter)
        res[counter] = parse(d, counter)
    fetch, write = res["FETCH_SIZE"], res["WRITE_SIZE"]
    if not fetch or not write:
        raise SystemExit(f"no samples for {KERNEL}: {res}")
    fetch_kib = sum(fetch) / len(fetch)
    write_kib = sum(write) / len(write)
    algo = 3 * (1 << 26) * 4
    hbm = (2 * fetch_kib + write_kib) * 1024
    out = {"reduce_copy": {"kernel": KERNEL, "algorithmic_bytes_per_launch": algo,
                           "fetch_kib_raw": fetch_kib, "write_kib": write_kib,
                           "hbm_bytes_per_launch": int(hbm),
                           "read_bytes_corrected": int(2 * fetch_kib * 1024),
                           "write_bytes": int(write_kib * 1024),
                           "traffic_over_algorithmic": round(hbm / algo, 4),
                           "samples": [len(fetch), len(write)],
                           "method": "rocprofv3 --pmc, separate passes; FETCH_SIZE x2 (gfx950), KiB x1024"}}
    json.dump(out, open(os.path.join(OUT, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
