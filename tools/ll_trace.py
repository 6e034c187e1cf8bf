#!/usr/bin/env python3
"""Per-call timeline of the LL all-reduce across ranks, from
the per-rank rocprofv3 traces tools/mp_prof.py writes
(MP_PROF_SCRIPT=tools/ll_latency.py, MP_PROF_FLAGS=--hip-runtime-trace):

    python tools/ll_trace.py OUTDIR [> summary.json]

For the i-th LL kernel of every rank (each call launches exactly one per
rank): start skew across ranks, each rank's kernel duration, the gap since
that rank's previous kernel ended, and — from the HIP API trace, joined on
the correlation id — the host submit time, so the late rank's start can be
split into "host had not submitted yet" and "submitted, GPU had not started
it".  The sequence is cut into runs of fast and slow calls (call period
below / above FAST_US) and each run summarised by medians.
Measurement tool, not product code."""
import csv
import glob
import json
import os
import statistics
import sys

FAST_US = float(os.environ.get("FAST_US", 15))


def _rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def load_rank(d):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    api = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
    ks = [r for f in kt for r in _rows(f) if "k_ll" in r["Kernel_Name"]]
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    sub = {}
    for f in api:
        for r in _rows(f):
            if "Launch" in r["Function"]:
                sub[r["Correlation_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
    out = []
    for r in ks:
        s = sub.get(r["Correlation_Id"])
        out.append({"start": int(r["Start_Timestamp"]), "end": int(r["End_Timestamp"]),
                    "submit": s[1] if s else None, "api": s[2] if s else None})
    return out


def med(v):
    v = [x for x in v if x is not None]
    return round(statistics.median(v), 2) if v else None


def main():
    outdir = sys.argv[1]
    ranks = sorted(glob.glob(os.path.join(outdir, "rank*")))
    ranks = [d for d in ranks if os.path.isdir(d)]
    seqs = [load_rank(d) for d in ranks]
    n = min(len(s) for s in seqs)
    calls = []
    for i in range(n):
        st = [s[i]["start"] for s in seqs]
        en = [s[i]["end"] for s in seqs]
        late = max(range(len(seqs)), key=lambda r: st[r])
        prev_end = seqs[late][i - 1]["end"] if i else None
        sub = seqs[late][i]["submit"]
        ready = max(x for x in (prev_end, sub) if x is not None) if (prev_end or sub) else None
        calls.append({
            "i": i,
            "period_us": (max(s[i]["start"] for s in seqs) - max(s[i - 1]["start"] for s in seqs)) / 1e3 if i else None,
            "skew_us": (max(st) - min(st)) / 1e3,
            "dur_max_us": (max(en) - min(st)) / 1e3,
            "dur_late_us": (en[late] - st[late]) / 1e3,
            "late_rank": late,
            # the late rank's kernel started this long after it could have:
            # after its host submit and after its previous kernel ended
            "late_dispatch_delay_us": (st[late] - ready) / 1e3 if ready else None,
            "late_submit_lag_us": (sub - min(st)) / 1e3 if sub else None,
            "api": seqs[late][i]["api"],
        })
    runs, cur = [], None
    for c in calls[1:]:
        fast = c["period_us"] is not None and c["period_us"] < FAST_US
        if cur is None or cur["fast"] != fast:
            cur = {"fast": fast, "from": c["i"], "calls": []}
            runs.append(cur)
        cur["calls"].append(c)
    summary = []
    for r in runs:
        cs = r["calls"]
        if len(cs) < 5:
            continue
        summary.append({"fast": r["fast"], "from": r["from"], "n": len(cs),
                        "period_us": med([c["period_us"] for c in cs]),
                        "skew_us": med([c["skew_us"] for c in cs]),
                        "dur_max_us": med([c["dur_max_us"] for c in cs]),
                        "dur_late_us": med([c["dur_late_us"] for c in cs]),
                        "late_dispatch_delay_us": med([c["late_dispatch_delay_us"] for c in cs]),
                        "late_submit_lag_us": med([c["late_submit_lag_us"] for c in cs]),
                        "api": cs[len(cs) // 2]["api"]})
    print(json.dumps({"ranks": len(seqs), "ll_kernels_per_rank": [len(s) for s in seqs], "runs": summary},
                     indent=1))


if __name__ == "__main__":
    main()
