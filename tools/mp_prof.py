#!/usr/bin/env python3
"""Kernel trace of the N > 1 bench line: N ranks of bench.py, each started
directly under `rocprofv3 --kernel-trace --stats` (the program right after
`--`; this launcher never touches the GPU), rendezvous on 127.0.0.1.

    python tools/mp_prof.py N OUTDIR [bench.py args...]

MP_PROF_SCRIPT=<path> runs that script instead of bench.py (e.g.
tools/ll_latency.py); MP_PROF_FLAGS adds rocprofv3 tracing flags (e.g.
"--hip-runtime-trace" for the host submit times; never --pmc here).
Per-rank outputs under OUTDIR/rank<r>/; rank 0's JSON line goes to
OUTDIR/bench.json.  Exits with the worst rank's status."""
import os
import subprocess
import sys


def main():
    n, out = int(sys.argv[1]), os.path.abspath(sys.argv[2])
    extra = sys.argv[3:]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(out, exist_ok=True)
    procs = []
    for r in range(n):
        env = {**os.environ, "RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
               "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29561"}
        script = os.environ.get("MP_PROF_SCRIPT")
        prog = ([os.path.join(root, script)] if script else
                [os.path.join(root, "bench.py"), "--gpus", str(n)])
        flags = os.environ.get("MP_PROF_FLAGS", "").split()
        assert not any("pmc" in f for f in flags), "counters need passes of their own"
        cmd = ["rocprofv3", "--kernel-trace", "--stats", *flags, "--output-format", "csv", "-d",
               os.path.join(out, f"rank{r}"), "-o", "run", "--", sys.executable, *prog, *extra]
        stdout = open(os.path.join(out, "bench.json" if r == 0 else f"rank{r}.out"), "w")
        stderr = open(os.path.join(out, f"rank{r}.err"), "w")
        procs.append(subprocess.Popen(cmd, env=env, stdout=stdout, stderr=stderr, cwd="/tmp"))
    rc = 0
    for p in procs:
        try:
            rc = max(rc, p.wait(timeout=540))
        except subprocess.TimeoutExpired:
            p.kill()
            rc = 124
    sys.exit(rc)


if __name__ == "__main__":
    main()
