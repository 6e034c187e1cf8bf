#!/usr/bin/env python3
"""Kernel trace of the N > 1 bench line: N ranks of bench.py, each started
directly under `rocprofv3 --kernel-trace --stats` (the program right after
`--`; this launcher never touches the GPU), rendezvous on 127.0.0.1.

    python tools/mp_prof.py N OUTDIR [bench.py args...]

Per-rank outputs under OUTDIR/rank<r>/; rank 0's bench JSON line goes to
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
        cmd = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d",
               os.path.join(out, f"rank{r}"), "-o", "run", "--", sys.executable,
               os.path.join(root, "bench.py"), "--gpus", str(n), *extra]
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
