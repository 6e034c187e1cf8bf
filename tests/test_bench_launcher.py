"""bench.py's own rank launcher (VERDICT r4 #1a), on the CPU.

`python bench.py --gpus N` without WORLD_SIZE must start N rank processes
(children, one per GPU, before the parent touches the GPU) and report n_gpus
= N; --gpus and a WORLD_SIZE that disagree must fail loudly instead of
producing the 1-GPU line."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_gpus_two_builds_two_ranks_without_world_size():
    plan = bench.rank_launch_plan(["--gpus", "2", "--steps", "3"], {"PATH": "/bin"}, port=29123)
    assert len(plan) == 2
    for r, (cmd, env) in enumerate(plan):
        assert cmd[-4:] == ["--gpus", "2", "--steps", "3"]
        assert cmd[0] == sys.executable and cmd[2].endswith("bench.py")
        assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"]) == (str(r), str(r), "2")
        assert (env["MASTER_ADDR"], env["MASTER_PORT"]) == ("127.0.0.1", "29123")
        assert env["PATH"] == "/bin"


@pytest.mark.parametrize("argv,env,want", [
    ([], {}, (1, False)),                                 # default: the N = 1 line
    (["--gpus", "1"], {}, (1, False)),
    (["--gpus=4"], {}, (4, True)),                        # spawn 4 ranks
    (["--gpus", "8"], {"WORLD_SIZE": "8"}, (8, False)),   # torch.distributed.run already did
    ([], {"WORLD_SIZE": "2"}, (2, False)),
])
def test_world_check(argv, env, want):
    assert bench.world_check(argv, env) == want
    if not want[1]:
        assert bench.rank_launch_plan(argv, env) == []


def test_gpus_and_world_size_disagree():
    with pytest.raises(SystemExit) as e:
        bench.world_check(["--gpus", "8"], {"WORLD_SIZE": "2"})
    assert "--gpus 8" in str(e.value) and "WORLD_SIZE=2" in str(e.value)


def test_spawned_ranks_relay_rank0_line_and_exit_codes():
    """_spawn_ranks with stand-in rank programs: rank 0's JSON line is
    printed, a failing rank's exit code is returned."""
    prog = ("import json, os, sys; r = int(os.environ['RANK']); "
            "print(json.dumps({'rank': r, 'n': int(os.environ['WORLD_SIZE'])}) if r == 0 else 'x'); "
            "sys.exit(int(os.environ.get('FAIL_RANK', '-1')) == r and 5 or 0)")
    code = ("import subprocess, sys\nsys.path.insert(0, %r)\nimport bench\n"
            "plan = [([sys.executable, '-c', %r], e) for _, e in "
            "bench.rank_launch_plan(['--gpus', '3'], dict(__import__('os').environ))]\n"
            "sys.exit(bench._spawn_ranks(plan, poll_s=0.05))\n") % (ROOT, prog)
    for fail, want_rc in ((None, 0), ("2", 5)):
        env = dict(os.environ)
        env.pop("WORLD_SIZE", None)
        if fail:
            env["FAIL_RANK"] = fail
        p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        assert p.returncode == want_rc, p.stderr
        assert p.stdout.strip() == '{"rank": 0, "n": 3}', p.stdout
