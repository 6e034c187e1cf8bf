"""Rank placement of the multi-process tests and bench.py (tests/_mp.py), on
the CPU with the device count stubbed: one rank per GPU where the box has
enough of them, round-robin sharing (and VCCL_ALLOW_SHARED_DEVICE) only
beyond that, and the channel count each rank then gets at library defaults
(VERDICT r4 #1b)."""
import pytest

from tests import _mp


@pytest.mark.parametrize("ndev,n,devs,shared,per_dev", [
    (1, 2, [0, 0], True, 2),                      # the one-GPU rehearsal
    (8, 8, list(range(8)), False, 1),              # one rank per GPU
    (8, 2, [0, 1], False, 1),
    (4, 8, [0, 1, 2, 3, 0, 1, 2, 3], True, 2),
    (2, 3, [0, 1, 0], True, 2),
])
def test_rank_device(monkeypatch, ndev, n, devs, shared, per_dev):
    monkeypatch.setattr(_mp, "device_count", lambda: ndev)
    for r in range(n):
        env = {"VCCL_ALLOW_SHARED_DEVICE": "1"}  # a parent's setting must not leak through
        assert _mp.rank_device(r, n, env) == devs[r]
        assert ("VCCL_ALLOW_SHARED_DEVICE" in env) == shared
    assert _mp.shares_device(n, ndev) == shared and _mp.ranks_per_device(n, ndev) == per_dev


def test_shared_channel_cap(monkeypatch):
    # host/init.cc: ranks sharing a GPU get 7/8 of its CUs / sharing ranks;
    # one rank per GPU keeps the link-bound default
    monkeypatch.setattr(_mp, "device_count", lambda: 8)
    assert _mp.shared_channel_cap(8, 63, 256) == 63
    monkeypatch.setattr(_mp, "device_count", lambda: 1)
    assert _mp.shared_channel_cap(8, 63, 256) == 28
    assert _mp.shared_channel_cap(2, 16, 256) == 16
    monkeypatch.setattr(_mp, "device_count", lambda: 2)
    assert _mp.shared_channel_cap(8, 63, 256) == 56


def test_worker_env_drops_the_parents_sharing_flag():
    env = _mp.worker_env({"VCCL_ALLOW_SHARED_DEVICE": "1", "X": "y"})
    assert env == {"X": "y"}
