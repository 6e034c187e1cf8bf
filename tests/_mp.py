"""Rank placement for the multi-process GPU tests and bench.py.

One rank per GPU wherever the box has enough of them: rank r runs on device
r % device_count.  Only when a job has more ranks than the box has GPUs (the
one-GPU rehearsals) do ranks share a device, and only then does the worker
set VCCL_ALLOW_SHARED_DEVICE (the library refuses two ranks on one GPU
otherwise, as the reference does, init.cc:732-735).  The same code runs the
suite on a 1-GPU box (every rank on device 0) and on an 8-GPU node (one rank
per device, peer FIFOs over xGMI).

torch.cuda.device_count() does not initialise the GPU on this image, so a
parent may call these before it spawns its rank processes.
"""
import os


def device_count():
    import torch
    return max(1, torch.cuda.device_count())


def ranks_per_device(nranks, ndev=None):
    """Largest number of ranks that land on one device (round-robin)."""
    ndev = ndev or device_count()
    return (nranks + ndev - 1) // ndev


def shares_device(nranks, ndev=None):
    return ranks_per_device(nranks, ndev) > 1


def rank_device(rank, nranks, env=os.environ):
    """Device of `rank` in a job of `nranks`; sets VCCL_ALLOW_SHARED_DEVICE
    in `env` exactly when the ranks outnumber the devices."""
    ndev = device_count()
    if shares_device(nranks, ndev):
        env["VCCL_ALLOW_SHARED_DEVICE"] = "1"
    else:
        env.pop("VCCL_ALLOW_SHARED_DEVICE", None)
    return rank % ndev


def bind(rank, nranks):
    """torch.cuda.set_device(rank_device(...)); returns the device."""
    import torch
    d = rank_device(rank, nranks)
    torch.cuda.set_device(d)
    return d


def worker_env(env):
    """The environment a test hands its rank processes: the workers decide
    about device sharing themselves (rank_device), so the parent's own
    VCCL_ALLOW_SHARED_DEVICE does not leak into a one-rank-per-GPU run."""
    env = dict(env)
    env.pop("VCCL_ALLOW_SHARED_DEVICE", None)
    return env


def shared_channel_cap(nranks, default, cus):
    """The ring channels each rank gets at library defaults: the default,
    capped at 7/8 of a shared GPU's CUs over the ranks sharing it
    (host/init.cc co-residency cap) — no cap at one rank per GPU."""
    k = ranks_per_device(nranks)
    return default if k <= 1 else min(default, max(1, cus * 7 // 8 // k))
