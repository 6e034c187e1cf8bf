"""The N > 1 bench line's `roofline` and `cpu_baseline`, on
the CPU: the xGMI ceiling comes from the ring set in use (not a hard-coded
link count), ranks sharing one device switch the bound to that device's HBM
(frac <= 1), and rank 0 of a stand-in gloo world adds a checked host-core
baseline of the per-rank bucket shape while the other rank waits."""
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from vccl_amd import nccl  # noqa: E402

L = bench.XGMI_LINK_GBS


@pytest.mark.parametrize("n,links", [(2, 1), (3, 2), (4, 3), (5, 4), (6, 4), (7, 6), (8, 7)])
def test_link_ceiling_follows_the_ring_set(n, links):
    # default channel counts: whole multiples of the ring count
    nch = {2: 16, 3: 32, 4: 48, 5: 64, 6: 64, 7: 60, 8: 63}[n]
    lp = bench.ring_link_peak(nccl.ring_orders(n), nch)
    assert lp["links"] == links
    assert lp["peak"] == pytest.approx(links * L)
    assert lp["links_used_per_rank"] == links


def test_link_ceiling_counts_uneven_channel_shares():
    # 4 ranks, 6 rings, 8 channels: rings 0 and 1 carry 2 channels each, so
    # their arcs are the worst loaded and the ceiling falls below 3 links
    orders = nccl.ring_orders(4)
    lp = bench.ring_link_peak(orders, 8)
    load = {}
    for c in range(8):
        ring = orders[c % len(orders)]
        for k, a in enumerate(ring):
            arc = (a, ring[(k + 1) % 4])
            load[arc] = load.get(arc, 0) + 1
    assert lp["peak"] == pytest.approx(L * 8 / max(load.values()))
    assert lp["peak"] < 3 * L


@pytest.mark.parametrize("n", [2, 4, 8])
def test_ring_hbm_bytes(n):
    S = 1 << 30
    # S->F, (n-2) S+F->F, S+F->F+O, (n-2) F->F+O, F->O in units of S/n
    reads = 1 + 2 * (n - 2) + 2 + (n - 2) + 1
    writes = 1 + (n - 2) + 2 + 2 * (n - 2) + 1
    assert bench.ring_ar_hbm_bytes(n, S) == (reads + writes) * S / n
    if n == 2:
        assert bench.ring_ar_hbm_bytes(n, S) == 4 * S


def test_shared_device_bound_is_hbm():
    # the round-5 N = 2 rehearsal: 1 GiB in 4.9 ms on one GPU read 2.86 of a
    # link; on the device's HBM it is 2 x 4 GiB / 4.9 ms
    S, t = 1 << 30, 4.9e-3
    busbw = S / t * 2 * 1 / 2 / 1e9
    r = bench.allreduce_roofline(busbw, t, S, 2, 2, "ring", nccl.ring_orders(2), 16)
    assert r["bound"] == "hbm" and r["peak"] == bench.HBM_PEAK_GBS
    assert r["achieved"] == pytest.approx(2 * 4 * S / t / 1e9, rel=1e-3)
    assert 0 < r["frac"] <= 1
    assert "measured_peer_copy" not in r and "links" not in r
    # 4 ranks on one device: 4 x 5 S per call
    r4 = bench.allreduce_roofline(busbw, t, S, 4, 4, "ring", nccl.ring_orders(4), 48)
    assert r4["achieved"] == pytest.approx(4 * 5 * S / t / 1e9, rel=1e-3)
    # a non-ring path on a shared device: no invented bytes
    rd = bench.allreduce_roofline(busbw, t, S, 4, 4, "direct", nccl.ring_orders(4), 48)
    assert rd["bound"] == "hbm" and rd["frac"] is None


def test_own_device_bound_is_xgmi():
    r = bench.allreduce_roofline(500.0, 1e-3, 1 << 30, 8, 1, "ring", nccl.ring_orders(8), 63, 70.0)
    assert r["bound"] == "xgmi" and r["links"] == 7
    assert r["peak"] == pytest.approx(7 * L)
    assert r["frac"] == pytest.approx(500.0 / (7 * L), abs=1e-4)
    assert r["frac_of_measured_copy"] == pytest.approx(500.0 / (7 * 70.0), abs=1e-4)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, visible, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    import bench as B
    from vccl_amd import nccl as N
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        S, t = 8 << 20, 2e-3  # stand-in timing of an 8 MiB bucket
        last = {"bytes": S, "us": t * 1e6, "busbw": S / t * 2 * (world - 1) / world / 1e9, "algo": "ring"}
        rpd, roof, cpu = B.line_roofline_and_baseline(dist, rank, world, last, visible, N.ring_orders(world),
                                                      16 * len(N.ring_orders(world)), None, cpu_seconds=0.3)
        q.put((rank, rpd, roof, cpu))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("visible", [1, 2])
def test_stand_in_ranks_line(visible):
    """Two gloo ranks (no GPU): on one visible device the bound is HBM, on
    two it is xGMI; rank 0 carries a checked cpu_baseline, rank 1 none."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, visible, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    res = {r: (rpd, roof, cpu) for r, rpd, roof, cpu in (q.get(timeout=5) for _ in range(world))}
    assert all(p.exitcode == 0 for p in procs)
    rpd, roof, cpu = res[0]
    assert rpd == (2 if visible == 1 else 1)
    if visible == 1:
        assert roof["bound"] == "hbm" and 0 < roof["frac"] <= 1
    else:
        assert roof["bound"] == "xgmi" and roof["links"] == 1
    assert cpu["value"] > 0 and cpu["unit"] == "GB/s" and cpu["kind"] == "port"
    assert cpu["cores"] >= 1 and "checked bit-exactly" in cpu["sample"]
    # configs 4 and 5 beside it (bf16 bucket on the baseline cores, f16 LL bucket on one core)
    oc = cpu["other_configs"]
    assert oc["config4_rs_ag_bf16"]["value"] > 0 and "bf16" in oc["config4_rs_ag_bf16"]["sample"]
    assert oc["config5_ll_f16"]["value"] > 0 and oc["config5_ll_f16"]["cores"] == 1
    assert res[1][2] is None  # only rank 0 measures the host


@pytest.mark.parametrize("dtype", [7, 6, 9])  # f32, f16, bf16
def test_cpu_rank_shape_checks_every_pass(dtype):
    from oracle import oracle as O
    for nsrc, ncopy in ((2, 0), (3, 3000), (8, 1 << 16)):
        r = O.cpu_bench_rank(5000, nsrc, ncopy, [0, 1], 0.05, dtype=dtype)
        assert r["correct"] and r["iters"] >= 1


def test_ring_trace_summary():
    """bench.ring_trace_summary on a hand-made timeline: one channel, two
    S+F->F+O slots (shape 0b1111) of 1 MiB at 100 MHz ticks."""
    import numpy as np
    dt = np.dtype([("t0", "<u8"), ("t1", "<u8"), ("t2", "<u8"), ("t3", "<u8"), ("t4", "<u8"),
                   ("shape", "<u4"), ("bytes", "<u4"), ("step", "<u8"), ("tc", "<u8")])
    tr = np.zeros((1, 4), dtype=dt)
    # slot 0: wait 1 us, release 0.5, copy 10 (issue 8 + drain 2), post 0.5; gap 1 us to slot 1
    tr[0, 0] = (1000, 1100, 1150, 2150, 2200, 0b1111, 1 << 20, 0, 1950)
    tr[0, 1] = (2300, 2300, 2350, 3350, 3400, 0b1111, 1 << 20, 1, 3150)
    s = bench.ring_trace_summary(tr)["S+F->F+O"]
    assert s["n"] == 2
    assert s["wait"] == pytest.approx(0.5) and s["release"] == pytest.approx(0.5)
    assert s["copy"] == pytest.approx(10.0) and s["issue"] == pytest.approx(8.0) and s["drain"] == pytest.approx(2.0)
    assert s["post"] == pytest.approx(0.5) and s["gap"] == pytest.approx(0.5)  # one gap of 1 us over 2 slots
    assert s["payload_GBs_in_copy"] == pytest.approx(round(2 * (1 << 20) / (20.0 * 1e3), 1))


def test_cpu_baseline_leaves_the_caller_unpinned():
    """The bench's calling thread is worker 0 of the host baseline: its own
    CPU affinity must come back afterwards (a pinned main thread made the next
    baseline on the N > 1 line see one CPU)."""
    before = os.sched_getaffinity(0)
    bench.cpu_baseline_allreduce(1 << 20, 2, 0.1)
    assert os.sched_getaffinity(0) == before


def test_handoff_exit_rule():
    """DESIGN §9's exit rule on the line's ring_handoff rows: it decides only
    at 8 ranks, one per GPU, 1 GiB; >= 3 % keeps the per-wave hand-off."""
    wg = {"bytes": 1 << 30, "us": 1030.0}
    r = bench.handoff_exit_rule(wg, {"bytes": 1 << 30, "us": 1000.0}, 8, 1)
    assert r["applies"] and r["per_wave_gain"] == 0.03 and "default" in r["verdict_if_checks_green"]
    r = bench.handoff_exit_rule(wg, {"bytes": 1 << 30, "us": 1010.0}, 8, 1)
    assert r["applies"] and "deleted" in r["verdict_if_checks_green"]
    for world, rpd, S in ((8, 8, 1 << 30), (4, 1, 1 << 30), (8, 1, 64 << 20)):
        r = bench.handoff_exit_rule({"bytes": S, "us": 2.0}, {"bytes": S, "us": 1.0}, world, rpd)
        assert not r["applies"] and r["verdict_if_checks_green"] is None


def test_channel_knee():
    rows = [{"n_channels": c, "busbw": b, "correct": True}
            for c, b in ((14, 100.0), (28, 180.0), (63, 300.0), (126, 310.0))]
    rows.append({"n_channels": 252, "busbw": 400.0, "correct": False})  # unchecked rows never count
    k = bench.channel_knee(rows, 63, 1)
    assert k["best_channels"] == 126 and k["knee_channels"] == 63 and k["default_over_best"] == 0.968
    assert k["one_rank_per_gpu"]
    assert bench.channel_knee([], 63, 1)["knee_channels"] is None
    assert not bench.channel_knee(rows, 16, 8)["one_rank_per_gpu"]
