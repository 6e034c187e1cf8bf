"""CPU checks of the full-size workload test's machinery (tests/_workload.py)
and of the CPU-baseline leg (oracle/cpu_bench.c)."""
import numpy as np
import torch

from oracle import oracle as O
from oracle import vccl_sched as S
from tests import _workload as W


def test_owner_at_equals_full_map():
    """allreduce_owner_at (sampled windows of 1 GiB buckets) vs the full
    owner map, over random geometries incl. short last loops."""
    rng = np.random.default_rng(0)
    for _ in range(200):
        n = int(rng.choice([2, 3, 4, 8]))
        esz = int(rng.choice([1, 2, 4, 8]))
        nch = int(rng.choice([1, 2, 7, 14, 48, 56]))
        count = int(rng.integers(1, 2_000_000))
        slot = int(rng.choice([4096, 64 << 10, 256 << 10]))
        nt = int(rng.choice([256, 512]))
        w = S.cbd_schedule("ar", count, esz, n, nch, buff_size=slot * S.NCCL_STEPS, nthreads=nt)
        chan, owner = S.allreduce_owner(w, count, n)
        idx = rng.integers(0, count, 300)
        c2, o2 = S.allreduce_owner_at(w, count, n, idx)
        assert (c2 == chan[idx]).all() and (o2 == owner[idx]).all(), (n, esz, nch, count, slot, nt)


def test_hashed_inputs_numpy_equals_torch():
    """The worker generates inputs with torch on the GPU, the test regenerates
    windows with numpy: same integer arithmetic, same bits (torch CPU here,
    the identical ops run on the GPU)."""
    for dt, tdt, view in ((9, torch.bfloat16, torch.int16), (7, torch.float32, torch.int32)):
        for r in range(4):
            base = (1 << 31) - 3000 if r % 2 else 17
            t = torch.empty(6000, dtype=tdt)
            W.device_fill(t, dt, r, base=base, slice_elems=2500)
            got = t.view(view).numpy().view(np.uint16 if dt == 9 else np.uint32)
            exp = W.host_values(dt, np.arange(base, base + 6000), r)
            assert np.array_equal(got, exp.view(got.dtype)), (dt, r)
    x = W.host_values(7, np.arange(1 << 16), 0)
    assert len(np.unique(np.floor(np.log2(np.abs(x))))) == 8  # 8 binades: fold order shows


def test_window_expectation_is_the_ring_fold():
    """expected_ar_windows equals the full-buffer ring fold at the windows."""
    from tests import _ring
    count, n, nch, slot = 300_001, 4, 14, 4096
    win, work = W.ar_windows(count, 4, n, nch, slot, 512)
    ins = [W.host_values(7, np.arange(count), r) for r in range(n)]
    full = _ring.expected_allreduce(0, 7, ins, nch, slot)
    assert np.array_equal(W.expected_ar_windows(7, win, n, work).view(np.uint32), full[win].view(np.uint32))
    rc = 70_001
    win, work = W.rs_windows(rc, 2, n, nch, slot, 512)
    ins = [W.host_values(9, np.arange(rc * n), r) for r in range(n)]
    full = _ring.expected_reducescatter(0, 9, ins, nch, slot)
    for r in range(n):
        assert np.array_equal(W.expected_rs_windows(9, win, n, r, rc, work), full[r][win])


def test_cpu_bench_leg():
    """The CPU baseline's pinned-worker reduce-copy: correct, first-touched,
    and timing a bounded loop."""
    res = O.cpu_bench(1 << 20, [0, 0], 0.2, native=False)
    assert res["correct"] and res["iters"] >= 1 and res["GB/s"] > 0
