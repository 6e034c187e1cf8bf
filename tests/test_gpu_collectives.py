"""Ring all-reduce / reduce-scatter / all-gather parity on MI355X.

The box has one GPU, so the multi-rank protocol is exercised with several
ranks sharing device 0: (a) one process driving n comms from
ncclCommInitAll([0]*n) inside ncclGroupStart/End, one stream per rank;
(b) 8 (and 2) separate processes joined through ncclGetUniqueId /
ncclCommInitRank, FIFOs mapped with hipIpcOpenMemHandle.  Expected outputs
come from the CPU oracle's ring fold over OUR channel partition
(tests/_ring.py), so every type/op is checked bit-exactly (min/max: +0 == -0).
Spins are bounded (VCCL_SPIN_TIMEOUT_S) so a protocol bug fails the test
instead of hanging the GPU.
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch

from tests import _mp
from tests import _ring
from tests import ring_cases as RC
from tests._util import assert_bitexact, assert_fold_tolerance, exact_f64

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from vccl_amd import nccl  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("VCCL_SPIN_TIMEOUT_S", "20")
# Several ranks share ONE GPU here, so every rank's channel workgroups must be
# co-resident: the tests pin a geometry that fits (library defaults are sized
# for one rank per GPU and are exercised by the 2-process default case).
TEST_GEOM = {"VCCL_NCHANNELS": "14", "VCCL_NTHREADS": "512", "VCCL_SLOT_BYTES": str(256 << 10),
             "VCCL_ALLOW_SHARED_DEVICE": "1", "VCCL_LL_THRESHOLD": str(1 << 20),
             "VCCL_LL_MAX_BLOCKS": "32", "VCCL_DIRECT_THRESHOLD": str(4 << 20),
             "VCCL_DIRECT_MAX_BLOCKS": "16", "VCCL_DIRECT_CHUNK_BYTES": str(1 << 20),
             "VCCL_DIRECT_RSAG_THRESHOLD": str(64 << 20),
             # the SIMPLE ring's per-wave hand-off (VCCL_RING_WAVE, the PART 4
             # kernels: f32 / f16 / bf16 sums, all-gather, broadcast) for every
             # slot, not only from 512 KiB up; "ring_only" below and the
             # library-default rows run the workgroup hand-off (the default)
             "VCCL_RING_WAVE": "1", "VCCL_RING_WAVE_MIN": "0"}
# the group tests' direct thresholds: a group's aggregate takes the path of
# its summed size, so the ZeRO loop's 128 MiB of reduce-scatters and 16 MiB
# of all-reduces need raised thresholds to stay on the direct path
GROUP_DIRECT = {"VCCL_DIRECT_THRESHOLD": str(32 << 20), "VCCL_DIRECT_RSAG_THRESHOLD": str(256 << 20)}
LL_DEFAULT = 1 << 20
DIRECT_TEST = 4 << 20
DIRECT_CHUNK_TEST = 1 << 20  # buckets of 1-4 MiB stream through the inbox in chunks


def _check(ci, n, outs, nch, slot, ll_max, direct_max, chunk=DIRECT_CHUNK_TEST, nthreads=512, proto=2,
           chain=None, ll_rs_max=None):
    """Bit-exact against the path's own fold order (the ring's IS VCCL's
    schedule on our rings and channels); for fp sum / prod additionally
    within the §8c tolerance of the exact value and of VCCL's result on its
    reference geometry (RC.vccl_reference)."""
    name, coll, op, dt, count = RC.CASES[ci]
    exp = RC.expected(ci, n, nch, slot, ll_max, direct_max, chunk, nthreads, proto, chain, ll_rs_max)
    for r in range(n):
        assert_bitexact(dt, outs[r], exp[r], minmax=op in (2, 3), what=f"{name} n={n} rank {r}")
    vref = RC.vccl_reference(ci, n)
    if vref is not None:
        ins = RC.inputs(ci, n)
        cnt = outs[0].size
        for r in range(n):
            blk = [x[r * cnt:(r + 1) * cnt] for x in ins] if coll == "rs" else ins
            assert_fold_tolerance(dt, op, outs[r], exact_f64(dt, op, blk), blk, exp_is_exact=True,
                                  what=f"{name} n={n} rank {r} vs exact")
            assert_fold_tolerance(dt, op, outs[r], vref[r], blk,
                                  what=f"{name} n={n} rank {r} vs VCCL ring schedule")


def test_duplicate_device_rejected():
    # reference init.cc:1782-1786 / :732-735: two ranks on one GPU
    with pytest.raises(nccl.VcclError) as e:
        nccl.Comm.init_all([0, 0])
    assert e.value.code == nccl.ncclInvalidUsage


def test_algorithm_choice(monkeypatch):
    """Library defaults at 2 ranks: AR LL up to 64 KiB, the ring above (the
    direct path defaults up to 64 MiB from 4 ranks); RS / AG LL / ring by
    bucket size; NCCL_ALGO / NCCL_PROTO force one (vcclCommCollAlgo), Direct
    for any size."""
    monkeypatch.setenv("VCCL_ALLOW_SHARED_DEVICE", "1")
    for k in ("NCCL_ALGO", "NCCL_PROTO", "VCCL_LL_THRESHOLD", "VCCL_DIRECT_THRESHOLD",
              "VCCL_LL_RSAG_THRESHOLD", "VCCL_DIRECT_RSAG_THRESHOLD"):
        monkeypatch.delenv(k, raising=False)
    # RS / AG at 2 ranks: one-hop LL while the bucket (n blocks) is <= n x
    # the AR LL threshold, the ring above (the one-hop direct path needs
    # n >= 4 by default: it saves n-2 hops).
    cases = {None: {(0, 16 << 10): "ll", (0, 17 << 10): "ring", (0, 1 << 24): "ring",
                    (0, (1 << 24) + 4): "ring", (0, 1 << 28): "ring",
                    (1, 1 << 10): "ll", (2, 1 << 10): "ll", (1, 16 << 10): "ll",
                    (1, 17 << 10): "ring", (2, 1 << 20): "ring", (2, 1 << 26): "ring"},
             # NCCL_ALGO=Ring: no LL all-reduce (VCCL's LL all-reduce is the
             # tree's here), ring LL for small RS / AG
             "Ring": {(0, 1 << 10): "ring", (0, 1 << 20): "ring", (1, 1 << 10): "ll",
                      (2, 1 << 20): "ring"},
             "Tree": {(0, 1 << 10): "ll", (0, 1 << 20): "ring", (1, 1 << 10): "ll",
                      (2, 1 << 26): "ring"},
             "Direct": {(0, 1 << 10): "direct", (0, 1 << 28): "direct", (1, 1 << 10): "direct",
                        (2, 1 << 10): "direct", (2, 1 << 26): "direct"}}
    for algo, expect in cases.items():
        if algo is None:
            monkeypatch.delenv("NCCL_ALGO", raising=False)
        else:
            monkeypatch.setenv("NCCL_ALGO", algo)
        comms = nccl.Comm.init_all([0, 0])
        try:
            for (coll, count), want in expect.items():
                assert comms[0].coll_algo(coll, count, 7) == want, (algo, coll, count)
        finally:
            for c in comms:
                c.destroy()


# One process drives n ranks on the single GPU: the ranks' kernels are only
# co-resident if their streams land on distinct hardware queues (HIP: 4 per
# process, assigned round-robin over every stream the process has created),
# so the single-process case is kept at n = 2; n >= 3 run as processes below.
# "all": ncclCommInitAll over every GPU of a multi-GPU box (the reference's
# single-process harness shape, peers mapped by peer access instead of IPC),
# bit-exact against the oracle like the shared-GPU case.
@pytest.mark.parametrize("n,placement", [(2, "shared"), (0, "all")])
def test_single_process_ranks(n, placement, monkeypatch):
    ndev = torch.cuda.device_count()
    if placement == "all":
        if ndev < 2:
            pytest.skip(f"ncclCommInitAll over every GPU needs >= 2 GPUs; this box has {ndev}")
        n = min(ndev, 8)
    devs = [0] * n if placement == "shared" else list(range(n))
    for k, v in TEST_GEOM.items():
        monkeypatch.setenv(k, v)
    if placement == "all":
        monkeypatch.delenv("VCCL_ALLOW_SHARED_DEVICE", raising=False)
    nch, slot = int(TEST_GEOM["VCCL_NCHANNELS"]), int(TEST_GEOM["VCCL_SLOT_BYTES"])
    comms = nccl.Comm.init_all(devs)

    def on(r):  # tensors of rank r live on its device
        return torch.device("cuda", devs[r])
    try:
        assert [c.rank for c in comms] == list(range(n)) and comms[0].count == n
        streams = [torch.cuda.Stream(device=on(r)) for r in range(n)]
        for ci, (name, coll, op, dt, count) in enumerate(RC.CASES):
            xs = [RC.gen_input(ci, r, n) for r in range(n)]
            xb = [torch.from_numpy(x.view(np.uint8).copy()).to(on(r)) for r, x in enumerate(xs)]
            nout = RC.out_count(ci, n)
            yb = [torch.empty(nout * xs[0].dtype.itemsize, dtype=torch.uint8, device=on(r))
                  for r in range(n)]
            keep = []
            if coll == "ar_mis":  # the same bytes at (send, recv) offsets off 16-byte alignment
                so, ro = RC.mis_offsets(dt)
                for r in range(n):
                    xm = torch.zeros(xb[r].numel() + 16, dtype=torch.uint8, device=on(r))
                    xm[so:so + xb[r].numel()] = xb[r]
                    keep.append((xm, torch.zeros(yb[r].numel() + 16, dtype=torch.uint8, device=on(r))))
            for r in range(n):
                torch.cuda.synchronize(on(r))
            nccl.group_start()
            for r, c in enumerate(comms):
                sp = streams[r].cuda_stream
                if coll == "ar":
                    c.all_reduce(xb[r].data_ptr(), yb[r].data_ptr(), count, dt, op, sp)
                elif coll == "ar_inplace":
                    c.all_reduce(xb[r].data_ptr(), xb[r].data_ptr(), count, dt, op, sp)
                elif coll == "ar_mis":
                    xm, ym = keep[r]
                    c.all_reduce(xm.data_ptr() + so, ym.data_ptr() + ro, count, dt, op, sp)
                    yb[r] = ym[ro:ro + yb[r].numel()]
                elif coll == "rs":
                    c.reduce_scatter(xb[r].data_ptr(), yb[r].data_ptr(), count, dt, op, sp)
                else:
                    c.all_gather(xb[r].data_ptr(), yb[r].data_ptr(), count, dt, sp)
            nccl.group_end()
            for r in range(n):
                torch.cuda.synchronize(on(r))
            for c in comms:
                assert c.async_error() == 0, f"{name}: spin timeout (protocol hang)"
            outs = [(xb[r] if coll == "ar_inplace" else yb[r]).cpu().numpy().view(xs[0].dtype)
                    for r in range(n)]
            _check(ci, n, outs, nch, slot, LL_DEFAULT, DIRECT_TEST)
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("n,geom", [(2, "default"), (3, "test"), (4, "test"), (6, "test"), (8, "test"),
                                    (2, "ring_only"), (4, "ring_only"), (7, "ring_only"),
                                    (8, "ring_only"), (4, "direct_only"), (8, "default8"), (2, "net"),
                                    (3, "net"), (2, "ll128"), (4, "ll128"), (8, "ll128"),
                                    (4, "chain"), (8, "chain"), (2, "net_ll128"), (4, "test_fences")])
def test_multi_process_ranks(n, geom):
    _ring_ranks(n, geom)


# the same parity run with ONE RANK PER GPU (peer FIFOs over
# xGMI, IPC-mapped across processes) at library defaults — fences off (the
# default) and on, and every call on the LL128 ring — collected the first time
# the suite runs on a box with more than one GPU.  Each rank process binds
# device rank % device_count (tests/_mp.py).
def _multi_gpu_ns():
    ndev = torch.cuda.device_count()
    return sorted({2, min(ndev, 8)}) if ndev >= 2 else [2]


@pytest.mark.parametrize("geom", ["xgmi", "xgmi_fences", "xgmi_ll128", "xgmi_wave"])
@pytest.mark.parametrize("n", _multi_gpu_ns())
def test_one_rank_per_gpu(n, geom):
    ndev = torch.cuda.device_count()
    if ndev < n:
        pytest.skip(f"one rank per GPU needs {n} GPUs; this box has {ndev} "
                    "(the shared-GPU rehearsals above cover the protocol)")
    _ring_ranks(n, geom)


def _ring_ranks(n, geom):
    uid = nccl.get_unique_id()  # root thread lives in this process
    hexid = nccl.unique_id_to_bytes(uid).hex()
    env = dict(os.environ)
    env.setdefault("VCCL_SPIN_TIMEOUT_S", "20")
    ll_max, direct_max, chunk = LL_DEFAULT, DIRECT_TEST, DIRECT_CHUNK_TEST
    nthreads, proto, chain, ll_rs_max = 512, 2, None, None
    if geom == "chain":
        # VERDICT r3 missing #2: the LL all-reduce folds along a chain other
        # than the identity (VCCL's tree chain follows its topology order,
        # graph/connect.cc:64-65), pinned with VCCL_LL_CHAIN
        env.update(TEST_GEOM)
        chain = {4: [2, 0, 3, 1], 8: [5, 2, 7, 0, 3, 6, 1, 4]}[n]
        env["VCCL_LL_CHAIN"] = ",".join(map(str, chain))
        nch, slot = int(TEST_GEOM["VCCL_NCHANNELS"]), int(TEST_GEOM["VCCL_SLOT_BYTES"])
    elif geom == "ll128":
        # NCCL_PROTO=LL128: every collective on the LL128 ring (ring.hpp
        # prim_ll128), on VCCL's LL128 partition and chunking
        env.update(TEST_GEOM)
        env["NCCL_PROTO"] = "LL128"
        nch, slot = int(TEST_GEOM["VCCL_NCHANNELS"]), int(TEST_GEOM["VCCL_SLOT_BYTES"])
        ll_max = direct_max = 0
        proto = 1
    elif geom in ("test", "ring_only", "direct_only", "test_fences"):
        env.update(TEST_GEOM)
        if geom == "test_fences":  # system-scope fences on every ring slot and direct flag (VCCL_FENCES)
            env["VCCL_FENCES"] = "1"
        nch, slot = int(TEST_GEOM["VCCL_NCHANNELS"]), int(TEST_GEOM["VCCL_SLOT_BYTES"])
        if geom == "ring_only":  # NCCL_ALGO=Ring: the ring for every all-reduce,
            env["NCCL_ALGO"] = "Ring"  # ring LL (one-hop) for small RS / AG
            env["VCCL_RING_WAVE"] = "0"  # the workgroup hand-off for every slot
            ll_max = direct_max = 0
            ll_rs_max = LL_DEFAULT
        if geom == "direct_only":  # every collective takes the direct path, any size
            env["NCCL_ALGO"] = "Direct"
            ll_max, direct_max = 0, 1 << 62
    elif geom in ("net", "net_ll128"):
        # every ring connection through the net proxy (host-pinned staging +
        # TCP, proxy.cc), as between nodes; LL / direct need the xGMI mesh,
        # so every all-reduce takes the ring, on NET_NCHANNELS channels
        env.update(TEST_GEOM)
        env.update(VCCL_NET_FORCE="1", VCCL_NET_NCHANNELS="3", VCCL_SLOT_BYTES=str(64 << 10))
        nch, slot = 3, 64 << 10
        ll_max = direct_max = 0
        if geom == "net_ll128":
            # LL128 FIFOs requested (VCCL_LL128_ALLOC) and the LL128
            # ring forced per call (vcclCommSetAlgo) on a comm with net peers —
            # no LL128 slot is mapped there, so every call must take the
            # SIMPLE ring, not a ring of null LL128 slots
            env.update(VCCL_LL128_ALLOC="1", VCCL_TEST_SET_ALGO="ll128")
    elif geom.startswith("xgmi"):
        # library defaults, one rank per device (nothing shared, no cap)
        for k in TEST_GEOM:
            env.pop(k, None)
        nch, slot = _ring.n_channels(n), 512 << 10
        ll_max = (64 << 10) if n <= 2 else (128 << 10)
        direct_max, chunk = (8 << 20) if n >= 4 else 0, 16 << 20
        if geom == "xgmi_fences":  # system-scope acquire / release around every slot
            env["VCCL_FENCES"] = "1"
        if geom == "xgmi_wave":  # the per-wave ring hand-off, where remote stores acknowledge slowly
            env.update(VCCL_RING_WAVE="1", VCCL_RING_WAVE_MIN="0")
        if geom == "xgmi_ll128":  # every collective on the LL128 ring
            env["NCCL_PROTO"] = "LL128"
            ll_max = direct_max = 0
            proto = 1
    elif geom == "default8":
        # library defaults except the LL grid (8 ranks share the one GPU)
        for k in TEST_GEOM:
            env.pop(k, None)
        env.update(VCCL_ALLOW_SHARED_DEVICE="1", VCCL_LL_MAX_BLOCKS="32",
                   VCCL_DIRECT_MAX_BLOCKS="16", VCCL_NTHREADS="256", VCCL_CHANNELS_PER_RING="2")
        nch, slot = _ring.n_channels(n, per_ring=2), 512 << 10
        ll_max, direct_max, chunk = 128 << 10, 8 << 20, 16 << 20
        nthreads = 256  # NCCL_NTHREADS steers VCCL's channel tuning too
    else:  # library defaults (2 ranks x 32 channels x 1024 threads fit on one GPU)
        for k in TEST_GEOM:
            env.pop(k, None)
        env["VCCL_ALLOW_SHARED_DEVICE"] = "1"
        nch, slot = _ring.n_channels(n), 512 << 10
        ll_max = (64 << 10) if n <= 2 else (128 << 10)
        direct_max, chunk = (8 << 20) if n >= 4 else 0, 16 << 20
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_ring_worker.py"),
                                   str(r), str(n), "0", hexid, d], env=_mp.worker_env(env),
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(n)]
        logs = []
        for p in procs:
            try:
                out, _ = p.communicate(timeout=420)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            logs.append(out.decode(errors="replace")[-2000:])
        codes = [p.returncode for p in procs]
        assert codes == [0] * n, f"worker exit codes {codes}\n" + "\n".join(logs)
        res = [np.load(os.path.join(d, f"rank{r}.npz")) for r in range(n)]
        for ci, case in enumerate(RC.CASES):
            _check(ci, n, [res[r][case[0]] for r in range(n)], nch, slot, ll_max, direct_max, chunk,
                   nthreads, proto, chain, ll_rs_max)
        assert [str(a) for a in res[0]["group_algos"]] == [str(a) for a in res[0]["lib_group_algos"]]
        _check_group(n, [{k: res[r][k] for k in res[r].files} for r in range(n)], nch, slot,
                     [str(a) for a in res[0]["group_algos"]], nthreads, chain)
        # every geometry fuses the group's runs (LL, direct or ring batches)
        fused = int(res[0]["launch_stats"][1])
        assert fused > 0, f"fused group launches: {fused}"
        for r in range(n):
            sent, recvd, conns = (int(v) for v in res[r]["net_stats"])
            if geom.startswith("net"):  # one send and one receive connection per channel
                assert conns == 2 * nch and sent > 0 and recvd > 0, (r, sent, recvd, conns)
            else:
                assert conns == 0 and sent == 0, (r, sent, conns)
        # VCCL_RING_WAVE=1 rows ran the per-wave ring kernels (their f16 / f32 /
        # bf16 sum ring calls and all-gathers), the others never did
        waves = [int(res[r]["wave_launches"]) for r in range(n)]
        if env.get("VCCL_RING_WAVE") == "1" and geom in ("test", "chain", "net", "xgmi_wave"):
            assert min(waves) > 0, waves
        elif env.get("VCCL_RING_WAVE", "0") == "0":
            assert max(waves) == 0, waves


@pytest.mark.parametrize("n", [2, 4])
def test_ring_handoff_switch(n):
    """vcclCommSetRingWave between calls of one comm (tests/mp_handoff_worker.py):
    the SIMPLE ring's workgroup and per-wave hand-offs share FIFOs, step
    counters, partition and fold, so f32 / f16 / bf16 sums, all-gather and
    broadcast give bitwise the same outputs in a workgroup / per-wave /
    workgroup sequence, the per-wave pass runs the per-wave kernel for
    exactly its eligible calls, and an f32 prod (no per-wave kernel) keeps the
    workgroup one."""
    uid = nccl.get_unique_id()
    hexid = nccl.unique_id_to_bytes(uid).hex()
    env = dict(os.environ)
    env.update(TEST_GEOM)
    env.setdefault("VCCL_SPIN_TIMEOUT_S", "20")
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_handoff_worker.py"),
                                   str(r), str(n), hexid, d], env=_mp.worker_env(env),
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(n)]
        outs = [p.communicate(timeout=300)[0].decode(errors="replace")[-2000:] for p in procs]
        res = []
        for r in range(n):
            path = os.path.join(d, f"rank{r}.json")
            res.append(json.load(open(path)) if os.path.exists(path) else None)
        assert [p.returncode for p in procs] == [0] * n, (res, "\n".join(outs))
    for v in res:
        assert all(v["equal"].values()), v
        assert v["wave_launches_per_pass"] == [0, v["eligible"], 0], v


def test_beyond_2gib_two_ranks():
    """Per-rank buffers past 2 GiB (BASELINE config 4 is 4 GiB per rank): user
    buffer and FIFO / inbox accesses must address bytes beyond a 32-bit
    offset.  Two processes (one HIP queue set each, so the two ranks' kernels
    are co-resident) run ring AR, direct AR, ring RS and ring AG
    (tests/mp_big_worker.py checks each output with torch)."""
    uid = nccl.get_unique_id()
    hexid = nccl.unique_id_to_bytes(uid).hex()
    env = dict(os.environ)
    env.update(TEST_GEOM)
    env.pop("VCCL_DIRECT_THRESHOLD")  # direct: no size cap, default 16 MiB inbox chunks
    env.pop("VCCL_DIRECT_CHUNK_BYTES")
    env.setdefault("VCCL_SPIN_TIMEOUT_S", "20")
    n = 2
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_big_worker.py"),
                               str(r), str(n), "0", hexid], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(n)]
    logs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(out.decode(errors="replace")[-2000:])
    codes = [p.returncode for p in procs]
    assert codes == [0] * n, f"worker exit codes {codes}\n" + "\n".join(logs)


def _check_group(n, outs, nch, slot, algos, nthreads=512, chain=None):
    """Bit-exact against VCCL's GROUPED schedule on our rings and channels:
    every call takes its aggregate's path (`algos`, RC.group_algos) and its
    place in VCCL's multi-task plan (oracle plan_schedule);
    fp sum / prod also within the §8c tolerance of the exact value and of
    VCCL's grouped result on its reference geometry."""
    plan = RC.group_plan_works(n, nch, slot, nthreads, algos)
    vplan = RC.group_plan_works(n, RC.VCCL_REF_CHANNELS, RC.VCCL_REF_SLOT)
    for gi, (name, op, dt, count) in enumerate(RC.GROUP_CASES):
        exp = RC.expected_group(gi, n, nch, slot, nthreads, plan=plan, algos=algos, chain=chain)
        for r in range(n):
            assert_bitexact(dt, outs[r][name], exp, minmax=op in (2, 3),
                            what=f"group {name} n={n} rank {r}")
        vref = RC.vccl_group_reference(gi, n, vplan)
        if vref is not None:
            ins = [RC.gen_group_input(gi, r) for r in range(n)]
            for r in range(n):
                assert_fold_tolerance(dt, op, outs[r][name], exact_f64(dt, op, ins), ins, exp_is_exact=True,
                                      what=f"group {name} n={n} rank {r} vs exact")
                assert_fold_tolerance(dt, op, outs[r][name], vref, ins,
                                      what=f"group {name} n={n} rank {r} vs VCCL grouped schedule")


def test_group_fusion_single_process(monkeypatch):
    """Two comms driven from one thread: both comms' GROUP_CASES in ONE group,
    calls interleaved per comm, two streams per comm; runs of small all-reduces
    of one comm are fused into single LL launches (vcclCommLaunchStats)."""
    for k, v in TEST_GEOM.items():
        monkeypatch.setenv(k, v)
    nch, slot = int(TEST_GEOM["VCCL_NCHANNELS"]), int(TEST_GEOM["VCCL_SLOT_BYTES"])
    comms = nccl.Comm.init_all([0, 0])
    try:
        streams = [[torch.cuda.Stream(), torch.cuda.Stream()] for _ in comms]
        outs = RC.run_group(list(zip(comms, streams)), [0, 1], 2)
        for c in comms:
            assert c.async_error() == 0
        algos = RC.group_algos(comms[0].coll_algo, 2)
        assert algos == comms[0].group_algos([(0, c, dt, op) for _, op, dt, c in RC.GROUP_CASES])
        _check_group(2, [outs[0], outs[1]], nch, slot, algos)
        n_coll, fused = comms[0].launch_stats()
        # GROUP_CASES: [f32 x3] [f16 x2] big [f32] [bf16 x2] [i32] [u8] [f32 min x20 -> 16 + 4]
        assert fused == 5, fused
        assert n_coll == len(RC.GROUP_CASES)
    finally:
        for c in comms:
            c.destroy()


def test_group_ll_rs_ag_fused(monkeypatch):
    """A group's small reduce-scatters and all-gathers on the one-hop LL path
    fuse like LL all-reduces: 6 f32 reduce-scatters then 6 all-gathers of
    mixed types (each 0.25-3 KiB per block; one 4x aggregate per collective,
    still LL) launch as ONE LL kernel per collective (vcclCommLaunchStats), each
    part on its own slot lines and partition; every output exact (two comms
    driven from one thread, 2 ranks)."""
    import bench
    for k, v in TEST_GEOM.items():
        monkeypatch.setenv(k, v)
    comms = nccl.Comm.init_all([0, 0])
    try:
        n = 2
        streams = [torch.cuda.Stream() for _ in comms]
        rs_counts = [64 * (1 + i) for i in range(6)]           # recvcount (f32)
        ag = [(torch.float32, 7, 100 + 37 * i) if i % 2 == 0 else (torch.bfloat16, 9, 300 + 11 * i)
              for i in range(6)]
        xs, ys = {}, {}
        for r in range(n):
            for i, rc in enumerate(rs_counts):
                x = torch.empty(rc * n, device="cuda")
                bench.pattern_fill(x, r, n, base=i << 12)
                xs[r, "rs", i] = x
                ys[r, "rs", i] = torch.full((rc,), float("nan"), device="cuda")
            for i, (tdt, code, c) in enumerate(ag):
                xs[r, "ag", i] = torch.full((c,), float(r * 100 + i), device="cuda").to(tdt)
                ys[r, "ag", i] = torch.full((c * n,), float("nan"), device="cuda").to(tdt)
        torch.cuda.synchronize()
        assert comms[0].group_algos([(1, rc, 7, 0) for rc in rs_counts]) == ["ll"] * 6
        f0 = comms[0].launch_stats()[1]
        nccl.group_start()
        for r, c in enumerate(comms):
            sp = streams[r].cuda_stream
            for i, rc in enumerate(rs_counts):
                c.reduce_scatter(xs[r, "rs", i].data_ptr(), ys[r, "rs", i].data_ptr(), rc, 7, 0, sp)
            for i, (tdt, code, cnt) in enumerate(ag):
                c.all_gather(xs[r, "ag", i].data_ptr(), ys[r, "ag", i].data_ptr(), cnt, code, sp)
        nccl.group_end()
        torch.cuda.synchronize()
        for c in comms:
            assert c.async_error() == 0
        assert comms[0].launch_stats()[1] - f0 == 2  # one LL RS launch + one LL AG launch
        for r in range(n):
            for i, rc in enumerate(rs_counts):
                assert bench.pattern_ok(ys[r, "rs", i], n, base=(i << 12) + r * rc), ("rs", r, i)
            for i, (tdt, code, cnt) in enumerate(ag):
                want = torch.cat([torch.full((cnt,), float(q * 100 + i), device="cuda").to(tdt) for q in range(n)])
                assert torch.equal(ys[r, "ag", i], want), ("ag", r, i)
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("n,geom", [(2, "test"), (3, "test"), (4, "test"), (4, "ll128"), (2, "default")])
def test_broadcast(n, geom):
    """ncclBroadcast / ncclBcast (broadcast.h ring, bytes): 1 B - 24 MiB,
    every root, out of place and in place, and a group of broadcasts from
    different roots fused with an all-reduce; every byte exact
    (tests/mp_bcast_worker.py; n ranks sharing the GPU; "ll128": the LL128
    ring)."""
    uid = nccl.get_unique_id()
    hexid = nccl.unique_id_to_bytes(uid).hex()
    env = dict(os.environ)
    env.setdefault("VCCL_SPIN_TIMEOUT_S", "20")
    if geom == "default":
        for k in TEST_GEOM:
            env.pop(k, None)
        env["VCCL_ALLOW_SHARED_DEVICE"] = "1"
    else:
        env.update(TEST_GEOM)
        if geom == "ll128":
            env["NCCL_PROTO"] = "LL128"
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_bcast_worker.py"),
                               str(r), str(n), hexid], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(n)]
    outs = [p.communicate(timeout=300)[0].decode(errors="replace")[-2000:] for p in procs]
    assert [p.returncode for p in procs] == [0] * n, "\n".join(outs)


@pytest.mark.parametrize("env,want", [({}, 16), ({"NCCL_NCHANNELS": "12"}, 12),
                                      ({"NCCL_MAX_NCHANNELS": "5"}, 5), ({"NCCL_MAX_NRINGS": "7"}, 7),
                                      ({"NCCL_NCHANNELS": "4", "NCCL_MIN_NCHANNELS": "9"}, 9),
                                      ({"NCCL_MAX_CTAS": "6"}, 6), ({"NCCL_MIN_CTAS": "20"}, 20)])
def test_channel_count_knobs(monkeypatch, env, want):
    """The ring channel count at 2 ranks: the link-bound default (16), then
    NCCL_NCHANNELS, NCCL_MIN/MAX_NCHANNELS (legacy MIN/MAX_NRINGS,
    graph/connect.cc:326-360) and NCCL_MIN/MAX_CTAS bounding it.  Init only:
    the data path at other channel counts runs in the ring tests; two ranks of
    one process here would only be co-resident when their streams land on
    distinct hardware queues (see test_single_process_ranks)."""
    for k in list(TEST_GEOM) + ["NCCL_NCHANNELS", "NCCL_MAX_NCHANNELS", "NCCL_MIN_NCHANNELS",
                                "NCCL_MAX_NRINGS", "NCCL_MIN_CTAS", "NCCL_MAX_CTAS", "VCCL_CHANNELS_PER_RING"]:
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("VCCL_ALLOW_SHARED_DEVICE", "1")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    comms = nccl.Comm.init_all([0, 0])
    try:
        assert [c.n_channels() for c in comms] == [want, want]
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("n,geom", [(2, "test"), (3, "test"), (4, "test"), (4, "ll128"), (2, "default")])
def test_reduce(n, geom):
    """ncclReduce (reduce.h ring): RC.REDUCE_CASES at every root, bit-exact
    against the oracle's fold on the call's ring partition (start at the
    root's successor, end at the root with postOp), fp sum / prod also within
    the §8c tolerance of the exact value; a group of reduces to different
    roots with an all-reduce against VCCL's grouped plan
    (tests/mp_reduce_worker.py; n ranks sharing the GPU; "ll128": the LL128
    ring)."""
    from tests.mp_reduce_worker import GROUP
    uid = nccl.get_unique_id()
    hexid = nccl.unique_id_to_bytes(uid).hex()
    env = dict(os.environ)
    env.setdefault("VCCL_SPIN_TIMEOUT_S", "20")
    proto = 2
    if geom == "default":
        for k in TEST_GEOM:
            env.pop(k, None)
        env["VCCL_ALLOW_SHARED_DEVICE"] = "1"
        nch, slot = _ring.n_channels(n), 512 << 10
    else:
        env.update(TEST_GEOM)
        nch, slot = int(TEST_GEOM["VCCL_NCHANNELS"]), int(TEST_GEOM["VCCL_SLOT_BYTES"])
        if geom == "ll128":
            env["NCCL_PROTO"] = "LL128"
            proto = 1
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_reduce_worker.py"),
                                   str(r), str(n), hexid, d], env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(n)]
        outs = [p.communicate(timeout=300)[0].decode(errors="replace")[-2000:] for p in procs]
        assert [p.returncode for p in procs] == [0] * n, "\n".join(outs)
        res = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(n)]
    for ri, (name, op, dt, count, _) in enumerate(RC.REDUCE_CASES):
        ins = [RC.gen_reduce_input(ri, r) for r in range(n)]
        for root in range(n):
            exp = _ring.expected_reduce(op, dt, ins, root, nch, slot, proto=proto)
            got = res[root][f"{name}_r{root}"]
            assert_bitexact(dt, got, exp, minmax=op in (2, 3), what=f"reduce {name} n={n} root {root}")
            if op in RC.TOLERANCE_OPS and dt in (6, 7, 8, 9):
                assert_fold_tolerance(dt, op, got, exact_f64(dt, op, ins), ins, exp_is_exact=True,
                                      what=f"reduce {name} n={n} root {root} vs exact")
    # the group: every call on its aggregate's path and its place in VCCL's plan
    algos = [str(a) for a in res[0]["group_algos"]]
    assert all(str(a) == algos[k] for r in range(n) for k, a in enumerate(res[r]["group_algos"]))
    calls = [("red", RC.REDUCE_CASES[ri][1], RC.REDUCE_CASES[ri][2], RC.REDUCE_CASES[ri][3]) for ri, _ in GROUP]
    calls.append(("ar", 0, 7, 1 << 20))
    works = _ring.group_works(calls, n, nch, slot, algos=algos)
    for k, (ri, root) in enumerate(GROUP):
        name, op, dt, count, _ = RC.REDUCE_CASES[ri]
        ins = [RC.gen_reduce_input(ri, r) for r in range(n)]
        exp = _ring.expected_reduce(op, dt, ins, root % n, nch, slot, proto=1 if algos[k] == "ll128" else 2,
                                    work=works[k])
        assert_bitexact(dt, res[root % n][f"group{k}"], exp, minmax=op in (2, 3),
                        what=f"group reduce {k} ({name}) n={n} root {root % n}")


@pytest.mark.parametrize("n", [2, 4])
def test_comm_split(n):
    """ncclCommSplit (nccl.h.in:173-174): by color with reversed keys, and
    with NCCL_SPLIT_NOCOLOR on one rank — sub-communicator sizes and ranks as
    the reference orders them, an exact all-reduce on each, the parent intact
    (tests/mp_split_worker.py; n ranks sharing the GPU)."""
    uid = nccl.get_unique_id()
    hexid = nccl.unique_id_to_bytes(uid).hex()
    env = dict(os.environ)
    env.setdefault("VCCL_SPIN_TIMEOUT_S", "20")
    env.update(TEST_GEOM)
    hexid2 = nccl.unique_id_to_bytes(nccl.get_unique_id()).hex()  # the CTA-bounded parent
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_split_worker.py"),
                               str(r), str(n), hexid, hexid2], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(n)]
    outs = [p.communicate(timeout=240)[0].decode(errors="replace")[-2000:] for p in procs]
    assert [p.returncode for p in procs] == [0] * n, "\n".join(outs)


@pytest.mark.parametrize("init", ["lazy", "eager"])
def test_torch_process_group_dropin(init):
    """The drop-in boundary from the reference's own caller:
    torch.distributed's "nccl" backend with libvccl.so preloaded — its
    ncclCommInitRankConfig / ncclAllReduce / ncclReduceScatter /
    ncclAllGather calls land in this library — runs all_reduce (sum, avg,
    max), reduce_scatter_tensor and all_gather_into_tensor exactly on 2 ranks
    sharing cuda:0 (which RCCL refuses), and a sub-group — created with its
    own ncclCommInitRankConfig (lazy init) or split from the default group's
    communicator with ncclCommSplit (eager init, device_id=); the library's
    own INFO lines (VCCL_DEBUG=INFO) prove it served the calls
    (tests/mp_torch_pg_worker.py)."""
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    vlib = os.path.join(ROOT, "vccl_amd", "lib", "libvccl.so")
    port = str(29700 + os.getpid() % 200)
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, LD_PRELOAD=f"{tlib}:{vlib}", VCCL_ALLOW_SHARED_DEVICE="1",
                   VCCL_SPIN_TIMEOUT_S="20", VCCL_DEBUG="INFO", VCCL_DEBUG_SUBSYS="INIT,COLL",
                   TORCH_NCCL_ASYNC_ERROR_HANDLING="1",
                   VCCL_TEST_TORCH_INIT=init)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_torch_pg_worker.py")],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=240)[0].decode(errors="replace"))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    tails = "\n".join(o[-2500:] for o in outs)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for r, o in enumerate(outs):  # the evidence: this library's own log lines per rank
        with open(os.path.join(ROOT, "gpurun_out", f"torch_dropin_{init}_rank{r}.txt"), "w") as f:
            f.write("\n".join(o.splitlines()[:300]))
    assert [p.returncode for p in procs] == [0, 0], tails
    for o in outs:
        assert "ok" in o.splitlines()[-1], tails
        assert "[vccl" in o and "AllReduce: opCount" in o, tails  # served by this library
        if init == "eager":  # torch split the default communicator for the sub-group
            assert "ncclCommSplit: comm" in o, tails


def test_graph_capture_replay():
    """Collectives captured into a HIP graph replay correctly (device-resident
    LL epoch and ring step counters; no host state baked into the graph)."""
    n = 2
    uid = nccl.get_unique_id()
    env = dict(os.environ)
    env.update(TEST_GEOM)
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_graph_worker.py"),
                               str(r), str(n), nccl.unique_id_to_bytes(uid).hex()], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(n)]
    outs = [p.communicate(timeout=300)[0].decode(errors="replace")[-2000:] for p in procs]
    assert [p.returncode for p in procs] == [0] * n, "\n".join(outs)


def test_shared_device_ranks_beyond_hw_queues_rejected(monkeypatch):
    """n ranks of one comm on one GPU in one process need n co-resident
    kernels; with HIP's 4 hardware queues per process (one taken by the
    process's own stream) n = 4 would deadlock until the spin timeout
    (profiles/r01_diag_protocol.log), so init refuses it up front."""
    monkeypatch.setenv("VCCL_ALLOW_SHARED_DEVICE", "1")
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    with pytest.raises(nccl.VcclError) as e:
        nccl.Comm.init_all([0, 0, 0, 0])
    assert e.value.code == nccl.ncclInvalidUsage


def test_epoch_wrap(monkeypatch):
    """the LL parity and the direct flag values must survive the
    32-bit epoch wrap (0xffffffff -> 2, never 0, parity alternating).  Epochs
    seeded just below the wrap on both ranks (vcclCommDebugSetEpochs), then
    LL and multi-chunk direct all-reduces run across it, integer-exact."""
    for k, v in TEST_GEOM.items():
        monkeypatch.setenv(k, v)
    import bench
    comms = nccl.Comm.init_all([0, 0])
    try:
        for c in comms:
            c.debug_set_epochs(0xFFFFFFFD, 0xFFFFFFFE)
        streams = [torch.cuda.Stream() for _ in comms]
        # LL: 6 calls (epochs ...fffe, ...ffff, 2, 3, 4, 5); direct: 3 MiB
        # buckets through 1 MiB inbox chunks (3 flag values per call)
        for it, (nbytes, algo) in enumerate([(40 << 10, "ll")] * 6 + [(3 << 20, "direct")] * 4):
            n = nbytes // 4
            xs = [torch.empty(n, device="cuda") for _ in comms]
            ys = [torch.full((n,), float("nan"), device="cuda") for _ in comms]
            for r, x in enumerate(xs):
                bench.pattern_fill(x, r, 2, base=it << 20)
            for c in comms:
                c.set_algo(algo)
            torch.cuda.synchronize()
            nccl.group_start()
            for r, c in enumerate(comms):
                c.all_reduce(xs[r].data_ptr(), ys[r].data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum,
                             streams[r].cuda_stream)
            nccl.group_end()
            torch.cuda.synchronize()
            for r, c in enumerate(comms):
                assert c.async_error() == 0, f"call {it} ({algo}): spin timeout"
                assert bench.pattern_ok(ys[r], 2, base=it << 20), f"call {it} ({algo}) rank {r}"
    finally:
        for c in comms:
            c.destroy()


def test_initall_single_process_worker():
    """tests/mp_initall_worker.py (run by bench.py on multi-GPU boxes): one
    process, ncclCommInitAll, LL / default / ring all-reduce and RS + AG in
    groups.  On a one-GPU box it rehearses with two ranks on device 0; with
    more GPUs it runs over every GPU (peer access, no IPC)."""
    ndev = torch.cuda.device_count()
    arg = str(ndev) if ndev > 1 else "0,0"
    env = dict(os.environ)
    if ndev == 1:
        env["VCCL_ALLOW_SHARED_DEVICE"] = "1"
    env.setdefault("VCCL_SPIN_TIMEOUT_S", "20")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "mp_initall_worker.py"), arg],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["ok"], res


@pytest.mark.parametrize("n,geom", [(2, "default"), (4, "test"), (4, "ring_only")])
def test_group_zero_pattern(n, geom):
    """a group of 16 x 8 MiB bf16 reduce-scatters (a ZeRO
    bucket loop) launches ONCE, and a group of 8 mid-size fp32 all-reduces
    once (vcclCommLaunchStats), each aggregate on the path the library picks
    for its summed size (128 MiB of RS, 16 MiB of AR) — the ring at 2 ranks
    and with NCCL_ALGO=Ring, the one-hop / two-shot direct path at 4 ranks
    with the direct thresholds raised to cover the aggregates — and every
    output is bit-exact against the oracle's fold in VCCL's grouped order
    (tests/mp_group_worker.py)."""
    from tests import mp_group_worker as G
    uid = nccl.get_unique_id()
    hexid = nccl.unique_id_to_bytes(uid).hex()
    env = dict(os.environ)
    env.setdefault("VCCL_SPIN_TIMEOUT_S", "20")
    if geom in ("test", "ring_only"):
        env.update(TEST_GEOM)
        env.update(GROUP_DIRECT)
        nch, slot = int(TEST_GEOM["VCCL_NCHANNELS"]), int(TEST_GEOM["VCCL_SLOT_BYTES"])
        if geom == "ring_only":
            env["NCCL_ALGO"] = "Ring"
    else:
        for k in TEST_GEOM:
            env.pop(k, None)
        env["VCCL_ALLOW_SHARED_DEVICE"] = "1"
        nch, slot = _ring.n_channels(n), 512 << 10
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_group_worker.py"),
                                   str(r), str(n), hexid, d], env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(n)]
        outs = [p.communicate(timeout=300)[0].decode(errors="replace")[-2000:] for p in procs]
        assert [p.returncode for p in procs] == [0] * n, "\n".join(outs)
        res = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(n)]
    want = {"default": ("ring", "ring"), "test": ("direct", "direct"), "ring_only": ("ring", "ring")}[geom]
    assert (str(res[0]["algo_rs"]), str(res[0]["algo_ar"])) == want
    assert int(res[0]["fused"]) == 2, int(res[0]["fused"])  # one RS launch + one AR launch
    # VCCL's grouped plan of the 24 calls: bit-exact on our
    # rings and channels, within tolerance of VCCL's grouped result on its
    # reference geometry
    calls = G.call_list(G.GROUP_RS, G.GROUP_AR, 1, n)
    algos = [str(a) for a in res[0]["group_algos"]]
    assert algos == [str(a) for a in res[0]["lib_group_algos"]]  # oracle aggregation == library's
    assert len(set(algos[:16])) == 1 and len(set(algos[16:])) == 1, algos  # one aggregate each
    works = _ring.group_works(calls, n, nch, slot, algos=algos)
    vworks = _ring.group_works(calls, n, RC.VCCL_REF_CHANNELS, RC.VCCL_REF_SLOT)
    ident = [list(range(n))]
    for i, (name, dt, count) in enumerate(G.GROUP_RS):
        ins = [G.gen(name, dt, count, r) for r in range(n)]
        exp = _ring.expected_reducescatter(0, dt, ins, nch, slot, work=works[i])
        vref = _ring.expected_reducescatter(0, dt, ins, RC.VCCL_REF_CHANNELS, RC.VCCL_REF_SLOT,
                                            rings=ident, work=vworks[i])
        blk = count // n
        for r in range(n):
            assert_bitexact(dt, res[r][name], exp[r], what=f"{name} n={n} {geom} rank {r}")
            xs = [x[r * blk:(r + 1) * blk] for x in ins]
            assert_fold_tolerance(dt, 0, res[r][name], vref[r], xs,
                                  what=f"{name} n={n} {geom} rank {r} vs VCCL grouped")
    for i, (name, dt, count) in enumerate(G.GROUP_AR):
        ins = [G.gen(name, dt, count, r) for r in range(n)]
        k = len(G.GROUP_RS) + i
        exp = _ring.expected_allreduce(0, dt, ins, nch, slot, work=works[k])
        vref = _ring.expected_allreduce(0, dt, ins, RC.VCCL_REF_CHANNELS, RC.VCCL_REF_SLOT, rings=ident,
                                        work=vworks[k])
        for r in range(n):
            assert_bitexact(dt, res[r][name], exp, what=f"{name} n={n} {geom} rank {r}")
            assert_fold_tolerance(dt, 0, res[r][name], vref, ins,
                                  what=f"{name} n={n} {geom} rank {r} vs VCCL grouped")


def test_group_mixed_direct_sizes():
    """a fused direct launch whose parts differ in size —
    reduce-scatters of 5 MiB and 48 MiB buckets (two aggregates, both direct
    under the raised thresholds, one run) and all-reduces of 1.1 MiB and
    4 MiB, interleaved in one group, 4 ranks — must not let one part's
    scatter overwrite inbox bytes a peer's other workgroup still folds: every
    part of a batch uses one block length.  The group runs 3 times (outputs
    NaN-filled before each) and every run is bit-exact against VCCL's
    grouped plan."""
    from tests import mp_group_worker as G
    n = 4
    uid = nccl.get_unique_id()
    hexid = nccl.unique_id_to_bytes(uid).hex()
    env = dict(os.environ)
    env.setdefault("VCCL_SPIN_TIMEOUT_S", "20")
    env.update(TEST_GEOM)
    env.update(GROUP_DIRECT)
    nch, slot = int(TEST_GEOM["VCCL_NCHANNELS"]), int(TEST_GEOM["VCCL_SLOT_BYTES"])
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_group_worker.py"),
                                   str(r), str(n), hexid, d, "mixed"], env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(n)]
        outs = [p.communicate(timeout=300)[0].decode(errors="replace")[-2000:] for p in procs]
        assert [p.returncode for p in procs] == [0] * n, "\n".join(outs)
        res = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(n)]
    assert (str(res[0]["algo_rs"]), str(res[0]["algo_ar"])) == ("direct", "direct")
    assert int(res[0]["fused"]) == 2, int(res[0]["fused"])
    for r in range(n):
        assert not [k for k in res[r] if k.endswith("_differs")], (r, [k for k in res[r] if k.endswith("_differs")])
    calls = G.call_list(G.MIXED_RS, G.MIXED_AR, 3, n)
    algos = [str(a) for a in res[0]["group_algos"]]
    assert algos == [str(a) for a in res[0]["lib_group_algos"]]
    assert set(algos) == {"direct"}, algos
    works = iter(_ring.group_works(calls, n, nch, slot, algos=algos))
    for i in range(max(len(G.MIXED_RS), len(G.MIXED_AR))):
        for lst, coll in ((G.MIXED_RS, "rs"), (G.MIXED_AR, "ar")):
            if i >= len(lst):
                continue
            name, dt, count = lst[i]
            ins = [G.gen(name, dt, count, r) for r in range(n)]
            w = next(works)
            if coll == "rs":
                exp = _ring.expected_reducescatter(0, dt, ins, nch, slot, work=w)
                for r in range(n):
                    assert_bitexact(dt, res[r][name], exp[r], what=f"{name} rank {r}")
            else:
                exp = _ring.expected_allreduce(0, dt, ins, nch, slot, work=w)
                for r in range(n):
                    assert_bitexact(dt, res[r][name], exp, what=f"{name} rank {r}")


@pytest.mark.parametrize("geom", ["test", "ring_only", "ll128_window"])
def test_group_plan_stress(geom):
    """36 calls in one group (AR / RS / AG of f32 / bf16 / i32, sum, avg, max,
    1 KiB - 6 MiB, two streams) at 4 ranks: several (func, op, type) bins,
    aggregates and batches of up to 16 parts with channels skipped per part.
    Every call on its aggregate's path (vcclCommCollAlgo on the aggregate's
    summed count) and its place in VCCL's grouped plan, LL calls included;
    every output bit-exact (ring / direct: the ring fold on that place; LL
    all-reduce: the chain fold; LL reduce-scatter: per channel of its LL
    place); a second run of the group is bitwise identical."""
    from oracle import oracle as O
    from tests import mp_group_stress_worker as G
    n = 4
    uid = nccl.get_unique_id()
    hexid = nccl.unique_id_to_bytes(uid).hex()
    env = dict(os.environ)
    env.setdefault("VCCL_SPIN_TIMEOUT_S", "20")
    env.update(TEST_GEOM)
    if geom == "ring_only":
        env["NCCL_ALGO"] = "Ring"
    if geom == "ll128_window":
        # every path in one plan: LL up to 64 KiB, the LL128 ring's window
        # 64 KiB - 1 MiB, direct up to 4 MiB, the SIMPLE ring above
        env.update(VCCL_LL128="1", VCCL_LL_THRESHOLD=str(64 << 10))
    nch, slot = int(TEST_GEOM["VCCL_NCHANNELS"]), int(TEST_GEOM["VCCL_SLOT_BYTES"])
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_group_stress_worker.py"),
                                   str(r), str(n), hexid, d], env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(n)]
        outs = [p.communicate(timeout=300)[0].decode(errors="replace")[-2000:] for p in procs]
        assert [p.returncode for p in procs] == [0] * n, "\n".join(outs)
        res = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(n)]
    calls = G.stress_calls(n)
    algos = [str(a) for a in res[0]["algos"]]
    assert algos == [str(a) for a in res[0]["lib_algos"]]  # oracle aggregation == library's
    assert set(algos) <= {"ll", "ring", "direct", "ll128"}, algos
    if geom == "ring_only":  # NCCL_ALGO=Ring: the ring, ring LL for small RS / AG only
        assert set(algos) <= {"ring", "ll"} and "ring" in algos, algos
        assert all(c in ("rs", "ag") for (_, c, _, _, _), a in zip(calls, algos) if a == "ll"), algos
    elif geom == "ll128_window":
        assert set(algos) == {"ll", "ll128", "direct", "ring"}, algos  # all four paths in one plan
    else:
        assert len(set(algos)) >= 2, algos  # the plan spans paths
    for r in range(n):
        assert not [k for k in res[r] if k.endswith("_differs")], r
    works = _ring.group_works(G.group_calls(calls), n, nch, slot, algos=algos)
    for i, (name, coll, dt, op, count) in enumerate(calls):
        ins = [G.gen(name, dt, G.in_count(coll, count, n), r) for r in range(n)]
        if coll == "ag":
            exp = [np.concatenate(ins)] * n
        elif coll == "rs":
            exp = _ring.expected_reducescatter(op, dt, ins, nch, slot, work=works[i])
        elif algos[i] == "ll":
            dev_op, arg = O.host_to_dev_redop(op, dt, n)
            exp = [O.chain_fold(dev_op, dt, arg, dev_op == O.DEV_PREMULSUM, ins)] * n
        else:
            exp = [_ring.expected_allreduce(op, dt, ins, nch, slot, work=works[i])] * n
        for r in range(n):
            assert_bitexact(dt, res[r][name], exp[r], minmax=op in (2, 3),
                            what=f"{name} ({algos[i]}) {geom} rank {r}")


@pytest.mark.parametrize("n,event", [(2, "1"), (4, "1"), (2, "0")])
def test_calls_on_alternating_streams(n, event):
    """Forty calls of one comm outside any group, back to back on three
    streams in turn (LL, direct and ring all-reduces, reduce-scatters,
    all-gathers of 64 B - 12 MiB): each launch must wait for the previous
    one (shared FIFOs, LL slots, inbox regions) through the comm's ordering
    event — bound to the kernel's completion (VCCL_LAUNCH_EVENT=1, the
    default) or a recorded marker (0); every output exact
    (tests/mp_stream_worker.py)."""
    uid = nccl.get_unique_id()
    hexid = nccl.unique_id_to_bytes(uid).hex()
    env = dict(os.environ)
    env.setdefault("VCCL_SPIN_TIMEOUT_S", "20")
    env.update(TEST_GEOM)
    env["VCCL_LAUNCH_EVENT"] = event
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_stream_worker.py"),
                               str(r), str(n), hexid], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(n)]
    outs = [p.communicate(timeout=300)[0].decode(errors="replace")[-2000:] for p in procs]
    assert [p.returncode for p in procs] == [0] * n, "\n".join(outs)


@pytest.mark.parametrize("n", [2, 4])
def test_ring_trace_and_shared_cap(n):
    """The SIMPLE ring's slot timeline (VCCL_RING_TRACE, vcclCommRingTrace)
    and the co-residency cap of ranks sharing one GPU: with library defaults,
    n ranks on one device get min(default, 7/8 CUs / n) ring channels (the
    peer table gives every rank the same count); every traced slot has
    ordered stamps, an all-reduce shape and payload, and the output is
    exact (tests/mp_trace_worker.py)."""
    uid = nccl.get_unique_id()
    hexid = nccl.unique_id_to_bytes(uid).hex()
    env = dict(os.environ)
    for k in TEST_GEOM:
        env.pop(k, None)
    env.update(VCCL_ALLOW_SHARED_DEVICE="1", VCCL_RING_TRACE="256", VCCL_SPIN_TIMEOUT_S="20")
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_trace_worker.py"),
                                   str(r), str(n), hexid, d], env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(n)]
        outs = [p.communicate(timeout=300)[0].decode(errors="replace")[-2000:] for p in procs]
        assert [p.returncode for p in procs] == [0] * n, "\n".join(outs)
        res = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(n)]
    cus = int(res[0]["cus"])
    want = _mp.shared_channel_cap(n, _ring.n_channels(n), cus)
    ar_shapes = {0b0110, 0b0111, 0b1111, 0b1011, 0b1001}  # S->F, S+F->F, S+F->F+O, F->F+O, F->O
    for r in range(n):
        assert bool(res[r]["ok"]), f"rank {r}: all-reduce output"
        assert int(res[r]["nch"]) == want, (int(res[r]["nch"]), want)
        t, shape, nbytes = res[r]["t"], res[r]["shape"], res[r]["bytes"]
        used = t[..., 5] > 0  # t4 stored
        assert used.any()
        ts = t[used]  # t0 <= t1 <= t2 <= tc (thread 0's accesses issued) <= t3 <= t4
        assert (np.diff(ts, axis=-1) >= 0).all(), "stamps out of order"
        assert set(int(s) for s in shape[used]) <= ar_shapes
        assert nbytes[used].sum() > 0 and (nbytes[used] % 16 == 0).all()
        # every traced channel ran at least the 2n-1 steps of one loop
        assert (used.sum(axis=1)[used.any(axis=1)] >= 2 * n - 1).all()
