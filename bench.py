#!/usr/bin/env python3
"""Benchmark of the bucket-reduction hot path (BASELINE.json metric).

N = 1 (default): BASELINE config 2 — 2-input fp32 sum reduce-copy, 256 MiB
  device-resident buffers, through the C ABI (vcclReduceCopy).  One step = one
  launch over the whole bucket; value = algorithmic GB/s = 3 * 2^28 B per step
  / time.  Adds `roofline` (per-launch HIP-event duration vs 8 TB/s HBM3E),
  `cpu_baseline` (the oracle's C restatement on the host cores, bounded sample)
  and `extras` (config 1: 1 KiB fp32 ncclAllReduce at world size 1, us/call).
N > 1 (torch.distributed.run, one process per GPU): BASELINE config 3 at a
  fixed bucket — all-reduce fp32 sum through ncclAllReduce (the repo's own
  transport over xGMI peer memory, no RCCL; the library's algorithm choice,
  reported as config.algorithm).  value = bus bandwidth per rank, busbw =
  (S/t) * 2(n-1)/n with t the max over ranks (nccl-tests convention); the sum
  over ranks rides along as config.aggregate_busbw_all_ranks.
  torch.distributed (gloo, CPU tensors) only ships the unique id, barriers and
  the max-over-ranks time.  The same run adds `extras` (not `value`): config 3
  at a few sizes, config 5 (fp16, 8 B - 128 KiB, beside the SIMPLE ring and
  in graph mode), config 4 (RS + AG bf16, 4 GiB bucket), the ring and the
  direct algorithm each forced at 64 MiB and the headline bucket, the
  mid-range paths, group aggregation (16 small all-reduces issued one by one
  vs in one group), and config 3 on comms bounded to rings x 2..64 channels
  — skip with --no-extras.  Every timed path is checked afterwards.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--bytes S]
       [--workload reduce_copy|allreduce|rs_ag] [--sweep] [--no-extras]
"""
import argparse
import ctypes
import json
import os
import sys
import time

_T_START = time.perf_counter()  # before torch import: the line's wall time includes it


# ------------------------------------------------------------ rank launcher
# `bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment (a
# driver that does not go through torch.distributed.run): this process spawns
# the N rank processes itself — children, never an exec, and before anything
# here touches the GPU (torch is not even imported yet) — each with RANK /
# LOCAL_RANK / WORLD_SIZE / MASTER_ADDR 127.0.0.1 / MASTER_PORT, so every rank
# binds device LOCAL_RANK % device_count (one rank per GPU), and prints rank
# 0's JSON line with n_gpus = N.  --gpus and a WORLD_SIZE that disagree are an
# error, not a silent 1-GPU line.
def _gpus_arg(argv):
    """The --gpus value in argv, or None when absent."""
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            return int(argv[i + 1])
        if a.startswith("--gpus="):
            return int(a.split("=", 1)[1])
    return None


def world_check(argv, env):
    """(n, spawn): the world size this run has, and whether this process must
    spawn the ranks.  Raises SystemExit when --gpus and WORLD_SIZE disagree."""
    g = _gpus_arg(argv)
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if g is not None and g != int(ws):
            raise SystemExit(f"bench.py: --gpus {g} but WORLD_SIZE={ws}; launch one process per GPU "
                             f"(torch.distributed.run --nproc-per-node {g}) or drop WORLD_SIZE")
        return int(ws), False
    g = g or 1
    if g < 1:
        raise SystemExit(f"bench.py: --gpus {g}")
    return g, g > 1


def rank_launch_plan(argv, env, script=None, port=None):
    """[(cmd, env)] of the N rank processes `bench.py --gpus N` starts."""
    import socket
    n, spawn = world_check(argv, env)
    if not spawn:
        return []
    if port is None:
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
    script = script or os.path.abspath(__file__)
    plan = []
    for r in range(n):
        e = dict(env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                 VCCL_BENCH_LAUNCHER="bench.py")
        plan.append(([sys.executable, "-u", script] + list(argv), e))
    return plan


def _spawn_ranks(plan, poll_s=0.5):
    import subprocess
    procs = [subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE if k == 0 else subprocess.DEVNULL)
             for k, (cmd, e) in enumerate(plan)]
    out0 = []
    import threading
    t = threading.Thread(target=lambda: out0.extend(procs[0].stdout.read().decode().splitlines()), daemon=True)
    t.start()
    rc, failed_at = 0, None
    while any(p.poll() is None for p in procs):
        bad = [p for p in procs if p.poll() not in (None, 0)]
        if bad and failed_at is None:
            failed_at = time.monotonic()
            rc = bad[0].returncode
        if failed_at is not None and time.monotonic() - failed_at > 60:
            for p in procs:  # the exact children this process started
                if p.poll() is None:
                    p.kill()
        time.sleep(poll_s)
    t.join(timeout=10)
    codes = [p.returncode for p in procs]
    rc = rc or next((c for c in codes if c), 0)
    for line in out0:
        if line.startswith("{"):
            print(line, flush=True)
        else:
            print(line, file=sys.stderr, flush=True)
    if rc:
        print(f"bench.py: rank exit codes {codes}", file=sys.stderr, flush=True)
    return rc


if __name__ == "__main__":
    _plan = rank_launch_plan(sys.argv[1:], os.environ)
    if _plan:
        sys.exit(_spawn_ranks(_plan))

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from vccl_amd import nccl  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK_GBS = 153.6 / 2    # per link per direction (spec 153.6 GB/s bidirectional)


def _evt():
    return torch.cuda.Event(enable_timing=True)


def bench_reduce_copy(args):
    n = (args.bytes or (256 << 20)) // 4
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    g1 = torch.Generator(device="cuda").manual_seed(1)
    g2 = torch.Generator(device="cuda").manual_seed(2)
    a = torch.rand(n, device="cuda", generator=g1) * 2 - 1
    b = torch.rand(n, device="cuda", generator=g2) * 2 - 1
    d = torch.empty_like(a)
    cfg = None
    if args.block or args.unroll or args.grid or args.nt_loads or args.nt_stores:
        cfg = {"blockSize": args.block, "unroll": args.unroll, "gridBlocks": args.grid,
               "ntLoads": args.nt_loads, "ntStores": args.nt_stores}
    L = nccl.lib()
    srcs = (ctypes.c_void_p * 2)(a.data_ptr(), b.data_ptr())
    dsts = (ctypes.c_void_p * 1)(d.data_ptr())
    ccfg = nccl.vcclLaunchConfig(**{**{"order": 0}, **cfg}) if cfg else None

    def step():  # one launch of the hot path over the whole bucket, through the C ABI
        if ccfg is None:
            rc = L.vcclReduceCopy(0, nccl.ncclFloat32, 0, 0, 0, 2, srcs, 1, dsts, n, sp)
        else:
            rc = L.vcclReduceCopyEx(0, nccl.ncclFloat32, 0, 0, 0, 2, srcs, 1, dsts, n, sp,
                                    ctypes.byref(ccfg))
        if rc:
            raise nccl.VcclError(rc, "vcclReduceCopy")

    # Untimed pre-roll (reported as `preroll`, never counted): a fresh box's
    # GPU starts the timed region cold otherwise — a 5-launch warmup is ~0.6
    # ms of work, too short for the clocks to ramp, and the driver's round-1
    # line read 0.890 of peak while the same kernel in the same run (after
    # the CPU leg) read 0.911.  Fixed wall-clock budget of back-to-back
    # launches, then the caller's --warmup and --steps unchanged.
    pre_n, pre_t0 = 0, time.perf_counter()
    while time.perf_counter() - pre_t0 < args.preroll_s:
        for _ in range(64):
            step()
        torch.cuda.synchronize()
        pre_n += 64
    preroll = {"launches": pre_n, "s": round(time.perf_counter() - pre_t0, 3)}
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    e0, e1 = _evt(), _evt()
    t0 = time.perf_counter()
    # e0 goes in behind the first timed launch: the event pair then spans
    # launches 2..K back to back on a fed queue, not the host's first-launch
    # latency after the synchronize (~15-20 us, ~0.8 % of a 20-step region).
    # `value` keeps the whole wall-clock region.
    lead = 1 if args.steps >= 2 else 0
    for _ in range(lead):
        step()
    e0.record(stream)
    for _ in range(args.steps - lead):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    gpu_s = e0.elapsed_time(e1) / 1e3
    ev_launches = args.steps - lead
    # correctness of the measured buffers (bit-exact f32 add), after the timed
    # region so no idle gap separates warmup and timing
    assert torch.equal(d.view(torch.int32), (a + b).view(torch.int32)), "reduce-copy mismatch"
    # per-launch kernel durations, separately (an event pair per launch
    # serialises the queue, so it stays out of the timed region)
    kern_ms = []
    for _ in range(min(args.steps, 20)):
        s0, s1 = _evt(), _evt()
        s0.record(stream)
        step()
        s1.record(stream)
        torch.cuda.synchronize()
        kern_ms.append(s0.elapsed_time(s1))
    bytes_per = 3 * n * 4
    avg_kern_s = gpu_s / ev_launches  # HIP events inside the timed region, launch stream
    achieved = bytes_per / avg_kern_s / 1e9
    value = bytes_per * args.steps / wall / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": "k_reduce_copy<FnSum<float>,2,1>", "algorithmic_bytes_per_launch": bytes_per,
            "avg_launch_us": round(avg_kern_s * 1e6, 2), "event_span_launches": ev_launches,
            "single_launch_us_median": round(float(np.median(kern_ms)) * 1e3, 2)}
    out = {"metric": "device reduce-copy GB/s vs HBM peak; all-reduce busbw at 1/2/4/8 GPUs",
           "value": round(value, 1), "unit": "GB/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic uniform[-1,1) seeds 1,2 (device-resident)",
           "config": {"workload": "reduce_copy 2-src fp32 sum, 256 MiB buffers (BASELINE config 2)",
                      "bytes_per_buffer": n * 4, "n_srcs": 2, "n_dsts": 1,
                      "launch": cfg or "library default"},
           "roofline": roof, "preroll": preroll}
    # HBM traffic of the same kernel measured live on this box (PMC passes in
    # child processes); the committed summary only when that is impossible
    if not args.no_pmc_live:
        live, why = _pmc_live(bytes_per)
        if live is not None:
            roof["traffic"] = live["hbm_bytes_per_launch"]
            roof["traffic_detail"] = live
        else:
            roof["traffic"] = _pmc_traffic("reduce_copy", bytes_per)
            roof["traffic_detail"] = {"source": "committed profiles/pmc_traffic.json",
                                      "live_error": why}
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(n)
        try:
            out["cpu_baseline"]["staging"] = staging_rates(a, b)
        except Exception as e:  # noqa: BLE001 - reported, not fatal to the headline
            out["cpu_baseline"]["staging_error"] = repr(e)
    if not args.no_extras:
        out["extras"] = {"config1_allreduce_1KiB_world1": bench_one_rank_latency()}
        del a, b, d
        try:
            out["extras"]["reduce_copy_by_dtype"] = bench_rc_dtypes(n * 4)
        except Exception as e:  # noqa: BLE001 - reported, not fatal to the headline
            out["extras"]["reduce_copy_by_dtype_error"] = repr(e)
    return out


def bench_rc_dtypes(nbytes, steps=20, warmup=3, preroll_s=0.1):
    """Config 2's shape (2 sources -> 1 destination, `nbytes` per buffer) for
    each element type's sum kernel: GB/s (3 x nbytes per launch / event time
    on the launch stream) and the HBM-roofline fraction, after an untimed
    `preroll_s` of launches of that kernel.  Not `value`."""
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    L = nccl.lib()
    rows = []
    for name, dt in (("f32", nccl.ncclFloat32), ("f16", nccl.ncclFloat16), ("bf16", nccl.ncclBfloat16),
                     ("f8e4m3", nccl.ncclFloat8e4m3), ("f8e5m2", nccl.ncclFloat8e5m2),
                     ("i32", nccl.ncclInt32), ("u8", nccl.ncclUint8), ("f64", nccl.ncclFloat64)):
        esz = {nccl.ncclFloat16: 2, nccl.ncclBfloat16: 2, nccl.ncclFloat8e4m3: 1,
               nccl.ncclFloat8e5m2: 1, nccl.ncclUint8: 1, nccl.ncclFloat64: 8}.get(dt, 4)
        n = nbytes // esz
        a = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
        b = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
        if dt in (nccl.ncclFloat8e4m3, nccl.ncclFloat8e5m2):  # finite codes (no NaN/inf)
            a &= 0x77
            b &= 0x77
        d = torch.empty_like(a)
        srcs = (ctypes.c_void_p * 2)(a.data_ptr(), b.data_ptr())
        dsts = (ctypes.c_void_p * 1)(d.data_ptr())

        def step():
            rc = L.vcclReduceCopy(0, dt, 0, 0, 0, 2, srcs, 1, dsts, n, sp)
            if rc:
                raise nccl.VcclError(rc, "vcclReduceCopy")

        # Untimed pre-roll per kernel: a kernel's first use in a process can
        # ramp for ~150 launches (E5M2: 2.0 -> 6.9 TB/s over 8 batches of 20,
        # then 7.1 TB/s whenever used again; tools/dtype_rows.py first_use,
        # profiles/r02u), so the row reads the steady state.
        t_pre = time.perf_counter()
        while time.perf_counter() - t_pre < preroll_s:
            for _ in range(8):
                step()
            torch.cuda.synchronize()
        for _ in range(warmup):
            step()
        e0, e1 = _evt(), _evt()
        e0.record(stream)
        for _ in range(steps):
            step()
        e1.record(stream)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / steps
        gbs = 3 * nbytes / t / 1e9
        rows.append({"dtype": name, "GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                     "avg_launch_us": round(t * 1e6, 2)})
        del a, b, d
    return rows


def bench_one_rank_latency(iters=1000):
    """BASELINE config 1: ncclAllReduce fp32 sum, 1 KiB (256 elements), world
    size 1 through the loopback bootstrap: init/enqueue plumbing only (a D2D
    copy out of place, nothing in place).  us per call = HIP-event time of
    `iters` back-to-back calls / iters; output checked bitwise = input."""
    uid = nccl.get_unique_id()
    comm = nccl.Comm.init_rank(1, uid, 0)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    x = torch.rand(256, device="cuda", generator=torch.Generator(device="cuda").manual_seed(0)) * 2 - 1
    y = torch.empty_like(x)
    res = {}
    for name, dst in (("out_of_place", y), ("in_place", x)):
        for _ in range(20):
            comm.all_reduce(x.data_ptr(), dst.data_ptr(), 256, nccl.ncclFloat32, nccl.ncclSum, sp)
        e0, e1 = _evt(), _evt()
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(iters):
            comm.all_reduce(x.data_ptr(), dst.data_ptr(), 256, nccl.ncclFloat32, nccl.ncclSum, sp)
        e1.record(stream)
        torch.cuda.synchronize()
        res[name + "_us_per_call"] = round(e0.elapsed_time(e1) * 1e3 / iters, 3)
        res[name + "_host_us_per_call"] = round((time.perf_counter() - t0) * 1e6 / iters, 3)
    res["bitwise_equal"] = bool(torch.equal(x.view(torch.int32), y.view(torch.int32)))
    comm.destroy()
    return res


PMC_KERNEL = "k_reduce_copy<vccl::FnSum<float>, 2, 1,"


def _pmc_live(algo_bytes, timeout_s=120):
    """HBM bytes per launch of the headline kernel measured on THIS box: two
    rocprofv3 `--pmc` passes (FETCH_SIZE, then WRITE_SIZE: they do not fit one
    pass on gfx950), kernel trace only, each over a short child run of this
    same benchmark (5 launches after 2, no CPU leg / extras / pre-roll) under
    its own hard time limit; FETCH_SIZE doubled and both KiB x 1024 as
    MI355X_MICROARCH.md §HBM prescribes.  Returns a dict, or None with the
    reason when the profiler is unavailable or a pass fails."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    if shutil.which("rocprofv3") is None:
        return None, "rocprofv3 not found"
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="vccl_pmc_")
        cmd = ["timeout", "-s", "KILL", str(timeout_s), "rocprofv3", "--pmc", counter,
               "--output-format", "csv", "-d", d, "-o", "run", "--", sys.executable,
               os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2", "--no-cpu",
               "--no-extras", "--no-pmc-live", "--preroll-s", "0"]
        try:
            p = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp",
                               env={**os.environ, "TMPDIR": "/tmp"}, timeout=timeout_s + 30)
        except subprocess.TimeoutExpired:
            return None, f"{counter} pass timed out"
        if p.returncode != 0:
            return None, f"{counter} pass rc {p.returncode}: {(p.stderr or '')[-300:]}"
        got = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if PMC_KERNEL in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    got.append(float(row["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if not got:
            return None, f"no {counter} samples for {PMC_KERNEL}"
        vals[counter] = sum(got) / len(got)
    hbm = int((2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024)
    return {"hbm_bytes_per_launch": hbm, "traffic_over_algorithmic": round(hbm / algo_bytes, 4),
            "fetch_kib_raw": vals["FETCH_SIZE"], "write_kib": vals["WRITE_SIZE"],
            "method": "live rocprofv3 --pmc, separate FETCH_SIZE / WRITE_SIZE passes on this box; "
                      "FETCH_SIZE x2 (gfx950), KiB x1024"}, None


def _pmc_traffic(workload, algo_bytes):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_traffic.py),
    or None when no summary for this workload exists."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
        rec = d.get(workload)
        if rec and rec.get("algorithmic_bytes_per_launch") == algo_bytes:
            return rec["hbm_bytes_per_launch"]
    except (OSError, ValueError):
        pass
    return None


def _nproc():
    """CPUs this process may run on (what `nproc` prints)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _cpulist(txt):
    out = []
    for part in (txt or "").split(","):
        if "-" in part:
            lo, hi = part.split("-")
            out += range(int(lo), int(hi) + 1)
        elif part:
            out.append(int(part))
    return out


def host_topology():
    """CPUs this process may run on, their NUMA nodes, sockets and physical
    cores (sysfs), and the cgroup CPU quota if one is set."""
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else \
        list(range(os.cpu_count() or 1))
    node_of = {}
    base = "/sys/devices/system/node"
    for name in sorted(os.listdir(base)) if os.path.isdir(base) else []:
        if name.startswith("node") and name[4:].isdigit():
            for c in _cpulist(_read(os.path.join(base, name, "cpulist"))):
                node_of[c] = int(name[4:])
    sock, core = {}, {}
    for c in cpus:
        t = f"/sys/devices/system/cpu/cpu{c}/topology"
        sock[c] = int(_read(t + "/physical_package_id") or 0)
        core[c] = (sock[c], int(_read(t + "/core_id") or c))
    quota = None
    cm = _read("/sys/fs/cgroup/cpu.max")
    if cm and not cm.startswith("max"):
        q, per = cm.split()[:2]
        quota = int(q) / int(per)
    phys, seen = [], set()
    for c in cpus:
        if core[c] not in seen:
            seen.add(core[c])
            phys.append(c)
    nodes = sorted({node_of.get(c, 0) for c in cpus})
    return {"cpus": cpus, "nproc": len(cpus), "physical_cores": phys,
            "numa_nodes": len(nodes), "sockets": len({sock[c] for c in cpus}),
            "node_of": node_of, "cgroup_cpu_quota": quota,
            "machine_cpus": os.cpu_count()}


def _spread(cands, k, node_of):
    """k CPUs of `cands`, dealt round-robin over their NUMA nodes."""
    by = {}
    for c in cands:
        by.setdefault(node_of.get(c, 0), []).append(c)
    out, lists = [], list(by.values())
    while len(out) < k and any(lists):
        for lst in lists:
            if lst and len(out) < k:
                out.append(lst.pop(0))
    return out


def _host_register():
    """hipHostRegister (torch's cudart binding) of an existing host range: pins
    the pages where their first touch placed them.  Returns an undo callable,
    or None when registration is unavailable."""
    try:
        rt = torch.cuda.cudart()
    except Exception:  # noqa: BLE001
        return None

    def reg(ptr, nbytes):
        if int(rt.cudaHostRegister(ptr, nbytes, 0)) != 0:
            return None
        return lambda: rt.cudaHostUnregister(ptr)
    return reg


def cpu_baseline(n_full, seconds=5.0):
    """SURVEY.md §8(d) CPU baseline: the oracle's C restatement (oracle/
    reduce_ref.c) of the same 2-src f32 sum over the SAME shape as the device
    step (2 x 256 MiB -> 256 MiB), compiled -O3 -march=native on this host
    (oracle.native_lib), on persistent worker threads pinned one per CPU, each
    first-touching its own page-aligned slices (so every slice sits on the
    NUMA node of the core that reduces it), the pages then pinned with
    hipHostRegister (page-locked host memory, as the survey specifies, left
    where the first touch put them).  Runs on 1 core, on every CPU this
    process may use, on one thread per physical core, and — when a cgroup CPU
    quota is set — on that many physical cores spread over the NUMA nodes;
    each a bounded ~`seconds` sample checked bit-exactly.  `value` is the best
    multi-core figure.  A reported baseline only (the reference has no CPU
    reduce path)."""
    from oracle import oracle as O
    n = n_full
    topo = host_topology()
    reg = _host_register()
    runs = {"one_core": [topo["cpus"][0]], "all_cpus": topo["cpus"]}
    if len(topo["physical_cores"]) != len(topo["cpus"]):
        runs["physical_cores"] = topo["physical_cores"]
    q = topo["cgroup_cpu_quota"]
    if q and int(q) < len(topo["cpus"]) and int(q) >= 2:
        runs["quota_cores"] = _spread(topo["physical_cores"], int(q), topo["node_of"])
    res = {}
    for name, cpus in runs.items():
        res[name] = O.cpu_bench(n, cpus, seconds, register=reg)
    multi = {k: v for k, v in res.items() if k != "one_core"}
    best = max(multi, key=lambda k: multi[k]["GB/s"])
    assert all(v["correct"] for v in res.values()), "cpu baseline mismatch"
    return {"value": res[best]["GB/s"], "unit": "GB/s", "cores": res[best]["threads"], "kind": "port",
            "sample": f"2-src f32 sum over {n} elems (3 x {n * 4 >> 20} MiB host buffers, "
                      f"first-touched per worker, pinned={res[best]['pinned']}), oracle/reduce_ref.c "
                      f"-O3 -march={res[best]['march']}: {res[best]['iters']} passes in {res[best]['s']} s "
                      f"on {res[best]['threads']} pinned threads ({best}); every run checked bit-exactly",
            "best": best, "runs": res, "one_core": res["one_core"]["GB/s"],
            "nproc": topo["nproc"], "physical_cores": len(topo["physical_cores"]),
            "numa_nodes": topo["numa_nodes"], "sockets": topo["sockets"],
            "cgroup_cpu_quota": q, "machine_cpus": topo["machine_cpus"]}


def staging_rates(a, b, reps=5):
    """SURVEY.md §8(d) staging row, the inter-node analogue (VCCL's net
    transport without GPUDirect stages FIFO slots through host-pinned buffers,
    src/transport/net.cc:830-835, 1293-1482): config 2's device bucket `a`
    moved to pinned host memory (D2H), back (H2D), and end to end D2H -> host
    2-source f32 sum with a "received" peer bucket (`b`'s values, already in
    pinned host memory) by the oracle's C reduce-copy -> H2D, checked
    bitwise against a + b.  GB/s of one bucket per pass (median of `reps`)."""
    from oracle import oracle as O
    n = a.numel()
    nbytes = n * a.element_size()
    h = torch.empty(n, dtype=a.dtype, pin_memory=True)
    peer = b.cpu().pin_memory()
    red = torch.empty(n, dtype=a.dtype, pin_memory=True)
    out = torch.empty_like(a)
    threads = min(16, os.cpu_count() or 1)

    def med(fn, k=reps):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(k):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    t_d2h = med(lambda: h.copy_(a, non_blocking=True))
    t_h2d = med(lambda: out.copy_(h, non_blocking=True))
    hn, pn, rn = h.numpy(), peer.numpy(), red.numpy()

    def staged():
        h.copy_(a, non_blocking=True)
        torch.cuda.synchronize()
        O.reduce_copy(O.DEV_SUM, 7, 0, [hn, pn], out=[rn], nthreads=threads)
        out.copy_(red, non_blocking=True)

    t_st = med(staged, 3)
    ok = torch.equal(out.view(torch.int32), (a + b).view(torch.int32))
    del h, peer, red, out
    return {"bucket_bytes": nbytes, "d2h_GBs": round(nbytes / t_d2h / 1e9, 2),
            "h2d_GBs": round(nbytes / t_h2d / 1e9, 2), "staged_reduce_GBs": round(nbytes / t_st / 1e9, 2),
            "host_threads": threads, "correct": bool(ok),
            "note": "staged = D2H + host 2-src f32 sum (oracle C, pthreads) + H2D of one 256 MiB bucket, "
                    "end to end; pinned host buffers (SURVEY §8d staging row)"}


def _baseline_cpus():
    """The cores the N > 1 host baselines run on: the cgroup quota's worth of
    physical cores spread over the NUMA nodes, every physical core without a
    quota."""
    topo = host_topology()
    q = topo["cgroup_cpu_quota"]
    if q and 2 <= int(q) < len(topo["cpus"]):
        return topo, _spread(topo["physical_cores"], int(q), topo["node_of"]), "quota_cores"
    return topo, topo["physical_cores"], "physical_cores"


def cpu_baseline_allreduce(S, world, seconds=5.0, dtype=7, cpus=None):
    """Host-core baseline beside the N > 1 line (north_star):
    one rank's share of the ring all-reduce of an S-byte bucket over `world`
    ranks done as host work by the oracle's C reduce-copy (oracle/
    cpu_bench.c, -O3 -march=native on this host) — a world-source sum over
    S / world bytes into the rank's shard (the reduce-scatter's reductions),
    then a copy of the S gathered bytes (the all-gather) — on pinned, first-
    touched host buffers, one bounded ~`seconds` sample on the cgroup quota's
    worth of physical cores (every physical core when no quota is set; or
    `cpus`), checked bit-exactly.  `value` is in the line's unit: the busbw a
    rank doing that work on these cores would reach, (S / t_pass) * 2(n-1)/n.
    dtype: f32 (7, config 3), bf16 (9, config 4), f16 (6, config 5)."""
    from oracle import oracle as O
    topo, auto, which = _baseline_cpus()
    if cpus is None:
        cpus = auto
    else:
        which = f"{len(cpus)} core(s)"
    esz = {7: 4, 6: 2, 9: 2}[dtype]
    m, ncopy = S // (esz * world), S // esz
    r = O.cpu_bench_rank(m, world, ncopy, cpus, seconds, register=_host_register(), dtype=dtype)
    assert r["correct"], "cpu baseline mismatch"
    busbw = S / r["s_per_pass"] * 2 * (world - 1) / world / 1e9
    tname = {7: "f32", 6: "f16", 9: "bf16"}[dtype]
    return {"value": round(busbw, 3), "unit": "GB/s", "cores": r["threads"], "kind": "port",
            "sample": (f"one rank's share of a {world}-rank ring all-reduce of {S} B {tname} as host work: "
                       f"{world}-source sum over {m} elems + copy of {ncopy} elems, oracle/reduce_ref.c "
                       f"-O3 -march={r['march']}, pinned={r['pinned']}: {r['iters']} passes in {r['s']} s "
                       f"on {r['threads']} pinned threads ({which}); checked bit-exactly; value = "
                       "(S / t_pass) * 2(n-1)/n, the line's busbw convention"),
            "mem_GBs": r["mem_GB/s"], "us_per_pass": round(r["s_per_pass"] * 1e6, 2), "which": which,
            "nproc": topo["nproc"], "physical_cores": len(topo["physical_cores"]),
            "numa_nodes": topo["numa_nodes"], "cgroup_cpu_quota": topo["cgroup_cpu_quota"],
            "machine_cpus": topo["machine_cpus"]}


# The other configs with a reduce (SURVEY.md §8d "CPU baseline (all configs
# with a reduce)"), on bounded samples: config 4's bf16 bucket shape at
# 32 MiB (the oracle's bf16 arithmetic is a scalar, integer-exact
# restatement: the full 4 GiB would take minutes), config 5's largest fp16 LL
# bucket on one core (a latency-regime call).
CPU_OTHER = (("config4_rs_ag_bf16", 9, 32 << 20, None), ("config5_ll_f16", 6, 128 << 10, 1))


def ring_link_peak(orders, nchannels, link_gbs=None):
    """Per-rank busbw ceiling of the ring set a call runs on, one rank per GPU
    over point-to-point xGMI: channel c runs on ring c mod R, so a rank's send
    traffic T splits over the rings as their channel shares w_j / W, and a
    directed arc (a -> b) carries T * (sum of w_j over the rings that use it)
    / W <= one link per direction.  Peak T = L * W / (worst arc load).  2 ranks:
    1 link; 4 ranks (all 6 directed cycles, every arc in 2): 3 links; 6 ranks (4
    rings on 4 of 5 links): 4; odd n (Walecki, n - 1 arc-disjoint rings): n - 1;
    8 ranks: 7.  Returns the peak and the links it amounts to."""
    L = XGMI_LINK_GBS if link_gbs is None else link_gbs
    R = len(orders)
    w = [0] * R
    for c in range(max(1, nchannels)):
        w[c % R] += 1
    W = sum(w)
    load = {}
    for j, ring in enumerate(orders):
        if not w[j]:
            continue
        for k, a in enumerate(ring):
            arc = (a, ring[(k + 1) % len(ring)])
            load[arc] = load.get(arc, 0) + w[j]
    worst = max(load.values())
    out_links = max(len({b for (a, b) in load if a == r}) for r in orders[0])
    return {"peak": L * W / worst, "links": round(W / worst, 4), "links_used_per_rank": out_links,
            "rings": R, "channels": W, "worst_arc_share": round(worst / W, 4)}


def ring_ar_hbm_bytes(world, S):
    """HBM bytes one rank's ring all-reduce of S bytes moves:
    in units of S/n, send S->F (1 read, 1 write), n-2 x S+F->F (2, 1),
    S+F->F+O (2, 2), n-2 x F->F+O (1, 2), F->O (1, 1): (3n-2) reads and (3n-2)
    writes, 2(3n-2) S / n in all (4 S at n = 2).  FIFO writes land in the next
    rank's HBM, so every device moves the same total."""
    return 2 * (3 * world - 2) * S / world


def allreduce_roofline(busbw, t_s, S, world, ranks_per_device, algo, orders, nchannels, measured_link=None):
    """The N > 1 line's roofline.  One rank per GPU: the xGMI bound of the
    ring set in use (ring_link_peak).  Ranks sharing a device (the rehearsals):
    no byte crosses a link, so the bound is that device's HBM — every sharing
    rank's ring_ar_hbm_bytes per call over the call's time — and frac <= 1."""
    if ranks_per_device > 1:
        if algo != "ring":
            return {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                    "traffic": None, "note": f"ranks share a device; HBM bytes modelled for the ring only ({algo} ran)"}
        ach = ranks_per_device * ring_ar_hbm_bytes(world, S) / t_s / 1e9
        return {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "note": (f"{ranks_per_device} ranks share each device, so no byte crosses xGMI: the bound is the "
                         f"device's HBM, {ranks_per_device} x 2(3n-2)S/n B per call (the ring's HBM bytes per "
                         "rank, DESIGN.md §4.2) / t")}
    lp = ring_link_peak(orders, nchannels)
    return {"bound": "xgmi", "achieved": round(busbw, 2), "peak": round(lp["peak"], 2), "unit": "GB/s",
            "frac": round(busbw / lp["peak"], 4), "traffic": None,
            "note": (f"per-rank busbw vs the ring set's link ceiling: {lp['links']} link(s) x {XGMI_LINK_GBS} "
                     f"GB/s per link and direction ({lp['rings']} rings on {lp['channels']} channels, "
                     f"worst arc share {lp['worst_arc_share']}; MI355X spec 153.6 GB/s per link, bidirectional)"),
            "links": lp["links"], "links_used_per_rank": lp["links_used_per_rank"],
            "frac_of_measured_copy": (round(busbw / (lp["links"] * measured_link), 4) if measured_link else None)}


def line_roofline_and_baseline(dist, rank, world, last, visible, ring_orders, n_channels, xgmi,
                               cpu=True, cpu_seconds=5.0):
    """The N > 1 line's `roofline` and `cpu_baseline`: the
    host-core baseline of the headline bucket runs after every timed region,
    on rank 0 while the other ranks wait at the barrier; the roofline switches
    to the device's HBM when ranks share one (ranks_per_device > 1).  Returns
    (ranks_per_device, roofline, cpu_baseline or None)."""
    cpu_base = None
    if cpu:
        if rank == 0:
            try:
                cpu_base = cpu_baseline_allreduce(last["bytes"], world, cpu_seconds)
                cpu_base["other_configs"] = {}
                for name, dt, S, ncores in CPU_OTHER:
                    cores = None if ncores is None else _baseline_cpus()[1][:ncores]
                    try:
                        cpu_base["other_configs"][name] = cpu_baseline_allreduce(
                            S, world, min(cpu_seconds, 2.0), dtype=dt, cpus=cores)
                    except Exception as e:  # noqa: BLE001
                        cpu_base["other_configs"][name] = {"value": None, "error": repr(e)}
            except Exception as e:  # noqa: BLE001 - a failed baseline is reported, not fatal
                cpu_base = {"value": None, "error": repr(e)}
        dist.barrier()
    rpd = -(-world // max(1, visible))
    measured_link = (xgmi or {}).get("one_peer_GBs")
    roof = allreduce_roofline(last["busbw"], last["us"] / 1e6, last["bytes"], world, rpd, last["algo"],
                              ring_orders, n_channels, measured_link)
    if rpd == 1:
        roof["measured_peer_copy"] = xgmi
    return rpd, roof, cpu_base


def _dist_setup():
    import torch.distributed as dist
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    # one process per GPU; on a box with fewer GPUs than ranks (rehearsal),
    # ranks share devices round-robin
    torch.cuda.set_device(local % torch.cuda.device_count())
    if world > torch.cuda.device_count():  # rehearsal on a smaller box only
        os.environ["VCCL_ALLOW_SHARED_DEVICE"] = "1"
    # gloo prints its connection summary on fd 1; keep stdout for the one JSON line
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)
    obj = [nccl.unique_id_to_bytes(nccl.get_unique_id()) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    # LL128 ring buffers for the mid-range rows (the automatic choice is
    # unchanged: VCCL_LL128_ALLOC only allocates them)
    os.environ.setdefault("VCCL_LL128_ALLOC", "1")
    comm = nccl.Comm.init_rank(world, nccl.unique_id_from_bytes(obj[0]), rank)
    return dist, rank, world, comm


class _Tolerant:
    """A comm as the extras and the checks drive it: a collective the library
    refuses once the comm carries an async error (ncclRemoteError after a
    spin timeout, ncclInternalError after a slot-size check) is recorded in
    `refused`, not raised.  Ranks see their error words at different calls, so
    a raise on one rank would skip gloo collectives its peers still enter and
    hang the line — on the driver's one multi-GPU run the line must always
    print.  Everything else passes through to the comm."""
    _COLLS = ("all_reduce", "reduce_scatter", "all_gather", "broadcast", "reduce")

    def __init__(self, comm):
        self._comm = comm
        self.refused = 0

    def __getattr__(self, name):
        attr = getattr(self._comm, name)
        if name not in self._COLLS:
            return attr

        def call(*a, **kw):
            try:
                attr(*a, **kw)
            except nccl.VcclError as e:
                self.refused = self.refused or e.code
        return call


def _group_end():
    """ncclGroupEnd for the bench's grouped rows: a refused launch is left to
    the comm's async error (reported), not raised (see _Tolerant)."""
    try:
        nccl.group_end()
    except nccl.VcclError:
        pass


def _any_error(dist, comm):
    """The largest async error of `comm` over the ranks (a collective: every
    rank calls it at the same point)."""
    e = torch.tensor([comm.async_error() or getattr(comm, "refused", 0)], dtype=torch.int64)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    return int(e.item())


def _time_coll(dist, fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dist.barrier()
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class _HipIpcHandle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]


def peer_copy_bench(dist, rank, world, nbytes=256 << 20, steps=10):
    """xGMI microbench: write a local buffer into the next rank's HBM (one link,
    one direction) and into all peers at once (every outgoing link), with the
    library's copy kernel; buffers mapped via hipIpcGetMemHandle/OpenMemHandle.
    Pins the per-link denominator of the all-reduce roofline."""
    hip = ctypes.CDLL("libamdhip64.so")
    vp = ctypes.c_void_p
    hip.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(vp), _HipIpcHandle, ctypes.c_uint]
    hip.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(_HipIpcHandle), vp]
    local, remote = vp(), vp()
    assert hip.hipMalloc(ctypes.byref(local), ctypes.c_size_t(nbytes)) == 0
    assert hip.hipMalloc(ctypes.byref(remote), ctypes.c_size_t(nbytes)) == 0
    handle = _HipIpcHandle()
    assert hip.hipIpcGetMemHandle(ctypes.byref(handle), remote) == 0
    handles = [None] * world
    dist.all_gather_object(handles, bytes(ctypes.string_at(ctypes.addressof(handle), 64)))
    peers = {}
    res = {}
    try:
        for r in range(world):
            if r == rank:
                continue
            p = vp()
            h = _HipIpcHandle()
            ctypes.memmove(ctypes.addressof(h), handles[r], 64)
            rc = hip.hipIpcOpenMemHandle(ctypes.byref(p), h, 1)
            if rc != 0:
                raise RuntimeError(f"hipIpcOpenMemHandle -> {rc}")
            peers[r] = p.value
        ok = 1
    except RuntimeError as e:
        res["error"] = str(e)
        ok = 0
    t = torch.tensor([ok], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    sp = torch.cuda.current_stream().cuda_stream
    if t.item() == 1:
        nxt = (rank + 1) % world
        for name, dsts in (("one_peer", [peers[nxt]]), ("all_peers", list(peers.values()))):
            def fn(d=dsts):
                nccl.reduce_copy(nccl.vcclDevCopy, nccl.ncclUint8, 0, [local.value], d, nbytes, sp)
            dt = _time_coll(dist, fn, steps, 2)
            res[name + "_GBs"] = round(nbytes * len(dsts) * steps / dt / 1e9, 2)
    torch.cuda.synchronize()
    dist.barrier()
    for p in peers.values():
        hip.hipIpcCloseMemHandle(vp(p))
    hip.hipFree(local)
    hip.hipFree(remote)
    res["bytes"] = nbytes
    return res


# ----------------------------------------------------------------- checks
# Every path the N > 1 line times gets a correctness verdict on the real
# topology from integer-valued inputs, whose sums are exact in any fold order
# (|partial sums| <= 16 n <= 128: exact in f32, f16 and bf16), so a transport
# fault (lost, duplicated, misplaced or stale data) shows as a mismatch
# whatever algorithm ran.  Rank r's element i is LUT_r[g(i)] with g a 32-bit
# avalanche hash of the global index (no period a misplaced block could hide
# in) and LUT_r[v] = ((v + 7 r) & 31) - 16; the expected reduction is
# LUT_sum[g(i)] — one gather per element, sliced so 4 GiB buckets need no
# 4 GiB temporaries.
_SLICE = 1 << 26
_TDT = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}
_CODE = {"f32": nccl.ncclFloat32, "f16": nccl.ncclFloat16, "bf16": nccl.ncclBfloat16}


def _hash32(lo, hi, device="cuda"):
    """5-bit digest of a 32-bit avalanche hash (murmur3 finaliser) of every
    index in [lo, hi), computed in int64 with explicit 32-bit wrap."""
    m = 0xFFFFFFFF
    h = torch.arange(lo, hi, device=device, dtype=torch.int64) & m
    h = (h * 0x9E3779B1) & m
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & m
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & m
    h = h ^ (h >> 16)
    return h & 31


_DIGEST = {}
_DIGEST_CHUNK = 1 << 24


def _digest(lo, hi):
    """5-bit digest of every index in [lo, hi): a per-device uint8 cache grown
    in fixed 2^24-index chunks, chunk j drawn by torch's counter-based
    (Philox) generator seeded with 4242 + j — identical on every rank and
    every device whatever the cache size, with no period a misplaced block
    could hide in (_hash32 below is the equivalent closed form, kept for
    reference and CPU use)."""
    dev = torch.cuda.current_device()
    g = _DIGEST.get(dev)
    if g is None or g.numel() < hi:
        have = 0 if g is None else g.numel() // _DIGEST_CHUNK
        # geometric growth: growing by the chunk would leave every outgrown
        # buffer cached in torch's allocator (quadratic reserved memory)
        nchunks = max(-(-hi // _DIGEST_CHUNK), 2 * have)
        new = torch.empty(nchunks * _DIGEST_CHUNK, dtype=torch.uint8, device="cuda")
        if g is not None:
            new[:g.numel()] = g
        gen = torch.Generator(device="cuda")
        for j in range(have, nchunks):
            gen.manual_seed(4242 + j)
            new[j * _DIGEST_CHUNK:(j + 1) * _DIGEST_CHUNK] = torch.randint(
                0, 32, (_DIGEST_CHUNK,), dtype=torch.uint8, device="cuda", generator=gen)
        _DIGEST[dev] = g = new
    return g[lo:hi]


def _luts(world):
    v = torch.arange(32, device="cuda")
    per = [((v + 7 * r) & 31) - 16 for r in range(world)]
    return per, sum(per)


def pattern_fill(buf, r, world, base=0):
    """Fill the 1-D tensor `buf` with rank r's pattern for global indices
    [base, base + numel)."""
    # LUT_r[v] = ((v + 7 r) & 31) - 16 by arithmetic on the uint8 digest (no
    # index tensor): v + (7 r & 31) < 64 stays exact in uint8
    off = (7 * r) & 31
    n = buf.numel()
    for lo in range(0, n, _SLICE):
        hi = min(n, lo + _SLICE)
        t = _digest(base + lo, base + hi) + off
        t.bitwise_and_(31)
        dst = buf[lo:hi]
        dst.copy_(t)
        dst.sub_(16)


def pattern_ok(buf, world, base=0):
    """buf == the reduction of every rank's pattern over [base, base + numel)."""
    _, tot = _luts(world)
    lut = tot.to(buf.dtype)
    n = buf.numel()
    for lo in range(0, n, _SLICE):
        hi = min(n, lo + _SLICE)
        if not torch.equal(buf[lo:hi], lut[_digest(base + lo, base + hi).long()]):
            return False
    return True


def _all_ok(dist, ok):
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def check_ar(dist, comm, rank, world, nbytes, dtype="f32", algo=None):
    """One all-reduce of `nbytes` (out of place) on the path `algo` (None =
    the library's choice) with pattern inputs; True on every rank iff every
    rank's output is exact and no spin timed out."""
    tdt = _TDT[dtype]
    n = max(1, nbytes // torch.tensor([], dtype=tdt).element_size())
    x = torch.empty(n, dtype=tdt, device="cuda")
    y = torch.full((n,), float("nan"), dtype=tdt, device="cuda")
    pattern_fill(x, rank, world)
    sp = torch.cuda.current_stream().cuda_stream
    comm.set_algo(algo)
    try:
        torch.cuda.synchronize()
        comm.all_reduce(x.data_ptr(), y.data_ptr(), n, _CODE[dtype], nccl.ncclSum, sp)
        torch.cuda.synchronize()
    finally:
        comm.set_algo(None)
    ok = pattern_ok(y, world) and comm.async_error() == 0
    del x, y
    return _all_ok(dist, ok)


def check_rs_ag(dist, comm, rank, world, nbytes, dtype="bf16", algo=None):
    """Reduce-scatter of an `nbytes` bucket, then all-gather of the shards back
    (the ZeRO bucket path of config 4) on the path `algo` (None = the
    library's choice): (rs_ok, ag_ok) on every rank."""
    comm.set_algo(algo)
    try:
        return _check_rs_ag(dist, comm, rank, world, nbytes, dtype)
    finally:
        comm.set_algo(None)


def _check_rs_ag(dist, comm, rank, world, nbytes, dtype):
    tdt = _TDT[dtype]
    n = nbytes // torch.tensor([], dtype=tdt).element_size()
    rc = n // world
    x = torch.empty(rc * world, dtype=tdt, device="cuda")
    pattern_fill(x, rank, world)
    shard = torch.full((rc,), float("nan"), dtype=tdt, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    comm.reduce_scatter(x.data_ptr(), shard.data_ptr(), rc, _CODE[dtype], nccl.ncclSum, sp)
    torch.cuda.synchronize()
    rs_ok = pattern_ok(shard, world, base=rank * rc) and comm.async_error() == 0
    x.fill_(float("nan"))  # reuse as the all-gather output
    comm.all_gather(shard.data_ptr(), x.data_ptr(), rc, _CODE[dtype], sp)
    torch.cuda.synchronize()
    ag_ok = pattern_ok(x, world) and comm.async_error() == 0
    del x, shard
    return _all_ok(dist, rs_ok), _all_ok(dist, ag_ok)


def check_group(dist, comm, rank, world, nbytes, k):
    """k all-reduces of `nbytes` in one ncclGroupStart/End (fused LL launches)."""
    n = nbytes // 4
    xs = [torch.empty(n, device="cuda") for _ in range(k)]
    ys = [torch.full((n,), float("nan"), device="cuda") for _ in range(k)]
    for j, x in enumerate(xs):
        pattern_fill(x, rank, world, base=j << 24)
    sp = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    nccl.group_start()
    for x, y in zip(xs, ys):
        comm.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum, sp)
    _group_end()
    torch.cuda.synchronize()
    ok = all(pattern_ok(y, world, base=j << 24) for j, y in enumerate(ys))
    return _all_ok(dist, ok and comm.async_error() == 0)


def check_zero_group(dist, comm, rank, world, nbytes, k, dtype="bf16"):
    """The ZeRO bucket loop: k reduce-scatters of `nbytes` buckets in one
    ncclGroupStart/End (VCCL's grouped plan, host/enqueue.cc group_plan),
    pattern inputs; True on every rank iff every shard is exact."""
    tdt = _TDT[dtype]
    n = nbytes // torch.tensor([], dtype=tdt).element_size()
    rc = n // world
    xs = [torch.empty(rc * world, dtype=tdt, device="cuda") for _ in range(k)]
    ys = [torch.full((rc,), float("nan"), dtype=tdt, device="cuda") for _ in range(k)]
    for j, x in enumerate(xs):
        pattern_fill(x, rank, world, base=j << 26)
    sp = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    nccl.group_start()
    for x, y in zip(xs, ys):
        comm.reduce_scatter(x.data_ptr(), y.data_ptr(), rc, _CODE[dtype], nccl.ncclSum, sp)
    _group_end()
    torch.cuda.synchronize()
    ok = all(pattern_ok(y, world, base=(j << 26) + rank * rc) for j, y in enumerate(ys))
    del xs, ys
    return _all_ok(dist, ok and comm.async_error() == 0)


def _fences_plan(plan, algo_of):
    """One check per path family (kind, dtype, algorithm actually run) for the
    fences-on pass, at the family's smallest planned size (RS + AG at <= 64
    MiB): every path runs once with fences, the biggest buckets only without.
    algo_of(kind, kw) -> the algorithm the library runs for that check."""
    fam = {}
    for name, (kind, kw) in plan.items():
        key = (kind, kw.get("dtype"), algo_of(kind, kw), kw.get("k"), kw.get("wave"))
        if key not in fam or kw.get("nbytes", 0) < fam[key][1][1].get("nbytes", 0):
            fam[key] = (name, (kind, kw))
    out = {}
    for name, (kind, kw) in fam.values():
        if kind == "rs_ag" and kw["nbytes"] > (64 << 20):
            kw = {**kw, "nbytes": 64 << 20}
            name = name.rsplit("_", 1)[0] + f"_{64 << 20}"
        out[name] = (kind, kw)
    return out


def run_checks(dist, comm, rank, world, plan):
    """Run every check of `plan` ({name: (kind, args)}) with the fences off
    (the default), then each path family once more with system-scope fences
    on (vcclCommSetFences, the VCCL_FENCES=1 path); returns
    {"fences_off": {...}, "fences_on": {...}, "check_ms": {...}}."""
    def algo_of(kind, kw):
        if kw.get("algo"):
            return kw["algo"]
        dflt = "bf16" if kind in ("rs_ag", "zero_group") else "f32"
        esz = torch.tensor([], dtype=_TDT[kw.get("dtype", dflt)]).element_size()
        n = max(1, kw["nbytes"] // esz)
        code = _CODE[kw.get("dtype", dflt)]
        if kind in ("rs_ag", "zero_group"):
            return comm.coll_algo(1, n // world, code)
        return comm.coll_algo(0, n, code)

    res = {"check_ms": {}}
    for mode, fences, pl in (("fences_off", False, plan),
                             ("fences_on", True, _fences_plan(plan, algo_of))):
        comm.set_fences(fences)
        r = {}
        for name, (kind, kw) in pl.items():
            t0 = time.perf_counter()
            kw = dict(kw)
            comm.set_ring_wave(kw.pop("wave", False))  # the ring's slot hand-off for this check
            try:
                if kind == "ar":
                    r[name] = check_ar(dist, comm, rank, world, **kw)
                elif kind == "group":
                    r[name] = check_group(dist, comm, rank, world, **kw)
                elif kind == "zero_group":
                    r[name] = check_zero_group(dist, comm, rank, world, **kw)
                else:
                    rs_ok, ag_ok = check_rs_ag(dist, comm, rank, world, **kw)
                    r[name + "_rs"], r[name + "_ag"] = rs_ok, ag_ok
            except Exception as e:  # noqa: BLE001 - a failed check is a verdict, not a crash
                r[name] = f"error: {e!r}"
            finally:
                comm.set_ring_wave(False)
            res["check_ms"][f"{mode}:{name}"] = round((time.perf_counter() - t0) * 1e3, 1)
        res[mode] = r
    comm.set_fences(False)
    return res


def initall_check(world_devices, timeout=240):
    """Single-process ncclCommInitAll over every visible GPU (the reference
    test-harness shape; peer access instead of IPC), run in a
    child process (tests/mp_initall_worker.py) so a fault there cannot take the
    bench line with it.  Returns the worker's JSON verdict."""
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "tests", "mp_initall_worker.py"), str(world_devices)]
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout,
                           env={**os.environ, "VCCL_SPIN_TIMEOUT_S": "30"})
    except subprocess.TimeoutExpired:
        return {"ok": False, "error": f"timeout {timeout} s"}
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"ok": False, "rc": p.returncode, "error": (p.stderr or p.stdout)[-400:]}
    return json.loads(lines[-1])


def _flatten_ok(checks):
    vals = [v for k, m in checks.items() if k != "check_ms" for v in m.values()]
    return all(v is True for v in vals)


def bench_allreduce(args):
    dist, rank, world, comm = _dist_setup()
    sp = torch.cuda.current_stream().cuda_stream
    # One-time warm-up of the checker's own torch kernels (pattern fill /
    # compare per dtype on 4 Ki elements: their first launches load code
    # objects for ~0.1-0.2 s); reported as check_warmup_s, outside check_s.
    t_w = time.perf_counter()
    for tdt in _TDT.values():
        w = torch.empty(4096, dtype=tdt, device="cuda")
        pattern_fill(w, rank, world)
        pattern_ok(w, world)
    torch.cuda.synchronize()
    check_warmup_s = time.perf_counter() - t_w
    xgmi = peer_copy_bench(dist, rank, world) if not args.no_peer else None
    sizes = [1 << p for p in range(3, 31)] if args.sweep else [args.bytes or (1 << 30)]
    rows = []
    call_errs = []
    for S in sizes:
        n = max(1, S // 4)
        g = torch.Generator(device="cuda").manual_seed(1000 + rank)
        x = torch.rand(n, device="cuda", generator=g) * 2 - 1
        y = torch.empty_like(x)
        steps = args.steps if S >= (64 << 20) else max(args.steps, 20)

        def fn():
            # a call refused after an async error (ncclInternalError /
            # ncclRemoteError) is recorded, not raised: every rank must still
            # reach the same gloo barriers
            try:
                comm.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum, sp)
            except nccl.VcclError as e:
                call_errs.append(e.code)
        dt = _time_coll(dist, fn, steps, args.warmup)
        algbw = n * 4 * steps / dt / 1e9
        busbw = algbw * 2 * (world - 1) / world
        rows.append({"bytes": n * 4, "us": dt / steps * 1e6, "algbw": algbw, "busbw": busbw,
                     "algo": comm.coll_algo(0, n, nccl.ncclFloat32)})
        del x, y
        if rank == 0 and args.sweep:
            print(f"# allreduce {n*4:>12d} B  {dt/steps*1e6:10.1f} us  algbw {algbw:8.2f}  "
                  f"busbw {busbw:8.2f} GB/s  {rows[-1]['algo']}", file=sys.stderr, flush=True)
    # Fail fast: a spin timeout during the headline timing (the comm's error
    # word, on any rank) means the path is broken on this topology — every
    # extras row would open fresh comms and wait out their own timeouts.  The
    # line is then printed at once with the error and correct: false.
    e = torch.tensor([comm.async_error() or max(call_errs, default=0)], dtype=torch.int64)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    head_err = int(e.item())
    full = not args.sweep and not args.no_extras and head_err == 0
    tcomm = _Tolerant(comm)
    extras = bench_extras(dist, tcomm, rank, world, args) if full else None
    # Correctness of everything timed above, on this topology (fences off and on).
    t_chk = time.perf_counter()
    head = rows[-1]["bytes"]
    plan = {f"ar_default_{head}": ("ar", {"nbytes": head})}
    if full:
        for S in EXTRA_F32_SIZES:
            plan[f"ar_default_{S}"] = ("ar", {"nbytes": S})
        for S in EXTRA_F16_SIZES:
            plan[f"ar_f16_{S}"] = ("ar", {"nbytes": S, "dtype": "f16"})
            plan[f"ar_f16_ring_{S}"] = ("ar", {"nbytes": S, "dtype": "f16", "algo": "ring"})
        for algo in ("ring", "direct"):
            for S in (64 << 20, head):
                plan[f"ar_{algo}_{S}"] = ("ar", {"nbytes": S, "algo": algo})
        for algo in MID_ALGOS:
            for S in MID_SIZES:
                plan[f"ar_mid_{algo}_{S}"] = ("ar", {"nbytes": S, "algo": algo})
        for S in (64 << 20, head):  # the ring's per-wave slot hand-off (ring_handoff rows)
            plan[f"ar_ring_wave_{S}"] = ("ar", {"nbytes": S, "algo": "ring", "wave": True})
        plan[f"rs_ag_bf16_ring_wave_{args.rs_ag_bytes}"] = ("rs_ag", {"nbytes": args.rs_ag_bytes, "algo": "ring",
                                                                      "wave": True})
        for S in EXTRA_GROUP_SIZES:
            plan[f"group16_{S}"] = ("group", {"nbytes": S, "k": 16})
        plan[f"zero_group16_{ZERO_BUCKET}"] = ("zero_group", {"nbytes": ZERO_BUCKET, "k": 16})
        plan[f"rs_ag_bf16_{args.rs_ag_bytes}"] = ("rs_ag", {"nbytes": args.rs_ag_bytes})
        plan[f"rs_ag_bf16_direct_{args.rs_ag_bytes}"] = ("rs_ag", {"nbytes": args.rs_ag_bytes,
                                                                   "algo": "direct"})
        for S in EXTRA_RSAG_SIZES:
            for algo in (None, "ring"):
                plan[f"rs_ag_f32_{algo or 'default'}_{S}"] = ("rs_ag", {"nbytes": S, "dtype": "f32",
                                                                        "algo": algo})
    # after a headline error (the same verdict on every rank) nothing more is
    # run on the comm: its calls are refused, and a rank that raised would
    # skip the gloo collectives of a check that its peers still enter
    checks = (run_checks(dist, tcomm, rank, world, plan) if head_err == 0
              else {"check_ms": {}, "fences_off": {}, "fences_on": {}})
    err = comm.async_error()
    n_channels, ring_orders = comm.n_channels(), nccl.ring_orders(world)
    comm.destroy()
    initall = None
    if not args.no_initall and world > 1 and torch.cuda.device_count() > 1 and head_err == 0:
        # one process drives every GPU while the other ranks wait at the barrier
        initall = initall_check(torch.cuda.device_count()) if rank == 0 else None
        dist.barrier()
    t_chk = time.perf_counter() - t_chk
    last = rows[-1]
    rpd, roof, cpu_base = line_roofline_and_baseline(dist, rank, world, last, torch.cuda.device_count(),
                                                     ring_orders, n_channels, xgmi, cpu=not args.no_cpu)
    line_s = time.perf_counter() - _T_START
    correct_all = (_flatten_ok(checks) and (initall is None or initall.get("ok") is True)
                   and head_err == 0)
    out = {"metric": "device reduce-copy GB/s vs HBM peak; all-reduce busbw at 1/2/4/8 GPUs",
           "value": round(last["busbw"], 2), "unit": "GB/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(last["us"] / 1e3, 4),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic uniform[-1,1) seed 1000+rank (device-resident)",
           "config": {"workload": f"all-reduce fp32 sum, {last['bytes']} B per rank "
                                  "(BASELINE config 3), value = busbw per rank (nccl-tests "
                                  "convention: (S/t) * 2(n-1)/n, max time over ranks)",
                      "algorithm": last["algo"],
                      "bytes_per_rank": last["bytes"], "busbw_per_rank": round(last["busbw"], 2),
                      "aggregate_busbw_all_ranks": round(last["busbw"] * world, 2),
                      "algbw": round(last["algbw"], 2), "parallelism": f"{last['algo']} x{world}",
                      "async_error": err, "correct": correct_all,
                      "launcher": os.environ.get("VCCL_BENCH_LAUNCHER", "torch.distributed.run"),
                      "devices": {"visible": torch.cuda.device_count(), "ranks_per_device": rpd},
                      "channels": n_channels, "rings": len(ring_orders)},
           "roofline": roof,
           "cpu_baseline": cpu_base,
           "correct": {"all": correct_all, **checks, "initall_single_process": initall,
                       "headline_async_error": head_err,
                       **({"extras_skipped": "async error during the headline timing"}
                          if head_err and not args.sweep and not args.no_extras else {}),
                       "check_s": round(t_chk, 2), "check_warmup_s": round(check_warmup_s, 3),
                       "line_s": round(line_s, 2),  # bench.py start (imports included) -> here
                       "check_frac": round(t_chk / line_s, 3),
                       "check_frac_incl_warmup": round((t_chk + check_warmup_s) / line_s, 3),
                       "inputs": "integer-valued pattern (exact in any fold order), per timed path"}}
    if extras is not None:
        out["extras"] = extras
    if args.sweep:
        out["sweep"] = [{k: round(v, 3) if isinstance(v, float) else v for k, v in r.items()} for r in rows]
    dist.destroy_process_group()
    return out if rank == 0 else None


EXTRA_F32_SIZES = (8, 1 << 10, 8 << 10, 64 << 10, 1 << 20, 8 << 20, 64 << 20)
EXTRA_F16_SIZES = tuple(8 << k for k in range(15))  # config 5: 8 B - 128 KiB in x2 steps
GRAPH_F16_SIZES = (8, 1 << 10, 16 << 10, 128 << 10)  # config 5 in graph mode
EXTRA_GROUP_SIZES = (4 << 10, 32 << 10)
EXTRA_RSAG_SIZES = (64 << 10, 1 << 20, 8 << 20)  # whole bucket (n blocks), f32
# the mid range VCCL's tuner gives LL128 (enqueue.cc:2032): every path forced
MID_SIZES = (256 << 10, 1 << 20, 8 << 20)
MID_ALGOS = ("ring", "direct", "ll128")


def channel_knee(rows, default_channels, ranks_per_device, within=0.95):
    """What the `allreduce_f32_by_channels` rows say about the link-bound
    channel model (DESIGN.md §4.2, H = 8): the fewest channels reaching
    `within` of the best checked busbw (the knee), and where the default
    count stands against the best.  Meaningful on one rank per GPU only (a
    shared device is CU-bound, and says so)."""
    ok = [r for r in rows if r.get("correct") is True]
    if not ok:
        return {"knee_channels": None, "note": "no checked row"}
    best = max(ok, key=lambda r: r["busbw"])
    knee = min((r for r in ok if r["busbw"] >= within * best["busbw"]), key=lambda r: r["n_channels"])
    at_default = [r for r in ok if r["n_channels"] == default_channels]
    return {"default_channels": default_channels, "best_channels": best["n_channels"],
            "best_busbw": best["busbw"], "knee_channels": knee["n_channels"], "knee_within": within,
            "default_over_best": (round(at_default[0]["busbw"] / best["busbw"], 3) if at_default else None),
            "one_rank_per_gpu": ranks_per_device == 1,
            "reading": ("link-bound: H is right if the knee <= the default" if ranks_per_device == 1 else
                        "ranks share a device: every channel is CU-bound, no statement on H")}


def handoff_exit_rule(wg, pw, world, ranks_per_device, threshold=0.03):
    """DESIGN.md §9's exit rule for the per-wave ring hand-off, evaluated on
    the line's own `ring_handoff` rows (the 1 GiB all-reduce under each
    hand-off): it decides only on 8 ranks with one GPU each at 1 GiB; the
    line's `correct` must be green as well."""
    gain = wg["us"] / pw["us"] - 1 if pw["us"] > 0 else float("nan")
    applies = world == 8 and ranks_per_device == 1 and wg["bytes"] == 1 << 30
    verdict = (None if not applies else
               "per-wave becomes the bandwidth-regime default" if gain >= threshold else
               "per-wave kernels are deleted (ring_kernels.hip PART 4, prim_ws, WaveSync)")
    return {"rule": f"per-wave >= {threshold:.0%} faster at 1 GiB, 8 ranks, one per GPU, checks green",
            "per_wave_gain": round(gain, 4), "applies": applies, "verdict_if_checks_green": verdict}


def _ar_size_row(dist, comm, rank, world, S, dtype, steps, warmup):
    sp = torch.cuda.current_stream().cuda_stream
    tdt, code = {"f32": (torch.float32, nccl.ncclFloat32), "f16": (torch.float16, nccl.ncclFloat16)}[dtype]
    esz = torch.tensor([], dtype=tdt).element_size()
    n = max(1, S // esz)
    g = torch.Generator(device="cuda").manual_seed((1000 if dtype == "f32" else 3000) + rank)
    x = (torch.rand(n, device="cuda", generator=g) * 2 - 1).to(tdt)
    y = torch.empty_like(x)
    dt = _time_coll(dist, lambda: comm.all_reduce(x.data_ptr(), y.data_ptr(), n, code, nccl.ncclSum, sp),
                    steps, warmup)
    algbw = n * esz * steps / dt / 1e9
    return {"bytes": n * esz, "us": round(dt / steps * 1e6, 2),
            "busbw": round(algbw * 2 * (world - 1) / world, 3), "algo": comm.coll_algo(0, n, code)}


def _ar_graph_row(dist, comm, rank, world, S, dtype="f16", calls=50, replays=10, stream=None):
    """Config 5 in graph mode (nccl-tests ``-G``): ``calls`` all-reduces of S
    bytes captured into one HIP graph, replayed ``replays`` times; us per call
    = replay time / calls (no per-call launch cost).  The replayed output is
    compared bitwise with an eager call of the same algorithm."""
    tdt, code = {"f32": (torch.float32, nccl.ncclFloat32), "f16": (torch.float16, nccl.ncclFloat16)}[dtype]
    esz = torch.tensor([], dtype=tdt).element_size()
    n = max(1, S // esz)
    g = torch.Generator(device="cuda").manual_seed(3000 + rank)
    x = (torch.rand(n, device="cuda", generator=g) * 2 - 1).to(tdt)
    y, ref = torch.empty_like(x), torch.empty_like(x)
    cs = stream if stream is not None else torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.stream(cs):
        graph.capture_begin(capture_error_mode="relaxed")
        try:
            for _ in range(calls):
                comm.all_reduce(x.data_ptr(), y.data_ptr(), n, code, nccl.ncclSum, cs.cuda_stream)
        finally:  # a failing call must not leave the stream capturing (the process would abort)
            graph.capture_end()
    torch.cuda.synchronize()
    dt = _time_coll(dist, graph.replay, replays, 2)
    # each replay alone (barrier, replay, synchronize; max over ranks): shows
    # whether the average hides a single slow replay
    per = []
    for _ in range(replays):
        per.append(_time_coll(dist, graph.replay, 1, 0) / calls * 1e6)
    sp = torch.cuda.current_stream().cuda_stream
    comm.all_reduce(x.data_ptr(), ref.data_ptr(), n, code, nccl.ncclSum, sp)
    torch.cuda.synchronize()
    ok = _all_ok(dist, bool(torch.equal(y.view(torch.int16 if esz == 2 else torch.int32),
                                        ref.view(torch.int16 if esz == 2 else torch.int32))))
    del graph
    us = dt / (replays * calls) * 1e6
    return {"bytes": n * esz, "us": round(us, 2), "calls_per_graph": calls,
            "busbw": round(n * esz / us / 1e3 * 2 * (world - 1) / world, 3),
            "us_per_call_each_replay": [round(v, 2) for v in per],
            "algo": comm.coll_algo(0, n, code), "matches_eager": ok}


def _group_row(dist, comm, rank, world, S, k, steps=20, warmup=3):
    """k all-reduces of S bytes (fp32 sum): issued one by one vs inside one
    ncclGroupStart/End, where runs of small buckets are fused into one launch."""
    sp = torch.cuda.current_stream().cuda_stream
    n = S // 4
    xs = [torch.rand(n, device="cuda") for _ in range(k)]
    ys = [torch.empty_like(x) for x in xs]

    def calls():
        for x, y in zip(xs, ys):
            comm.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum, sp)

    def grouped():
        nccl.group_start()
        calls()
        _group_end()
    t_sep = _time_coll(dist, calls, steps, warmup)
    f0 = comm.launch_stats()[1]
    t_grp = _time_coll(dist, grouped, steps, warmup)
    return {"bytes": S, "calls": k, "us_separate": round(t_sep / steps * 1e6, 2),
            "us_grouped": round(t_grp / steps * 1e6, 2),
            "fused_launches_per_group": (comm.launch_stats()[1] - f0) / (steps + warmup),
            "algo": comm.coll_algo(0, n, nccl.ncclFloat32),
            # grouped, the calls take the path of their aggregate (VCCL's plan)
            "algo_grouped": comm.group_algos([(0, n, nccl.ncclFloat32, nccl.ncclSum)] * k)[0]}


ZERO_BUCKET = 8 << 20  # bytes per bucket of the ZeRO reduce-scatter group row


def _zero_group_row(dist, comm, rank, world, S=ZERO_BUCKET, k=16, steps=10, warmup=2):
    """The ZeRO bucket loop: k reduce-scatters of S-byte bf16 buckets issued
    one by one vs inside one ncclGroupStart/End, where they take VCCL's
    grouped plan (shared channels, one fused launch); busbw per rank over the
    k buckets, (k S / t) (n-1)/n."""
    sp = torch.cuda.current_stream().cuda_stream
    n = S // 2
    rc = n // world
    xs = [torch.rand(rc * world, device="cuda").to(torch.bfloat16) for _ in range(k)]
    ys = [torch.empty(rc, dtype=torch.bfloat16, device="cuda") for _ in range(k)]

    def calls():
        for x, y in zip(xs, ys):
            comm.reduce_scatter(x.data_ptr(), y.data_ptr(), rc, nccl.ncclBfloat16, nccl.ncclSum, sp)

    def grouped():
        nccl.group_start()
        calls()
        _group_end()
    t_sep = _time_coll(dist, calls, steps, warmup)
    f0 = comm.launch_stats()[1]
    t_grp = _time_coll(dist, grouped, steps, warmup)
    bw = lambda t: round(k * S * steps / t / 1e9 * (world - 1) / world, 2)  # noqa: E731
    del xs, ys
    return {"bucket_bytes": S, "calls": k, "dtype": "bf16", "us_separate": round(t_sep / steps * 1e6, 2),
            "us_grouped": round(t_grp / steps * 1e6, 2), "busbw_separate": bw(t_sep),
            "busbw_grouped": bw(t_grp),
            "fused_launches_per_group": (comm.launch_stats()[1] - f0) / (steps + warmup),
            "algo": comm.coll_algo(1, rc, nccl.ncclBfloat16),
            # grouped, the k buckets aggregate and take the aggregate's path
            "algo_grouped": comm.group_algos([(1, rc, nccl.ncclBfloat16, nccl.ncclSum)] * k)[0]}


def bench_extras(dist, comm, rank, world, args):
    """Secondary BASELINE configs measured in the same multi-GPU run (reported
    beside the headline, never as ``value``): config 3 at a few sizes (fp32),
    config 5 (fp16, LL sizes), the ring and the direct algorithm each forced,
    group aggregation, and config 4 (RS + AG bf16, 4 GiB bucket).  Each part
    records its own error instead of aborting; run_checks verifies each."""
    ex = {}

    def go():  # the same verdict on every rank: stop at the first async error
        err = _any_error(dist, comm)
        if err:
            ex["stopped"] = f"async error {err}: the remaining rows were skipped"
        return err == 0
    try:
        ex["allreduce_f32_sizes"] = [_ar_size_row(dist, comm, rank, world, S, "f32", 20, 5)
                                     for S in EXTRA_F32_SIZES]
        ex["allreduce_f16_ll"] = [_ar_size_row(dist, comm, rank, world, S, "f16", 50, 5)
                                  for S in EXTRA_F16_SIZES]
        comm.set_algo("ring")  # config 5's comparison: the SIMPLE ring at the same sizes
        ex["allreduce_f16_ring"] = [_ar_size_row(dist, comm, rank, world, S, "f16", 50, 5)
                                    for S in EXTRA_F16_SIZES]
    except Exception as e:  # noqa: BLE001 - reported, not fatal to the headline
        ex["allreduce_error"] = repr(e)
    finally:
        comm.set_algo(None)
    if not go():
        return ex
    try:
        ex["group_fusion_f32"] = [_group_row(dist, comm, rank, world, S, 16) for S in EXTRA_GROUP_SIZES]
        ex["zero_group_rs_bf16"] = _zero_group_row(dist, comm, rank, world)
    except Exception as e:  # noqa: BLE001
        ex["group_error"] = repr(e)
    if not go():
        return ex
    try:  # each algorithm forced at two bucket sizes (vcclCommSetAlgo): the SIMPLE
        # ring of the north-star target beside the automatic choice
        ex["allreduce_f32_by_algo"] = {}
        for algo in ("ring", "direct"):
            comm.set_algo(algo)
            ex["allreduce_f32_by_algo"][algo] = [
                _ar_size_row(dist, comm, rank, world, S, "f32", st, 2)
                for S, st in ((64 << 20, 10), (args.bytes or (1 << 30), 5))]
    except Exception as e:  # noqa: BLE001
        ex["by_algo_error"] = repr(e)
    finally:
        comm.set_algo(None)
    if not go():
        return ex
    try:  # the SIMPLE ring's slot hand-off: the workgroup one (default) vs per wave
        # (vcclCommSetRingWave / VCCL_RING_WAVE), config 3 and config 4 on the ring
        ex["ring_handoff"] = {}
        comm.set_algo("ring")
        for wave in (False, True):
            comm.set_ring_wave(wave)
            ex["ring_handoff"]["per_wave" if wave else "workgroup"] = {
                "allreduce_f32": [_ar_size_row(dist, comm, rank, world, S, "f32", st, 2)
                                  for S, st in ((64 << 20, 10), (args.bytes or (1 << 30), 5))],
                "rs_ag_bf16": _rs_ag(dist, comm, rank, world, args.rs_ag_bytes, min(args.steps, 10), 2)}
        ex["ring_handoff"]["per_wave_launches"] = comm.set_ring_wave(False)
        ex["ring_handoff"]["exit_rule"] = handoff_exit_rule(
            ex["ring_handoff"]["workgroup"]["allreduce_f32"][-1],
            ex["ring_handoff"]["per_wave"]["allreduce_f32"][-1], world,
            -(-world // torch.cuda.device_count()))
    except Exception as e:  # noqa: BLE001
        ex["ring_handoff_error"] = repr(e)
    finally:
        comm.set_ring_wave(False)
        comm.set_algo(None)
    if not go():
        return ex
    try:  # the mid range (64 KiB - 8 MiB: LL128's slot in VCCL's tuner), each path forced
        ex["allreduce_f32_mid_by_algo"] = {}
        for algo in MID_ALGOS:
            comm.set_algo(algo)
            ex["allreduce_f32_mid_by_algo"][algo] = [
                _ar_size_row(dist, comm, rank, world, S, "f32", 20, 3) for S in MID_SIZES]
    except Exception as e:  # noqa: BLE001
        ex["mid_by_algo_error"] = repr(e)
    finally:
        comm.set_algo(None)
    if not go():
        return ex
    try:
        ex["rs_ag_bf16"] = _rs_ag(dist, comm, rank, world, args.rs_ag_bytes, min(args.steps, 10), 2)
        comm.set_algo("direct")
        ex["rs_ag_bf16_direct"] = _rs_ag(dist, comm, rank, world, args.rs_ag_bytes,
                                         min(args.steps, 10), 2)
    except Exception as e:  # noqa: BLE001
        ex["rs_ag_error"] = repr(e)
    finally:
        comm.set_algo(None)
    if not go():
        return ex
    try:  # the ring broadcast (DDP's construction-time state broadcast), root 0
        ex["broadcast_f32"] = [_bcast_row(dist, comm, rank, world, S) for S in BCAST_SIZES]
    except Exception as e:  # noqa: BLE001
        ex["broadcast_error"] = repr(e)
    if not go():
        return ex
    try:  # the ring reduce into the last rank
        ex["reduce_f32"] = [_reduce_row(dist, comm, rank, world, S) for S in BCAST_SIZES]
    except Exception as e:  # noqa: BLE001
        ex["reduce_error"] = repr(e)
    if not go():
        return ex
    try:  # small / mid buckets: the one-hop LL / direct RS + AG vs the ring
        ex["rs_ag_f32_sizes"] = []
        for S in EXTRA_RSAG_SIZES:
            for algo in (None, "ring"):
                comm.set_algo(algo)
                ex["rs_ag_f32_sizes"].append(_rs_ag(dist, comm, rank, world, S, 20, 3, dtype="f32"))
    except Exception as e:  # noqa: BLE001
        ex["rs_ag_sizes_error"] = repr(e)
    finally:
        comm.set_algo(None)
    if not go():
        return ex
    try:  # config 3 on communicators bounded to C ring channels: the link model's headroom
        ex["allreduce_f32_by_channels"] = _channel_rows(dist, rank, world, args.bytes or (1 << 30),
                                                        min(args.steps, 5))
        ex["channel_model"] = channel_knee(ex["allreduce_f32_by_channels"], comm.n_channels(),
                                           -(-world // torch.cuda.device_count()))
    except Exception as e:  # noqa: BLE001
        ex["channels_error"] = repr(e)
    if not go():
        return ex
    try:  # the ring's slot timeline on the headline bucket, both hand-offs
        ex["ring_trace"] = _ring_trace_row(dist, rank, world, args.bytes or (1 << 30))
    except Exception as e:  # noqa: BLE001
        ex["ring_trace_error"] = repr(e)
    if not go():
        return ex
    try:  # the inter-node path with its staging copies, on the ranks of this run
        ex["allreduce_f32_net"] = _net_row(dist, rank, world)
    except Exception as e:  # noqa: BLE001
        ex["net_error"] = repr(e)
    # Last: config 5 without per-call launch cost (nccl-tests -G: HIP graph
    # replay).  Its capture stream is one more hardware queue per process;
    # with 8 ranks sharing one GPU (rehearsal) that oversubscribes the
    # scheduler's queues and every later row would run time-sliced.
    if not go():
        return ex
    try:
        # one capture stream for every row: with ranks sharing one GPU, the
        # second stream a process creates served ~28 us per replayed call
        # whatever the size, while every row on one shared stream ran at
        # ~4.2 us (tools/ll_graph_probe.py, profiles/r04g)
        cap = torch.cuda.Stream()
        ex["allreduce_f16_ll_graph"] = [_ar_graph_row(dist, comm, rank, world, S, stream=cap)
                                        for S in GRAPH_F16_SIZES]
    except Exception as e:  # noqa: BLE001
        ex["graph_error"] = repr(e)
    ex["async_error"] = comm.async_error()
    return ex


_TRACE_SHAPES = {0b0110: "S->F", 0b0111: "S+F->F", 0b1111: "S+F->F+O", 0b1101: "S+F->O", 0b1011: "F->F+O",
                 0b1001: "F->O", 0b1110: "S->F+O"}


def ring_trace_summary(tr):
    """Per primitive shape of a VCCL_RING_TRACE timeline (vcclCommRingTrace,
    one record per FIFO slot per channel, s_memrealtime at 100 MHz): the mean
    time per slot waiting for credits (t1-t0), for the workgroup release
    (t2-t1), moving and draining the payload (t3-t2 = issue tc-t2 + drain
    t3-tc), posting (t4-t3), the gap to the channel's next slot, and the
    payload rate of the copy phase."""
    rows = {}
    for ch in range(tr.shape[0]):
        rec = tr[ch][tr[ch]["t4"] > 0]
        for i, r in enumerate(rec):
            d = rows.setdefault(_TRACE_SHAPES.get(int(r["shape"]), str(int(r["shape"]))),
                                {"n": 0, "wait": 0.0, "release": 0.0, "copy": 0.0, "post": 0.0, "gap": 0.0,
                                 "issue": 0.0, "drain": 0.0, "bytes": 0})
            d["n"] += 1
            d["wait"] += (int(r["t1"]) - int(r["t0"])) / 100.0  # us
            d["release"] += (int(r["t2"]) - int(r["t1"])) / 100.0
            d["copy"] += (int(r["t3"]) - int(r["t2"])) / 100.0
            d["post"] += (int(r["t4"]) - int(r["t3"])) / 100.0
            if int(r["tc"]):
                d["issue"] += (int(r["tc"]) - int(r["t2"])) / 100.0
                d["drain"] += (int(r["t3"]) - int(r["tc"])) / 100.0
            if i + 1 < len(rec):
                d["gap"] += (int(rec[i + 1]["t0"]) - int(r["t4"])) / 100.0
            d["bytes"] += int(r["bytes"])
    out = {}
    for k, d in rows.items():
        n = d["n"]
        out[k] = {"n": n, **{f: round(d[f] / n, 2) for f in ("wait", "release", "copy", "issue", "drain", "post",
                                                              "gap")},
                  "payload_GBs_in_copy": round(d["bytes"] / (d["copy"] * 1e3), 1) if d["copy"] else None}
    return out


def _net_row(dist, rank, world, S=256 << 20, steps=3, warmup=1):
    """North_star's staged rate, "including the copies to and from the GPU":
    config 3's fp32 all-reduce of an S-byte bucket on a fresh comm created
    with VCCL_NET_FORCE=1, so every ring connection moves through host-pinned
    staging slots and the TCP proxy pair (host/proxy.cc; the reference's net
    transport without GPUDirect, src/transport/net.cc:1293-1482) — on one rank
    per GPU each rank stages over its own host link.  busbw per rank, checked
    (DESIGN.md §4.6)."""
    old = os.environ.get("VCCL_NET_FORCE")
    os.environ["VCCL_NET_FORCE"] = "1"
    try:
        obj = [nccl.unique_id_to_bytes(nccl.get_unique_id()) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        c = _Tolerant(nccl.Comm.init_rank(world, nccl.unique_id_from_bytes(obj[0]), rank))
    finally:
        if old is None:
            os.environ.pop("VCCL_NET_FORCE", None)
        else:
            os.environ["VCCL_NET_FORCE"] = old
    sp = torch.cuda.current_stream().cuda_stream
    n = S // 4
    x = torch.rand(n, device="cuda")
    y = torch.empty_like(x)
    try:
        dt = _time_coll(dist, lambda: c.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32,
                                                   nccl.ncclSum, sp), steps, warmup)
        ok = check_ar(dist, c, rank, world, S)
        return {"bytes": n * 4, "channels": c.n_channels(), "us": round(dt / steps * 1e6, 1),
                "busbw": round(n * 4 * steps / dt / 1e9 * 2 * (world - 1) / world, 3), "correct": ok,
                "async_error": c.async_error(),
                "path": "VCCL_NET_FORCE=1: device -> pinned host slot -> TCP proxy -> pinned host -> device"}
    finally:
        c.destroy()
        del x, y


def _ring_trace_row(dist, rank, world, S, cap=1024):
    """The SIMPLE ring's slot timeline on the headline bucket (config 3, ring
    forced), both hand-offs, on a fresh comm created with VCCL_RING_TRACE:
    on one rank per GPU it shows whether a slot waits on credits (the link /
    the peer), on its copy or on the drain of its remote stores — what decides
    the channel model's headroom and the per-wave hand-off.  Two
    untimed calls, then one traced call per hand-off; per rank the span of
    the traced call and ring_trace_summary."""
    old = os.environ.get("VCCL_RING_TRACE")
    os.environ["VCCL_RING_TRACE"] = str(cap)
    try:
        obj = [nccl.unique_id_to_bytes(nccl.get_unique_id()) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        c = _Tolerant(nccl.Comm.init_rank(world, nccl.unique_id_from_bytes(obj[0]), rank))
    finally:
        if old is None:
            os.environ.pop("VCCL_RING_TRACE", None)
        else:
            os.environ["VCCL_RING_TRACE"] = old
    sp = torch.cuda.current_stream().cuda_stream
    n = S // 4
    x = torch.rand(n, device="cuda")
    y = torch.empty_like(x)
    out = {"bytes": n * 4, "channels": c.n_channels()}
    try:
        c.set_algo("ring")
        for wave in (False, True):
            c.set_ring_wave(wave)
            for _ in range(2):
                c.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum, sp)
            torch.cuda.synchronize()
            dist.barrier()
            c.ring_trace()  # clears
            dist.barrier()
            c.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, nccl.ncclSum, sp)
            torch.cuda.synchronize()
            tr = c.ring_trace()
            t0 = tr["t0"][tr["t0"] > 0]
            span = round((int(tr["t4"].max()) - int(t0.min())) / 100.0, 1) if t0.size else None
            res = [None] * world
            dist.all_gather_object(res, {"rank": rank, "span_us": span, "shapes": ring_trace_summary(tr)})
            out["per_wave" if wave else "workgroup"] = res
        out["async_error"] = c.async_error()
    finally:
        c.set_ring_wave(False)
        c.destroy()
    del x, y
    return out


BCAST_SIZES = (64 << 10, 8 << 20, 256 << 20)
CHANNELS_PER_RING = (2, 4, 8, 16, 32, 64)  # x rings, within the device limit of 128


def _channel_rows(dist, rank, world, S, steps, warmup=2):
    """Config 3 (S-byte fp32 ring all-reduce) on fresh communicators bounded
    to C ring channels (ncclConfig minCTAs = maxCTAs = C, graph/connect.cc:
    486-490), C = rings x {2 .. 64}: on one rank per GPU the row where busbw
    stops growing measures the headroom H the default channel model assumes
    (host/init.cc); ranks sharing a GPU are capped to their
    co-resident share (n_channels says what ran).  Each row's output is
    checked on the same comm (pattern inputs, every rank)."""
    rings = len(nccl.ring_orders(world))
    counts = sorted({min(128, rings * k) for k in CHANNELS_PER_RING})
    sp = torch.cuda.current_stream().cuda_stream
    n = S // 4
    x = torch.rand(n, device="cuda") * 2 - 1
    y = torch.empty_like(x)
    rows = []
    for C in counts:
        obj = [nccl.unique_id_to_bytes(nccl.get_unique_id()) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        cfg = nccl.ncclConfig_t.initializer(minCTAs=C, maxCTAs=C)
        c = _Tolerant(nccl.Comm.init_rank(world, nccl.unique_id_from_bytes(obj[0]), rank, config=cfg))
        try:
            c.set_algo("ring")
            dt = _time_coll(dist, lambda: c.all_reduce(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32,
                                                       nccl.ncclSum, sp), steps, warmup)
            c.set_algo(None)
            ok = check_ar(dist, c, rank, world, S, algo="ring")
            algbw = n * 4 * steps / dt / 1e9
            rows.append({"channels_asked": C, "n_channels": c.n_channels(), "bytes": n * 4,
                         "us": round(dt / steps * 1e6, 1),
                         "busbw": round(algbw * 2 * (world - 1) / world, 2), "correct": ok})
            # `ok` is already every rank's verdict; the error gate is a collective
            stop = ok is not True or _any_error(dist, c) != 0
        finally:
            c.destroy()
        if stop:
            rows[-1]["stopped"] = "error on this comm: the larger counts were skipped"
            break
    del x, y
    return rows


def _bcast_row(dist, comm, rank, world, S, root=0):
    """ncclBroadcast of S bytes (f32) from `root`: us per call and busbw
    (nccl-tests: busbw = algbw = S / t for broadcast); output checked."""
    sp = torch.cuda.current_stream().cuda_stream
    n = S // 4
    x = torch.empty(n, device="cuda")
    pattern_fill(x, root, world)
    y = x if rank == root else torch.full((n,), float("nan"), device="cuda")
    steps = 20 if S <= (8 << 20) else 5

    def call():
        comm.broadcast(x.data_ptr(), y.data_ptr(), n, nccl.ncclFloat32, root, sp)
    t = _time_coll(dist, call, steps, 2)
    ref = torch.empty(n, device="cuda")
    pattern_fill(ref, root, world)
    ok = bool(_all_ok(dist, torch.equal(y, ref)))
    del x, y, ref
    return {"bytes": S, "us": round(t / steps * 1e6, 2), "busbw": round(S / (t / steps) / 1e9, 3),
            "correct": ok, "algo": comm.coll_algo(3, S, nccl.ncclUint8)}


def _reduce_row(dist, comm, rank, world, S, root=None):
    """ncclReduce (f32 sum) of S bytes into `root` (default the last rank):
    us per call and busbw (nccl-tests: busbw = algbw = S / t for reduce);
    the root's output checked."""
    root = world - 1 if root is None else root
    sp = torch.cuda.current_stream().cuda_stream
    n = S // 4
    x = torch.empty(n, device="cuda")
    pattern_fill(x, rank, world)
    y = torch.full((n,), float("nan"), device="cuda") if rank == root else None
    steps = 20 if S <= (8 << 20) else 5

    def call():
        comm.reduce(x.data_ptr(), y.data_ptr() if y is not None else 0, n, nccl.ncclFloat32, nccl.ncclSum,
                    root, sp)
    t = _time_coll(dist, call, steps, 2)
    ok = bool(_all_ok(dist, pattern_ok(y, world) if y is not None else True))
    del x, y
    return {"bytes": S, "us": round(t / steps * 1e6, 2), "busbw": round(S / (t / steps) / 1e9, 3),
            "correct": ok, "algo": comm.coll_algo(4, n, nccl.ncclFloat32)}


def _rs_ag(dist, comm, rank, world, S, steps, warmup, dtype="bf16"):
    """Reduce-scatter of an S-byte bucket (n blocks) then all-gather of the
    shards back: busbw = (S / t) (n-1)/n each, and us per call."""
    sp = torch.cuda.current_stream().cuda_stream
    tdt, code = _TDT[dtype], _CODE[dtype]
    n = S // torch.tensor([], dtype=tdt).element_size()
    rc = n // world
    g = torch.Generator(device="cuda").manual_seed(2000 + rank)
    x = (torch.rand(n, device="cuda", generator=g) * 2 - 1).to(tdt)
    shard = torch.empty(rc, dtype=tdt, device="cuda")
    y = torch.empty_like(x)

    def rs():
        comm.reduce_scatter(x.data_ptr(), shard.data_ptr(), rc, code, nccl.ncclSum, sp)

    def ag():
        comm.all_gather(shard.data_ptr(), y.data_ptr(), rc, code, sp)
    t_rs = _time_coll(dist, rs, steps, warmup)
    t_ag = _time_coll(dist, ag, steps, warmup)
    frac = (world - 1) / world
    del x, y, shard
    torch.cuda.empty_cache()
    return {"bytes": S, "dtype": dtype, "steps": steps,
            "rs_busbw": round(S * steps / t_rs / 1e9 * frac, 2),
            "ag_busbw": round(S * steps / t_ag / 1e9 * frac, 2),
            "rs_us": round(t_rs / steps * 1e6, 2), "ag_us": round(t_ag / steps * 1e6, 2),
            "ms_per_rs_ag": round((t_rs + t_ag) / steps * 1e3, 3),
            "algo_rs": comm.coll_algo(1, rc, code), "algo_ag": comm.coll_algo(2, rc, code)}


def bench_rs_ag(args):
    """BASELINE config 4: reduce-scatter + all-gather bf16 bucket."""
    dist, rank, world, comm = _dist_setup()
    r = _rs_ag(dist, comm, rank, world, args.bytes or (4 << 30), args.steps, args.warmup)
    rs_ok, ag_ok = check_rs_ag(dist, comm, rank, world, args.bytes or (4 << 30))
    comm.destroy()
    dist.destroy_process_group()
    if rank:
        return None
    return {"metric": "reduce-scatter + all-gather busbw (BASELINE config 4)",
            "value": round((r["rs_busbw"] + r["ag_busbw"]) / 2, 2), "unit": "GB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": r["ms_per_rs_ag"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"workload": f"RS+AG bf16 {r['bytes']} B bucket, value = mean of the RS and AG "
                                   "busbw per rank", "rs_busbw": r["rs_busbw"],
                       "ag_busbw": r["ag_busbw"], "correct": {"rs": rs_ok, "ag": ag_ok}}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--bytes", type=int, default=0)
    ap.add_argument("--workload", default="")
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-peer", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--no-initall", action="store_true")
    ap.add_argument("--no-pmc-live", action="store_true")
    ap.add_argument("--rs-ag-bytes", type=int, default=4 << 30)
    ap.add_argument("--block", type=int, default=0)
    ap.add_argument("--unroll", type=int, default=0)
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--nt-loads", type=int, default=0)
    ap.add_argument("--nt-stores", type=int, default=0)
    ap.add_argument("--preroll-s", type=float, default=0.5)
    args = ap.parse_args()
    world, _ = world_check(sys.argv[1:], os.environ)
    workload = args.workload or ("reduce_copy" if world == 1 else "allreduce")
    if workload == "reduce_copy":
        out = bench_reduce_copy(args)
    elif workload == "allreduce":
        out = bench_allreduce(args)
    else:
        out = bench_rs_ag(args)
    if out is not None:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
