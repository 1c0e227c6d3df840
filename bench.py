"""bench.py -- headline benchmark of the MI355X backend for HPX's data-parallel
algorithm layer.

metric (BASELINE.json): achieved GB/s (% HBM peak) for triad/reduce/scan/sort
at 2^30, 1-8 MI355X.

One *step* = one pass of the hot path over 2^30 elements per GPU (weak
scaling; configs[1] of BASELINE.json plus the STREAM triad leg):
    STREAM triad      a = b + 3.0*c            2^30 doubles   24 B/elem
    transform_reduce  sum(x), init 0           2^30 int64      8 B/elem
    inclusive_scan    y = scan(x, plus, 0)     2^30 int64     16 B/elem
through the segmented algorithms over a partitioned_vector with one
partition per GPU (N = 1: the plain hip-executor algorithms; N > 1: segment
totals/carries exchanged with one RCCL all-gather of 8 B per GPU).
value = algorithmic bytes of all GPUs / max-over-ranks wall time of K steps.

Also reported (outside the timed region, rank 0): sort of 2^30 uint64 keys
(56 B/key executed by the hybrid path; 136 B/key for the 8-pass LSD), copy_if, f64 reduce/scan, the 1d_stencil heat
solver, the per-kernel HIP-event timings, the roofline of the dominant
kernel, and the HPX-par host baseline (oracle restatement) on a 2^27 sample.

Usage: python bench.py [--gpus N --steps K --warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...
`--gpus N` (N > 1) without torchrun starts the N ranks itself (launch_ranks);
a WORLD_SIZE that differs from --gpus is an error.  The JSON line carries
`ranks` (the communicator's size) and `rank_devices` (per rank: device
ordinal and PCI ids, all-gathered).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


class Events:
    """HIP events on the library's stream (torch.cuda.Event would only see
    torch's current stream)."""

    def __init__(self, L, count):
        self.L = L
        self.ev = []
        for _ in range(count):
            h = ctypes.c_void_p()
            L.call("hpxhip_event_create", ctypes.byref(h))
            self.ev.append(h)
        self.i = 0

    def record(self, stream):
        e = self.ev[self.i]
        self.i += 1
        self.L.call("hpxhip_event_record", e, stream)
        return e

    def ms(self, a, b):
        f = ctypes.c_float()
        self.L.call("hpxhip_event_elapsed_ms", a, b, ctypes.byref(f))
        return f.value


def max_over_ranks(comm, v: float) -> float:
    """Max of a host float over the ranks (one small all-gather)."""
    if comm.size == 1:
        return v
    g = comm.allgather_host(np.array([v], np.float64).view(np.int64))
    return float(np.asarray(g).view(np.float64).max())


def pct(gbs):
    return round(100.0 * gbs / HBM_PEAK_GBS, 2)


def launch_ranks(argv, n):
    """`bench.py --gpus N` (N > 1) without a torchrun environment: run the
    same command as N ranks under torch.distributed.run (one process per
    GPU, rendezvous on 127.0.0.1) and return its exit code.  This process
    stays a plain launcher: it never imports the HIP library or torch, so
    no GPU state exists in it (and nothing is exec'd over a GPU process).
    Rank 0 prints the one JSON line; a rank that fails or hangs past the
    collective timeout makes the whole launch exit non-zero."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    rc = subprocess.call(cmd, env=env)
    with open("/proc/self/maps") as f:
        if "libhpxhip" in f.read():
            print("bench.py launcher: the HIP library was loaded in the launcher process", file=sys.stderr)
            return rc or 3
    return rc


def launch_probe(args):
    """Hidden launcher check (no GPU): each rank joins a gloo group with the
    collective timeout and rank 0 prints one JSON line with every rank's
    RANK / LOCAL_RANK / WORLD_SIZE and pid."""
    import torch.distributed as dist
    from datetime import timedelta
    world = int(os.environ.get("WORLD_SIZE", "1"))
    mine = {k: int(os.environ.get(k, "0")) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    mine["pid"] = os.getpid()
    mine["hip_library_loaded"] = "libhpxhip" in open("/proc/self/maps").read()
    ranks = [mine]
    if world > 1:
        dist.init_process_group("gloo", timeout=timedelta(seconds=float(
            os.environ.get("HPXHIP_COLLECTIVE_TIMEOUT_S", "600"))))
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
        size = dist.get_world_size()
        dist.destroy_process_group()
    else:
        size = 1
    if mine["RANK"] == 0:
        print(json.dumps({"launch_probe": True, "n_gpus": args.gpus, "ranks": size, "rank_env": ranks}), flush=True)


def rank_devices(comm, tgt):
    """[[rank, device ordinal, PCI bus id, PCI device id], ...] of every rank,
    all-gathered, so the JSON line shows which GPUs the ranks ran on."""
    p = tgt.properties()
    mine = np.array([comm.rank, tgt.device, p["pci_bus_id"], p["pci_device_id"]], np.int64)
    if comm.size == 1:
        return [mine.tolist()]
    return np.asarray(comm.allgather_host(mine)).reshape(comm.size, -1).tolist()


def main(argv=None, comm_tgt=None):
    """argv: command line (default sys.argv); comm_tgt: an already built
    (communicator, target) pair -- the multi-rank test drives the N > 1 path
    through it on one GPU (tests/test_gpu_bench_ranks.py)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--logn", type=int, default=30)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--cpu-logn", type=int, default=27)
    ap.add_argument("--stencil-logn", type=int, default=32, help="1d_stencil points (total over the ranks)")
    ap.add_argument("--stencil-steps", type=int, default=100)
    ap.add_argument("--strong-logn", type=int, default=32,
                    help="segmented reduce / scan strong-scaling row: elements in total over the ranks")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic pass")
    ap.add_argument("--triad-only", action="store_true", help=argparse.SUPPRESS)  # PMC child mode
    # launcher check without a GPU: the ranks rendezvous over gloo and report
    # their environment (tests/test_bench_launcher.py)
    ap.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args(argv)
    if args.triad_only:
        return triad_only(args.logn)
    if comm_tgt is None:
        env_world = os.environ.get("WORLD_SIZE")
        if env_world is None and args.gpus > 1:
            # `bench.py --gpus N` outside torchrun: start the N ranks here,
            # before anything in this process touches the GPU
            sys.exit(launch_ranks(sys.argv[1:] if argv is None else list(argv), args.gpus))
        if env_world is not None and int(env_world) != args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}; refusing to report "
                     f"a {env_world}-rank run as {args.gpus} GPUs")
    if args.launch_probe:
        return launch_probe(args)

    import hpx_amd as hpx
    from hpx_amd import _lib as L
    from hpx_amd import execution as ex, functional as F, segmented as S

    comm, tgt = comm_tgt if comm_tgt is not None else S.init_distributed()
    rank, world = comm.rank, comm.size
    if comm_tgt is None and world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the communicator has {world} ranks")
    devices = rank_devices(comm, tgt)
    stream = tgt.stream
    pol = ex.par.on(hpx.default_executor(tgt))
    # The step runs under par(task), as an HPX program composes asynchronous
    # algorithms: each call returns a future and the work is ordered on the
    # target's stream, so no host round trip sits between the three kernels.
    # The reduce value is taken (get()) once the scan is enqueued; every step
    # still completes and is checked (scan-last == reduce) below.
    pol_task = ex.par(ex.task).on(hpx.default_executor(tgt))
    seg = S.algorithms

    n_local = 1 << args.logn
    n = n_local * world
    a = S.partitioned_vector(n, np.float64, comm=comm, tgt=tgt)
    b = S.partitioned_vector(n, np.float64, comm=comm, tgt=tgt)
    c = S.partitioned_vector(n, np.float64, comm=comm, tgt=tgt)
    x = S.partitioned_vector(n, np.int64, comm=comm, tgt=tgt)
    y = S.partitioned_vector(n, np.int64, comm=comm, tgt=tgt)
    seg.generate(pol, b.begin(), b.end(), "unit", 1)
    seg.generate(pol, c.begin(), c.end(), "unit", 2)
    seg.generate(pol, x.begin(), x.end(), "range", 0x5EED, -(1 << 20), 1 << 20)
    tgt.synchronize()

    triad = F.triad_step(3.0)
    ev = Events(L, 6 * (args.steps + args.warmup) + 8)
    marks = []

    def step(timed):
        e0 = ev.record(stream) if timed else None
        seg.transform_binary(pol_task, b.begin(), b.end(), c.begin(), a.begin(), triad)
        e1 = ev.record(stream) if timed else None
        fr = seg.reduce(pol_task, x.begin(), x.end(), 0, F.plus)
        e2 = ev.record(stream) if timed else None
        seg.inclusive_scan(pol_task, x.begin(), x.end(), y.begin(), F.plus, 0)
        e3 = ev.record(stream) if timed else None
        if timed:
            marks.append((e0, e1, e2, e3))
        return fr.get()

    for _ in range(args.warmup):
        step(False)
    tgt.synchronize()
    comm.barrier()
    tgt.synchronize()
    t0 = time.perf_counter()
    r = None
    for _ in range(args.steps):
        r = step(True)
    tgt.synchronize()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(comm, elapsed)

    # per-kernel HIP-event timings (segment-local kernels + their collectives)
    k_triad = np.mean([ev.ms(m[0], m[1]) for m in marks])
    k_reduce = np.mean([ev.ms(m[1], m[2]) for m in marks])
    k_scan = np.mean([ev.ms(m[2], m[3]) for m in marks])

    # cheap self-check: last inclusive-scan value == reduce result (int64 exact)
    if len(y.local) and rank == world - 1:
        last_local = y.local[len(y.local) - 1]
        assert last_local == r, f"scan/reduce mismatch {last_local} != {r}"
    from oracle import oracle as O  # checker only
    for i in [0, 1, n_local // 3, n_local - 1]:
        bb = O.generate(np.float64, "unit", 1, 1, offset=a.lo + i)[0]
        cc = O.generate(np.float64, "unit", 1, 2, offset=a.lo + i)[0]
        assert a.local[i] == bb + cc * 3.0, "triad parity"

    bytes_step = (24 + 8 + 16) * n_local
    value = world * bytes_step * args.steps / elapsed / 1e9
    ms_step = 1000.0 * elapsed / args.steps
    triad_gbs = 24 * n_local / (k_triad * 1e-3) / 1e9
    out = {
        "metric": "achieved GB/s (% HBM peak) for triad/reduce/scan/sort at 2^30, 1-8 MI355X",
        "value": round(value, 1),
        "unit": "GB/s",
        "n_gpus": world,
        "ranks": comm.size,
        "rank_devices": devices,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64+int64",
        "data": "synthetic (splitmix64 of the global index, seeded)",
        "config": {"workload": "STREAM triad (f64) + transform_reduce (int64) + inclusive_scan (int64) per step",
                   "elements_per_gpu": n_local, "global_elements": n, "partitioning": f"partitioned_vector x{world}",
                   "bytes_per_step_per_gpu": bytes_step, "pct_hbm_peak": pct(value / world)},
        "kernels_ms": {"triad": round(k_triad, 4), "transform_reduce": round(k_reduce, 4),
                       "inclusive_scan": round(k_scan, 4)},
        "kernels_gbs": {"triad": round(triad_gbs, 1),
                        "transform_reduce": round(8 * n_local / (k_reduce * 1e-3) / 1e9, 1),
                        "inclusive_scan": round(16 * n_local / (k_scan * 1e-3) / 1e9, 1)},
        "roofline": {"kernel": "triad (transform_binary f64)", "bound": "hbm", "achieved": round(triad_gbs, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(triad_gbs / HBM_PEAK_GBS, 4),
                     "traffic": None, "bytes_per_launch": 24 * n_local},
    }
    for v in (a, b, c):
        v.local.free()
    # HPXHIP_RCCL_SELF=1 (one rank through TorchComm under torchrun): the
    # N > 1 rows instead, as a rehearsal of the 8-GPU run on one GPU
    rehearse = world == 1 and os.environ.get("HPXHIP_RCCL_SELF") == "1"
    if not args.no_extras and world == 1 and not rehearse:
        out["extras"] = extras(hpx, L, ex, F, S, comm, tgt, pol, x, y, n_local, world, args)
    y.local.free()
    if not args.no_extras and (world > 1 or rehearse):
        out["extras"] = dist_extras(S, F, comm, tgt, pol, x, n_local, world, args)
    else:
        x.local.free()
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args.cpu_logn)
    if rank == 0 and world == 1 and not args.no_pmc:
        traffic, detail = pmc_traffic(args.logn)
        out["roofline"]["traffic"] = traffic
        out["roofline"]["traffic_detail"] = detail
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1 or rehearse:
        comm.barrier()
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def timed(L, tgt, fn, reps=3):
    """Best of `reps` HIP-event intervals on the target's stream around fn().
    A task-policy call returns its future once the work is enqueued, so the
    interval is the device time of the call; the future is taken after the
    stop event (a sync call's interval would also hold the host round trip
    that returns its result)."""
    ev = Events(L, 2 * reps + 2)
    _take(fn())
    tgt.synchronize()
    best = 1e30
    for _ in range(reps):
        e0 = ev.record(tgt.stream)
        r = fn()
        e1 = ev.record(tgt.stream)
        tgt.synchronize()
        _take(r)
        best = min(best, ev.ms(e0, e1))
    return best


def _take(r):
    from hpx_amd.future import future
    return r.get() if isinstance(r, future) else r


def extras(hpx, L, ex, F, S, comm, tgt, pol, x, y, n_local, world, args):
    from hpx_amd import parallel as P
    res = {}
    xv, yv = x.local, y.local
    n = n_local
    # timed as the step is: par(task), device events around the enqueue
    tpol = ex.par(ex.task).on(hpx.default_executor(tgt))
    ms = timed(L, tgt, lambda: P.copy_if(tpol, xv.begin(), xv.end(), yv.begin(), F.not_less_than(0)))
    hits = int(P.copy_if(tpol, xv.begin(), xv.end(), yv.begin(), F.not_less_than(0)).get()[1] - yv.begin())
    res["copy_if_int64"] = {"ms": round(ms, 4), "gbs_model_12B": round(12 * n / ms / 1e6, 1),
                            "pct_peak": pct(12 * n / ms / 1e6), "hits": hits,
                            "gbs_actual_bytes": round((8 * n + 8 * hits) / ms / 1e6, 1)}
    res["segmented_reduce_int64"] = seg_reduce_row(S, F, comm, tgt, pol, x)
    res["strong_2p32_int64"] = strong_row(S, F, comm, tgt, pol, args.strong_logn)
    res["double_reduce_scan"] = double_row(hpx, L, P, F, tgt, pol, tpol, n)
    res["stream_2p30"] = stream_row(hpx, L, P, F, tgt, pol, n)
    res["cxx_drop_in"] = cxx_drop_in_row(args, world)
    # sort of 2^30 uint64 keys (8 GiB + 8 GiB workspace)
    keys = hpx.vector(n, dtype=np.uint64, tgt=tgt)
    regen = lambda: P.generate(pol, keys.begin(), keys.end(), "bits", 7)  # noqa: E731
    ms_gen = timed(L, tgt, regen, reps=2)
    ms_sort = timed(L, tgt, lambda: (regen(), P.sort(pol, keys.begin(), keys.end())), reps=2) - ms_gen
    # executed traffic of the hybrid path random 64-bit keys take (sort.hip):
    # histogram 8 B + two onesweep prefix passes 2 x 16 B + the LDS segment
    # sort 16 B = 56 B/key; the 8-pass LSD it replaces moves 136 B/key
    res["sort_uint64"] = {"ms": round(ms_sort, 3), "gkeys_per_s": round(n / ms_sort / 1e6, 3),
                          "path": "hybrid: 2 x 9-bit prefix passes + LDS segment sort of ~4096-key buckets",
                          "gbs_executed_56B": round(56 * n / ms_sort / 1e6, 1),
                          "pct_peak": pct(56 * n / ms_sort / 1e6)}
    res["sort_uint64"].update(sort_check(P, F, pol, tgt, keys, regen))
    keys.free()
    # 32-bit keys: the hybrid (4 B/key histogram + two 8 B/key prefix passes +
    # 8 B/key segment sort = 28 B/key; the 4-pass LSD would move 36 B/key)
    k32 = hpx.vector(n, dtype=np.uint32, tgt=tgt)
    regen32 = lambda: P.generate(pol, k32.begin(), k32.end(), "bits", 11)  # noqa: E731
    ms_gen = timed(L, tgt, regen32, reps=2)
    ms32 = timed(L, tgt, lambda: (regen32(), P.sort(pol, k32.begin(), k32.end())), reps=2) - ms_gen
    res["sort_uint32"] = {"keys": n, "ms": round(ms32, 3), "gkeys_per_s": round(n / ms32 / 1e6, 3),
                          "path": "hybrid (18-bit prefix: two 9-bit passes + LDS segment sort)", "gbs_executed_28B": round(28 * n / ms32 / 1e6, 1),
                          "pct_peak": pct(28 * n / ms32 / 1e6)}
    k32.free()
    nkv = n // 4
    kk = hpx.vector(nkv, dtype=np.uint64, tgt=tgt)
    vv = hpx.vector(nkv, dtype=np.uint64, tgt=tgt)
    regenkv = lambda: (P.generate(pol, kk.begin(), kk.end(), "bits", 13),  # noqa: E731
                       P.generate(pol, vv.begin(), vv.end(), "bits", 17))
    ms_gen = timed(L, tgt, regenkv, reps=2)
    mskv = timed(L, tgt, lambda: (regenkv(), P.sort_by_key(pol, kk.begin(), kk.end(), vv.begin())), reps=2) - ms_gen
    ok = bool(P.is_sorted(pol, kk.begin(), kk.end()))
    # hybrid for pairs: histogram 8 B + two prefix passes over keys and
    # values 2 x 32 B + the LDS segment sort 32 B = 104 B/pair (the 8-pass
    # LSD moves 264)
    res["sort_by_key_u64_u64"] = {"pairs": nkv, "ms": round(mskv, 3), "gpairs_per_s": round(nkv / mskv / 1e6, 3),
                                  "path": "hybrid: 2 prefix passes + LDS segment sort (values staged beside keys)",
                                  "gbs_executed_104B": round(104 * nkv / mskv / 1e6, 1),
                                  "pct_peak": pct(104 * nkv / mskv / 1e6), "keys_sorted": ok}
    kk.free()
    vv.free()
    # 1d_stencil heat: 2^32 points, 100 steps (BASELINE.md plan), through the
    # partitioned solver -- the same row the N > 1 run reports
    res["stencil_heat_dist"] = stencil_row(S, comm, tgt, 1 << args.stencil_logn, args.stencil_steps)
    # host <-> device transfer (hpx/compute/cuda/transfer.hpp:188-348): 1 GiB,
    # pinned (hpxhip_malloc_host) and pageable host buffers
    nb = 1 << 30
    dbuf = hpx.vector(nb // 8, dtype=np.uint64, tgt=tgt)
    hp = ctypes.c_void_p()
    L.call("hpxhip_malloc_host", ctypes.byref(hp), nb)
    pageable = np.ones(nb // 8, np.uint64)
    xfer = {}
    for name, host in (("pinned", hp), ("pageable", pageable.ctypes.data_as(ctypes.c_void_p))):
        for kind, (dst, src) in (("h2d", (ctypes.c_void_p(dbuf.data()), host)),
                                 ("d2h", (host, ctypes.c_void_p(dbuf.data())))):
            k = L.H2D if kind == "h2d" else L.D2H
            ms = timed(L, tgt, lambda: L.call("hpxhip_memcpy_async", dst, src, nb, k, tgt.stream), reps=3)
            xfer[f"{kind}_{name}_gbs"] = round(nb / ms / 1e6, 1)
    L.call("hpxhip_free_host", hp)
    dbuf.free()
    res["host_device_copy_1GiB"] = xfer
    return res


def stream_row(hpx, L, P, F, tgt, pol, n, iterations=10, scalar=3.0):
    """BASELINE configs[0]: the whole STREAM benchmark (stream.cpp:294-375)
    through the hip executor at 2^30 doubles per array: fill, a *= 2, then
    `iterations` rounds of copy / scale / add / triad, each bracketed by HIP
    events on the target's stream; best and average of iterations 1.. (the
    first is skipped, :485-495), rates on the reference's byte model (:478-483:
    2, 2, 3, 3 x 8 B per element).  check_results (:82-133) on the device:
    min == max == the closed-form aj, bj, cj for each array."""
    a = hpx.vector(n, dtype=np.float64, value=1.0, tgt=tgt)
    b = hpx.vector(n, dtype=np.float64, value=2.0, tgt=tgt)
    c = hpx.vector(n, dtype=np.float64, value=0.0, tgt=tgt)
    P.transform(pol, a.begin(), a.end(), a.begin(), F.multiply_step(2.0))
    kernels = (("copy", 16, lambda: P.copy(pol, a.begin(), a.end(), c.begin())),
               ("scale", 16, lambda: P.transform(pol, c.begin(), c.end(), b.begin(), F.multiply_step(scalar))),
               ("add", 24, lambda: P.transform(pol, a.begin(), a.end(), b.begin(), b.end(), c.begin(), F.add_step())),
               ("triad", 24, lambda: P.transform(pol, b.begin(), b.end(), c.begin(), c.end(), a.begin(),
                                                 F.triad_step(scalar))))
    ev = Events(L, 8 * iterations + 2)
    marks = []
    for _ in range(iterations):
        row = []
        for _name, _b, fn in kernels:
            e0 = ev.record(tgt.stream)
            fn()
            row.append((e0, ev.record(tgt.stream)))
        marks.append(row)
    tgt.synchronize()
    from oracle import oracle as O  # checker only, after the timed kernels
    aj, bj, cj = O.stream_expected(iterations, scalar)
    ok = True
    for v, exp in ((a, aj), (b, bj), (c, cj)):
        lo = P.reduce(pol, v.begin(), v.end(), float("inf"), F.minimum)
        hi = P.reduce(pol, v.begin(), v.end(), float("-inf"), F.maximum)
        ok = ok and lo == exp and hi == exp
    for v in (a, b, c):
        v.free()
    out = {"elements": n, "iterations": iterations, "check_results": bool(ok)}
    for k, (name, nbytes, _fn) in enumerate(kernels):
        t = [ev.ms(*marks[i][k]) for i in range(1, iterations)]
        best = min(t)
        out[name] = {"best_gbs": round(nbytes * n / best / 1e6, 1), "pct_peak": pct(nbytes * n / best / 1e6),
                     "min_ms": round(best, 4), "avg_ms": round(sum(t) / len(t), 4), "max_ms": round(max(t), 4),
                     "bytes_per_elem": nbytes}
    return out


def double_row(hpx, L, P, F, tgt, pol, tpol, n):
    """configs[1]'s double leg: transform_reduce and inclusive_scan over 2^30
    doubles in [0, 1) (53-bit mantissas, so the sums round).  Check: the last
    inclusive value against the reduce within the FP-scan tolerance of
    DESIGN.md ((ntiles + 64) * u * value)."""
    xd = hpx.vector(n, dtype=np.float64, tgt=tgt)
    yd = hpx.vector(n, dtype=np.float64, tgt=tgt)
    P.generate(pol, xd.begin(), xd.end(), "unit", 3)
    ms_r = timed(L, tgt, lambda: P.reduce(tpol, xd.begin(), xd.end(), 0.0, F.plus))
    ms_s = timed(L, tgt, lambda: P.inclusive_scan(tpol, xd.begin(), xd.end(), yd.begin(), F.plus, 0.0))
    r = float(P.reduce(pol, xd.begin(), xd.end(), 0.0, F.plus))
    last = float(yd[n - 1])
    ntiles = -(-n // (1024 * 12 * 2))
    ok = abs(last - r) <= (ntiles + 64) * 2.0 ** -53 * abs(r) * 2
    xd.free()
    yd.free()
    return {"elements": n, "reduce_ms": round(ms_r, 4), "reduce_gbs": round(8 * n / ms_r / 1e6, 1),
            "reduce_pct_peak": pct(8 * n / ms_r / 1e6), "scan_ms": round(ms_s, 4),
            "scan_gbs": round(16 * n / ms_s / 1e6, 1), "scan_pct_peak": pct(16 * n / ms_s / 1e6),
            "sum": r, "scan_last_matches_reduce": bool(ok)}


def sort_check(P, F, pol, tgt, keys, regen):
    """Full-size check of the 2^30 sort, on the device: the sorted keys are
    a permutation of the generated ones (XOR and wrapping sum of all keys
    unchanged) and no adjacent pair is out of order (is_sorted)."""
    regen()
    xor0 = P.reduce(pol, keys.begin(), keys.end(), 0, F.bit_xor)
    sum0 = P.reduce(pol, keys.begin(), keys.end(), 0, F.plus)
    P.sort(pol, keys.begin(), keys.end())
    ok = bool(P.is_sorted(pol, keys.begin(), keys.end()))
    same = (P.reduce(pol, keys.begin(), keys.end(), 0, F.bit_xor) == xor0 and
            P.reduce(pol, keys.begin(), keys.end(), 0, F.plus) == sum0)
    return {"is_sorted_full": ok, "checksums_match": bool(same)}


def seg_reduce_row(S, F, comm, tgt, pol, x, reps=5):
    """Segmented transform_reduce of the int64 partitioned_vector x
    (segmented_algorithms/reduce.hpp:112-209): local kernel + one 8-B
    all-gather + device fold per call; max-over-ranks wall time of `reps`
    back-to-back calls between barriers."""
    import time
    n_local = len(x.local)
    S.algorithms.reduce(pol, x.begin(), x.end(), 0, F.plus)
    tgt.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = S.algorithms.reduce(pol, x.begin(), x.end(), 0, F.plus)
    tgt.synchronize()
    comm.barrier()
    el = max_over_ranks(comm, (time.perf_counter() - t0) / reps)
    per_rank = 8 * n_local / el / 1e9
    return {"elements_per_rank": n_local, "ranks": comm.size, "ms": round(1e3 * el, 4),
            "gbs_per_rank": round(per_rank, 1), "gbs_total": round(per_rank * comm.size, 1),
            "pct_peak_per_rank": pct(per_rank), "value": int(r)}


def strong_row(S, F, comm, tgt, pol, logn, reps=5):
    """Strong scaling of the segmented algorithms (2^32 int64 in
    total, the north star's >= 7x node-scaling target is stated on segmented
    reduce): one int64 partitioned_vector of 2^logn elements over the ranks,
    segmented reduce (segmented_algorithms/reduce.hpp:112-209) and segmented
    inclusive_scan (detail/scan.hpp:527-696), each `reps` back-to-back calls
    under the plain par policy (reduce returns its value: a host round trip
    per call) between barriers, max over ranks.  Bytes: 8 B/elem (reduce), 16
    B/elem at N = 1 and 24 at N > 1 (scan: the totals pass, the reference's
    step 1).  Check: the scan's last element == the reduce (int64 exact) on
    the last rank, max-over-ranks agreed."""
    import time
    n = 1 << logn
    x = S.partitioned_vector(n, np.int64, comm=comm, tgt=tgt)
    y = S.partitioned_vector(n, np.int64, comm=comm, tgt=tgt)
    S.algorithms.generate(pol, x.begin(), x.end(), "range", 0x5EED, -(1 << 20), 1 << 20)
    tgt.synchronize()

    def run(fn):
        fn()
        tgt.synchronize()
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            r = fn()
        tgt.synchronize()
        comm.barrier()
        return max_over_ranks(comm, (time.perf_counter() - t0) / reps), r

    t_red, total = run(lambda: S.algorithms.reduce(pol, x.begin(), x.end(), 0, F.plus))
    t_scan, _ = run(lambda: S.algorithms.inclusive_scan(pol, x.begin(), x.end(), y.begin(), F.plus, 0))
    ok = True
    if comm.rank == comm.size - 1 and len(y.local):
        ok = int(y.local[len(y.local) - 1]) == int(total)
    ok = bool(max_over_ranks(comm, 0.0 if ok else 1.0) == 0.0)
    x.local.free()
    y.local.free()
    scan_b = 16 if comm.size == 1 else 24
    return {"elements_total": n, "elements_per_rank": n // comm.size, "ranks": comm.size, "scaling": "strong",
            "reduce_ms": round(1e3 * t_red, 4), "reduce_gbs_total": round(8 * n / t_red / 1e9, 1),
            "reduce_pct_peak_per_rank": pct(8 * n / t_red / 1e9 / comm.size),
            "scan_ms": round(1e3 * t_scan, 4), "scan_bytes_per_elem": scan_b,
            "scan_gbs_total": round(scan_b * n / t_scan / 1e9, 1),
            "scan_pct_peak_per_rank": pct(scan_b * n / t_scan / 1e9 / comm.size),
            "reduce_elements_per_s": round(n / t_red, 1), "scan_elements_per_s": round(n / t_scan, 1),
            "scan_last_equals_reduce": ok}


STENCIL_SEED = 0xC0FFEE


def stencil_windows(nx, nt):
    """Checked ranges [lo, lo + count) of the stencil row: the periodic seam
    (0 and nx - 1), 2^31 +- nt points, 2^28 / 2^29 points (2^31 / 2^32 bytes),
    2^32 - 1 and seeded random positions (tests/test_gpu_stencil_fullsize.py)."""
    w = [(0, 64), (nx - 64, 64), ((1 << 31) - nt - 32, 2 * nt + 64), ((1 << 28) - 32, 64), ((1 << 29) - 32, 64),
         (nx // 2 + 1000, 64), (nx - 1, 1)]
    w += [(int(s), 96) for s in np.random.default_rng(7).integers(0, max(1, nx - 96), 4)]
    return [(lo, c) for lo, c in w if 0 <= lo and lo + c <= nx]


def stencil_row(S, comm, tgt, nx, nt):
    """examples/1d_stencil heat over the ranks (strong scaling: nx points in
    total), partitioned solver with temporal blocking and the halo ring;
    max-over-ranks wall time of nt steps (after nt untimed warm-up steps).  Initial state: U0[i] =
    splitmix64(seed ^ i) in [0, 1), generated on the device (no steady
    state: every wrong neighbour, skipped step or index wrap shows).  Check:
    sampled windows bit for bit against the serial oracle run on +-nt
    points around each window (after nt steps point i depends only on
    U0[i-nt .. i+nt]); each rank checks the windows inside its partition."""
    import time
    from hpx_amd import _lib as L
    from oracle import oracle as O  # checker only, after the timed region
    hs = S.heat_solver(nx, comm, tgt, init=("unit", STENCIL_SEED))
    hs.do_work(nt)   # warm-up: first launches, first touch of the second buffer
    hs.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    hs.do_work(nt)
    hs.synchronize()
    comm.barrier()
    el = max_over_ranks(comm, time.perf_counter() - t0)
    cur = hs.current
    ok, checked = True, 0
    for lo, c in stencil_windows(nx, 2 * nt):
        if lo < hs.lo or lo + c > hs.hi:
            continue
        win = np.empty(c, np.float64)
        L.call("hpxhip_memcpy_async", win.ctypes.data_as(ctypes.c_void_p),
               ctypes.c_void_p(cur.data() + 8 * (lo - hs.lo)), 8 * c, L.D2H, tgt.stream)
        tgt.synchronize()
        ok = ok and bool(np.array_equal(win, O.stencil_window(nx, 2 * nt, STENCIL_SEED, lo, c)))
        checked += c
    ok = bool(max_over_ranks(comm, 0.0 if ok else 1.0) == 0.0)
    for v in hs.U + [hs.H]:
        v.free()
    # executed HBM traffic: one 16-B/point read + write per fused pass of
    # halo_width steps (the unfused per-step model, 16 B per point-step, is
    # not a roofline: the fused passes never move those bytes)
    passes = -(-nt // max(1, hs.W))
    return {"points": nx, "ranks": comm.size, "steps": nt, "ms": round(1e3 * el, 3),
            "gpoint_steps_per_s": round(nx * nt / el / 1e9, 2),
            "gbs_executed_16B_per_pass": round(16 * nx * passes / el / 1e9, 1),
            "init": "splitmix64(seed ^ i) in [0, 1)", "window_check_bit_exact": ok, "steps_checked": 2 * nt,
            "points_checked_rank0": checked, "halo_width": hs.W}


def dist_extras(S, F, comm, tgt, pol, x, n_local, world, args):
    """Multi-GPU rows of SURVEY.md section 8(e) (all ranks, max-over-ranks
    wall time between barriers):
      * segmented reduce of the step's int64 partitioned_vector (GB/s per
        rank and in total);
      * strong scaling of segmented reduce and inclusive_scan over 2^32 int64
        in total (strong_row);
      * segmented sort of 2^logn uint64 keys per GPU (weak scaling): local
        radix sort, exact global cut, one RCCL all-to-all, then the received
        runs merged (hpxhip_merge_runs in one pass for 4 <= p <= 8, pairwise
        merge-path rounds otherwise);
        checked on the device: every partition sorted (is_sorted) and the
        partitions ordered across ranks (first/last keys all-gathered);
      * 1d_stencil heat, 2^32 points over the ranks, 100 steps (strong
        scaling), halo ring over RCCL send/recv overlapped with the interior;
      * the C++ drop-in (cxx_drop_in_row): partitioned_vector over every
        local GPU from one process, run by rank 0."""
    import time
    from hpx_amd import parallel as P
    res = {"segmented_reduce_int64": seg_reduce_row(S, F, comm, tgt, pol, x)}

    def tmax(v):
        return max_over_ranks(comm, v)

    n = n_local * world
    x.local.free()
    res["strong_2p32_int64"] = strong_row(S, F, comm, tgt, pol, args.strong_logn)
    keys = S.partitioned_vector(n, np.uint64, comm=comm, tgt=tgt)
    best = None
    for rep in range(3):
        S.algorithms.generate(pol, keys.begin(), keys.end(), "bits", 7 + rep)
        tgt.synchronize()
        comm.barrier()
        t0 = time.perf_counter()
        S.algorithms.sort(pol, keys.begin(), keys.end())
        tgt.synchronize()
        comm.barrier()
        el = tmax(time.perf_counter() - t0)
        best = el if best is None else min(best, el)
    loc = keys.local
    m = len(loc)
    ok = bool(P.is_sorted(pol, loc.begin(), loc.end())) if m else True
    ends = np.array([loc[0], loc[m - 1]] if m else [0, 0], np.uint64).view(np.int64)
    g = comm.allgather_host(ends).view(np.uint64)
    ok = ok and all(g[r, 1] <= g[r + 1, 0] for r in range(world - 1))
    ok = bool(tmax(0.0 if ok else 1.0) == 0.0)
    res["segmented_sort_uint64"] = {"keys_per_gpu": n_local, "keys_total": n, "ms": round(1e3 * best, 3),
                                    "gkeys_per_s": round(n / best / 1e9, 3), "sorted_and_ordered": ok}
    loc.free()
    res["stencil_heat_dist"] = stencil_row(S, comm, tgt, 1 << args.stencil_logn, args.stencil_steps)
    # the C++ drop-in over every local GPU, run by rank 0 while the others wait
    tgt.synchronize()
    comm.barrier()
    if comm.rank == 0:
        res["cxx_drop_in"] = cxx_drop_in_row(args, world)
    comm.barrier()
    return res


def triad_only(logn):
    """PMC child: the dominant kernel alone (3 launches over 2^logn doubles)."""
    import hpx_amd as hpx
    from hpx_amd import execution as ex, functional as F, parallel as P
    t = hpx.target(0)
    pol = ex.par.on(hpx.default_executor(t))
    n = 1 << logn
    a, b, c = (hpx.vector(n, dtype=np.float64, tgt=t) for _ in range(3))
    P.generate(pol, b.begin(), b.end(), "unit", 1)
    P.generate(pol, c.begin(), c.end(), "unit", 2)
    for _ in range(3):
        P.transform(pol, b.begin(), b.end(), c.begin(), c.end(), a.begin(), F.triad_step(3.0))
    t.synchronize()


def pmc_traffic(logn):
    """HBM bytes per triad launch from rocprofv3 PMC counters, collected as
    MI355X_MICROARCH.md's HBM/rocprofv3 section prescribes: FETCH_SIZE and
    WRITE_SIZE in separate passes (TCC slots), kilobytes -> bytes, and
    FETCH_SIZE doubled (gfx950 tallies 128-B streaming reads at 64 B)."""
    import csv
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        return None, {"error": "rocprofv3 not found"}
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="hpxhip_pmc_", dir="/tmp")
        cmd = [exe, "--pmc", counter, "-d", d, "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__), "--triad-only", "--logn", str(logn)]
        try:
            subprocess.run(cmd, check=True, capture_output=True, timeout=300, cwd="/tmp",
                           env=dict(os.environ, TMPDIR="/tmp"))
        except Exception as e:  # noqa: BLE001 -- report, never fake a number
            return None, {"error": f"{counter}: {type(e).__name__}"}
        per = []
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    for row in csv.DictReader(open(os.path.join(root, f))):
                        if "k_binary" in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                            per.append(float(row["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if not per:
            return None, {"error": f"{counter}: no k_binary rows"}
        vals[counter] = sum(per) / len(per)
    fetch = 2.0 * vals["FETCH_SIZE"] * 1024.0
    write = vals["WRITE_SIZE"] * 1024.0
    return round(fetch + write), {"FETCH_SIZE_kb_raw": vals["FETCH_SIZE"], "WRITE_SIZE_kb": vals["WRITE_SIZE"],
                                  "read_bytes_corrected": round(fetch), "write_bytes": round(write),
                                  "algorithmic_bytes": 24 * (1 << logn)}


def cxx_drop_in_row(args, world):
    """The C++ drop-in path as an HPX program calls it (tests/cxx/bench_targets.hip,
    VERDICT r05 item 7): partitioned_vector over hip::target_layout(targets),
    the step (triad + reduce + inclusive_scan under par(task)) and the
    heat_solver ring, through include/hpx and the C ABI in a process of its
    own.  One GPU: 4 targets on device 0 of 2^(logn-2) elements each (the
    step's 2^logn in total; every cross-target hand-off runs, without peer
    copies); N GPUs (rank 0, the other ranks idle at a barrier): one target
    per local GPU, 2^logn each, peer copies included.  Returns the program's
    JSON row, or an error entry (never a made-up number)."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "cxx", "bin", "bench_targets")
    if not os.path.exists(exe):
        return {"error": "tests/cxx/bin/bench_targets not built (make cxxtests)"}
    if world == 1:
        cmd = [exe, "--targets", "4", "--logn", str(args.logn - 2), "--heat-logn", "26"]
    else:
        cmd = [exe, "--logn", str(args.logn), "--heat-logn", "28"]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    except Exception as e:  # noqa: BLE001 -- report, never fake a number
        return {"error": f"{type(e).__name__}"}
    for line in out.stdout.splitlines():
        if line.startswith("{\"cxx_drop_in\""):
            row = json.loads(line)["cxx_drop_in"]
            row["command"] = " ".join(["tests/cxx/bin/bench_targets"] + cmd[1:])
            return row
    return {"error": f"rc={out.returncode}", "stderr_tail": out.stderr[-400:]}


def cpu_baseline(logn):
    """HPX-par restatement (oracle) of the same step on the host cores, on a
    2^logn sample: triad + reduce + inclusive scan; plus the extras' host
    rows: copy_if on the same sample, sort of 2^(logn-2)
    uint64 keys (sort.hpp:78-229 restated: parallel quicksort, std::sort
    leaves) and the 1d_stencil heat solver (1d_stencil_4_parallel.cpp:87-156
    restated) on 2^(logn-3) points x 20 steps."""
    from oracle import oracle as O
    # cores this process may run on (affinity, not the machine's count), the
    # threads used (OMP_NUM_THREADS caps them: 16 on the GPU box), the model
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or affinity
    threads = max(1, min(threads, affinity))
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    n = 1 << logn
    t_triad = O.par_triad(n, threads, reps=3)
    x = O.generate(np.int64, "range", n, 0x5EED, -(1 << 20), 1 << 20)
    t_red, _ = O.par_reduce_i64(x, threads, reps=3)
    t_scan, _ = O.par_scan_i64(x, threads, reps=3)
    gbs = (24 + 8 + 16) * n / (t_triad + t_red + t_scan) / 1e9
    t_cif, _ = O.par_copy_if_i64(x, threads, reps=2)
    del x
    ns = 1 << max(10, logn - 2)
    keys = O.generate(np.uint64, "bits", ns, 7)
    t_sort, _ = O.par_sort_u64(keys, threads)
    del keys
    nx, nt = 1 << max(10, logn - 3), 20
    t_st, _ = O.par_stencil(np.arange(nx, dtype=np.float64), nt, threads)
    # configs[0] itself: the STREAM benchmark at 2^27 doubles on host par
    st, abc = O.par_stream(n, threads, 3.0, 10)
    stream = {"elements": n, "iterations": 10,
              "check_results": bool(tuple(abc) == tuple(O.stream_expected(10, 3.0)))}
    for name, nbytes in (("copy", 16), ("scale", 16), ("add", 24), ("triad", 24)):
        best, avg = st[name]
        stream[name] = {"best_gbs": round(nbytes * n / best / 1e9, 2), "min_ms": round(1e3 * best, 3),
                        "avg_ms": round(1e3 * avg, 3)}
    return {"value": round(gbs, 2), "unit": "GB/s", "cores": threads, "kind": "port",
            "cpu_model": model, "affinity_cpus": affinity, "machine_cpus": os.cpu_count(),
            "sample": f"2^{logn} elements: triad f64 + reduce int64 + inclusive_scan int64, best of 3, "
                      f"HPX par chunking (4*cores chunks) on {threads} std::threads",
            "triad_gbs": round(24 * n / t_triad / 1e9, 2), "reduce_gbs": round(8 * n / t_red / 1e9, 2),
            "scan_gbs": round(16 * n / t_scan / 1e9, 2),
            "extras": {"copy_if_int64": {"elements": n, "ms": round(1e3 * t_cif, 2),
                                         "gbs_model_12B": round(12 * n / t_cif / 1e9, 2)},
                       "sort_uint64": {"keys": ns, "ms": round(1e3 * t_sort, 2),
                                       "gkeys_per_s": round(ns / t_sort / 1e9, 4)},
                       "stencil_heat": {"points": nx, "steps": nt, "ms": round(1e3 * t_st, 2),
                                        "gpoint_steps_per_s": round(nx * nt / t_st / 1e9, 3),
                                        "gbs_model_16B": round(16 * nx * nt / t_st / 1e9, 2)},
                       "stream": stream}}


if __name__ == "__main__":
    main()
