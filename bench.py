#!/usr/bin/env python3
"""Headline benchmark: GB/s of gradient buckets reduced, device-resident.

  python bench.py [--gpus N] [--steps K] [--warmup W]

N = 1 (default): config C2 of BASELINE.json — one MI355X sums 8 staged 64 MiB fp32
buckets into one output with the hand-written HIP tree kernel (esgd_reduce).
N > 1 (one rank per GPU): solo-allreduce of one 256 MiB fp32 bucket per rank (config C3)
through the esgd data plane.  Under torch.distributed.run (WORLD_SIZE set) each process
is one rank; a bare `python bench.py --gpus N` starts its own N ranks the same way (a
fresh `python -m torch.distributed.run` child, before this process touches HIP) and
exits with their status -- rank 0 prints the line.

value = bucket bytes reduced per second over the whole job = (#contributing buckets
x bucket bytes) / wall time of the K timed steps (max over ranks), inputs resident in
HBM before the timed region.  roofline = the dominant kernel's algorithmic bytes per
launch / its average launch time from HIP events on its own stream.  cpu_baseline =
the oracle's restatement of fflib2's recursive doubling (oracle/ffref.c) timed on
this host's cores for the same workload shape (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "eager-sgd_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
XGMI_LINK_GBS = 153.0      # per-link figure used by SURVEY.md §8d
SHARED_GPU = False         # N > 1 with ranks sharing a device (set in run_allreduce)
SEED = 0x5EEDE56D
MiB = 1 << 20
_LINE_FD = None            # N > 1: the rank's real stdout, kept for the JSON line alone


def _quiet_stdout():
    """Under a launcher every rank shares the job's stdout, and native libraries write
    to fd 1 (gloo's "[Gloo] Rank r is connected to ..." at init, RCCL/HIP notices).
    Point fd 1 at stderr for the whole run and keep a private copy of the real stdout,
    so the only thing a rank ever writes there is rank 0's JSON line."""
    global _LINE_FD
    sys.stdout.flush()
    _LINE_FD = os.dup(1)
    os.dup2(2, 1)


def emit(line: dict) -> None:
    """Print the one JSON line (to the real stdout when _quiet_stdout ran)."""
    text = json.dumps(line) + "\n"
    if _LINE_FD is None:
        sys.stdout.write(text)
        sys.stdout.flush()
    else:
        os.write(_LINE_FD, text.encode())


LEGS_HELP = """N > 1 extra legs (after the C3 headline, under a watchdog; ESGD_BENCH_LEGS=a,b picks a
subset in that order): sweep_c5_majority, sweep_c5_majority_bf16, ab_one_launch_threshold,
c3_wire_bf16, c1_host_majority, small_round_after_idle, straggler_c4_majority,
c4_resnet50_161_vs_fused, optimizer_resnet50_161, c3_host_buckets, c3_rccl_transport,
rccl_as_default_c3_c4, ab_flag_pages.  rccl_as_default_c3_c4 is the one-shot head-to-head of
the north star's named data plane: RCCL P2P (grouped ncclSend/ncclRecv + the tree kernel on
a side stream) set as the transport of C3 (solo, 256 MiB per GPU) and C4 (majority, the
ResNet-50 fused gradient, one rank 0.2 T late), against the IPC-pull numbers of the same job
(the headline and straggler_c4_majority).  It needs one GPU per rank: with ranks sharing a
GPU (a 1-GPU rehearsal) it is skipped and says why.  ESGD_BENCH_RCCL=0 skips both RCCL legs."""


def parse():
    ap = argparse.ArgumentParser(epilog=LEGS_HELP, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--buckets", type=int, default=8, help="N=1: staged buckets (fan-in k)")
    ap.add_argument("--bucket-mib", type=float, default=None,
                    help="bucket size (default 64 at N=1, 256 at N>1)")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--schedule", choices=["solo", "majority", "allreduce"], default="solo")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic pass")
    ap.add_argument("--no-gate", action="store_true", help="skip the 8 x 256 MiB gate shape")
    ap.add_argument("--no-extras", action="store_true",
                    help="N>1: skip the C5 size sweep and the C4 straggler case")
    ap.add_argument("--transport", choices=["ipc", "rccl"], default=None,
                    help="N>1 data plane (default: ESGD_TRANSPORT or ipc)")
    ap.add_argument("--pmc-child", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--no-trace", action="store_true",
                    help="N=1: skip the rocprofv3 kernel-trace pass behind roofline.rocprof_kernel_us")
    return ap.parse_args()


def launch_ranks(args) -> int:
    """`bench.py --gpus N` without a launcher: start N ranks as torch.distributed.run
    would (the reference's launcher starts its ranks the same way,
    test_scripts_imagenet/daint_eagersgd_imagenet.sh:2-5).  Called before anything in
    this process touches HIP; the ranks inherit stdout, so rank 0's JSON line is the
    output, and this process exits with the launcher's status."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC (RCCL / peer buckets)
    env["ESGD_BENCH_SELF_LAUNCHED"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def run_labels(world: int, devs, transport: str) -> dict:
    """config.parallelism and config.transport from the devices the ranks actually used
    (VERDICT r05 item 5): ranks sharing one GPU are a rehearsal, whose bytes never cross xGMI."""
    n = len(set(devs))
    if n == 1 and world > 1:
        par, where = f"dp{world} ({world} ranks on one GPU: rehearsal)", "in one GPU's HBM"
    elif n < world:
        par, where = f"dp{world} ({world} ranks on {n} GPUs, shared)", "over xGMI and within shared GPUs' HBM"
    else:
        par, where = f"dp{world} (one rank per GPU)", "over xGMI"
    if transport == "rccl":
        return {"parallelism": par, "transport": "rccl p2p send/recv + tree kernel on a side stream"}
    return {"parallelism": par, "transport": "ipc pull (reduce-scatter tree kernel + all-gather) " + where}


def _baseline_cpus(P: int):
    """2P cores for the CPU baseline's P simulated ranks: the first 2P physical cores of this
    process's affinity set in id order (one thread of each SMT pair; rank r on the (2r,
    2r + 1)-th), so neighbouring ranks share an L3 as an MPI job's packed placement does.
    (Spreading the ranks one L3 domain each -- `--map-by l3cache` -- was slower for both
    baselines on the 9575F boxes: 4.2 against 6.1-9.0 GB/s, and C1 2.7 against 6.0-6.8, the
    ranks' exchanges then crossing CCDs; r06l.)  None when fewer than 2P exist."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None
    cores, seen = [], set()
    for c in allowed:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                sib = f.read().strip()
        except OSError:
            sib = str(c)
        if sib in seen:   # an SMT sibling of a core already taken
            continue
        seen.add(sib)
        cores.append(c)
    return cores[:2 * P] if len(cores) >= 2 * P else None


def _pinned_samples(P: int, count: int, reps: int, samples: int = 3):
    """`samples` runs of the pinned C1-shaped harness (each a median step over `reps`):
    (median, [each], cores, every result correct)."""
    from oracle import ffref
    cpus = _baseline_cpus(P)
    ts, good = [], True
    for _ in range(samples):
        t, ok = ffref.time_c1(P, count, reps, cpus)
        ts.append(t)
        good = good and ok
    return statistics.median(ts), ts, cpus, good


def cpu_baseline(k: int, count: int):
    """fflib2 restated (oracle/ffref.c) on this host for the same k x bucket workload, with
    the core budget SURVEY.md §8(d) gives the reference: 2 cores per rank -- each simulated
    rank a main thread (the wrapper's copy-in, post, spin-wait, copy-out, zeroing of the
    send bucket) and a progress thread (the move + recursive doubling with VSUM; ff.c:72's
    pthread), 2k threads in all, each pinned to a physical core of its own (_baseline_cpus).
    DRAM-bound on a shared host: within a box the 3 samples agree to 1-5 %, across boxes the
    same placement gave 6.11 and 9.03 GB/s (r06d, r06k; unpinned in round 5: 6.35 and 10.59).  The value is the median of 3
    samples; the spread is beside it.  Also reported: the recursive doubling alone, one
    pthread per rank (the round-4 figure, unpinned)."""
    from oracle import ffref
    t1, _ = ffref.time_c1(k, count, 2, _baseline_cpus(k))   # warm + size the sample
    reps = max(3, min(250, int(4.0 / max(t1, 1e-3))))           # ~4 s of CPU work per sample
    t, ts, cpus, ok = _pinned_samples(k, count, reps)
    t_rd1 = ffref.time_allreduce(k, count, k, max(1, reps // 2))
    gbs = [k * count * 4 / x / 1e9 for x in ts]
    return {"value": round(k * count * 4 / t / 1e9, 3), "unit": "GB/s", "cores": 2 * k, "kind": "port",
            "sample": f"full workload: {k} ranks x {count * 4 / MiB:.0f} MiB fp32, each a main thread (copy-in, "
                      f"post, wait, copy-out, zero) + a progress thread (move + recursive doubling, VSUM) = "
                      f"{2 * k} threads pinned one per physical core (oracle/ffref.c ffref_time_c1_pinned), "
                      f"median of 3 "
                      f"samples, each the median step of {reps}: {t * 1e3:.1f} ms",
            "samples_GBs": [round(x, 3) for x in gbs],
            "spread": round((max(gbs) - min(gbs)) / statistics.median(gbs), 3),
            "core_list": cpus, "correct": ok,
            "recursive_doubling_only_1_thread_per_rank": {
                "value": round(k * count * 4 / t_rd1 / 1e9, 3), "cores": k,
                "sample": f"{k}-rank recursive doubling alone (1 pthread/rank, unpinned), best of "
                          f"{max(1, reps // 2)}: {t_rd1 * 1e3:.1f} ms"},
            "host_cpus": os.cpu_count(), "cpu_model": _cpu_model()}


def cpu_baseline_c1(P: int = 2, count: int = 262144):
    """BASELINE.json configs[0] (C1): P ranks reducing one 1 MiB fp32 bucket per step the
    way the wrapper drives fflib2 -- each rank a main thread (copy-in, post, spin-wait,
    copy-out, zero) and a progress thread (move + recursive doubling, ff.c:72), i.e. 2
    cores per rank, each thread pinned to a physical core of its own
    (_baseline_cpus; 6.03 and 6.80 GB/s on two boxes, r06d / r06k); value = P x
    bucket bytes per step / step time, the median of 3 samples."""
    from oracle import ffref
    t1, _ = ffref.time_c1(P, count, 20, _baseline_cpus(P))
    reps = max(50, min(20000, int(4.0 / max(t1, 1e-5))))   # ~4 s of steps per sample
    t, ts, cpus, ok = _pinned_samples(P, count, reps)
    gbs = [P * count * 4 / x / 1e9 for x in ts]
    return {"value": round(P * count * 4 / t / 1e9, 3), "unit": "GB/s", "cores": 2 * P, "kind": "port",
            "sample": f"C1: {P} ranks x {count * 4 / MiB:g} MiB fp32, main + progress thread per rank, each "
                      f"pinned to a core (oracle/ffref.c ffref_time_c1_pinned), median of 3 samples, each the "
                      f"median step of {reps}: {t * 1e6:.1f} us",
            "samples_GBs": [round(x, 3) for x in gbs],
            "spread": round((max(gbs) - min(gbs)) / statistics.median(gbs), 3),
            "core_list": cpus, "correct": ok, "host_cpus": os.cpu_count(), "cpu_model": _cpu_model()}


PMC_CALLS = 5   # reduction calls of the PMC child run


def _under_profiler():
    """True when this process runs under rocprofv3 (it configures its tool library
    through ROCPROF* variables)."""
    return any(k.startswith("ROCPROF") for k in os.environ)


def pmc_traffic(args, mib):
    """HBM bytes per reduction call (k buckets of `mib` MiB) from rocprofv3 PMC counters,
    in separate passes (FETCH_SIZE, WRITE_SIZE), corrected as MI355X_MICROARCH.md §HBM
    prescribes: gfx950 FETCH_SIZE counts half the bytes of a wide streaming read.  A call
    over buckets larger than the kernel's 64 MiB window is several dispatches: their
    counters are summed and divided by the child's PMC_CALLS calls."""
    import shutil
    out = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(ROOT, "gpurun_out", f"bench_pmc_{ctr}_{mib:g}MiB")
        shutil.rmtree(d, ignore_errors=True)
        os.makedirs(d, exist_ok=True)
        cmd = ["rocprofv3", "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", "1",
               "--buckets", str(args.buckets), "--bucket-mib", str(mib),
               "--dtype", args.dtype]
        subprocess.run(cmd, check=True, timeout=240, stdout=subprocess.DEVNULL,
                       stderr=subprocess.DEVNULL, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"))
        vals = []
        for dp, _, files in os.walk(d):
            for fn in files:
                if fn.endswith("counter_collection.csv"):
                    import csv
                    with open(os.path.join(dp, fn)) as f:
                        for row in csv.DictReader(f):
                            if "k_tree_sum" in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                                vals.append(float(row["Counter_Value"]))
        if not vals:
            return None
        out[ctr] = sum(vals) / PMC_CALLS   # KiB per call
    # FETCH_SIZE/WRITE_SIZE are in KiB; FETCH_SIZE x2 on gfx950 for 16-B streaming loads
    return 2 * out["FETCH_SIZE"] * 1024 + out["WRITE_SIZE"] * 1024


TRACE_WARM, TRACE_C2, TRACE_GATE = 3, 40, 20   # calls of the kernel-trace child run
TREE_KERNEL = "k_tree_sum_buf<esgd::F32, 8, 4, 2, 16, false"   # the production fp32 fan-in-8 kernel
GATE_WINDOWS = 4                                # 256 MiB / kWindowBytes (reduce_core.h)


def trace_child(dev, dt, ptrs, out, count, k, s):
    """The kernel-trace child (rocprofv3 --kernel-trace runs it), in the order the line is
    measured: the gate's 8 x 256 MiB calls, then the C2 launches, each group after its own
    warm-up; one small fill kernel between the groups marks the boundary in the trace."""
    gcount = (256 * MiB) // 4
    gb = [dev.DeviceBuffer(gcount, dt) for _ in range(k)]
    for r, b in enumerate(gb):
        dev.fill_uniform(b, SEED, r, stream=s)
    go = dev.DeviceBuffer(gcount, dt)
    for _ in range(TRACE_WARM + TRACE_GATE):
        dev.reduce(dt, [b.ptr for b in gb], go, gcount, stream=s)
    mark = dev.DeviceBuffer(1024, dt)
    dev.fill_uniform(mark, SEED, 0, stream=s)
    for _ in range(TRACE_WARM + TRACE_C2):
        dev.reduce(dt, ptrs, out, count, stream=s)
    s.synchronize()


def kernel_trace(args):
    """The dominant kernel's dispatch durations on THIS box: a rocprofv3 --kernel-trace
    child pass (the program right after `--`) over the same C2 launches and gate calls
    the line is timed on.  Returns (C2 average dispatch us, gate average call us = the
    sum of its 4 window dispatches, split summary for profiles/)."""
    import csv
    import shutil
    import statistics
    d = os.path.join(ROOT, "gpurun_out", "bench_kernel_trace")
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d, exist_ok=True)
    cmd = ["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "kt", "--",
           sys.executable, os.path.abspath(__file__), "--pmc-child", "trace",
           "--buckets", str(args.buckets), "--bucket-mib", str(args.bucket_mib), "--dtype", args.dtype]
    subprocess.run(cmd, check=True, timeout=240, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                   cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"))
    rows = []
    for dp, _, files in os.walk(d):
        for fn in files:
            if fn.endswith("kernel_trace.csv"):
                with open(os.path.join(dp, fn)) as f:
                    for row in csv.DictReader(f):
                        rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row["Kernel_Name"]))
    rows.sort()
    fills = [i for i, r in enumerate(rows) if "k_fill_uniform" in r[2]]
    tree = [(i, r[1] - r[0]) for i, r in enumerate(rows) if TREE_KERNEL in r[2]]
    if not fills or not tree:
        return None
    last_fill = fills[-1]
    c2 = [dur / 1e3 for i, dur in tree if i > last_fill][TRACE_WARM:]
    g = [dur for i, dur in tree if i < last_fill][TRACE_WARM * GATE_WINDOWS:]
    gate = [sum(g[j:j + GATE_WINDOWS]) / 1e3 for j in range(0, len(g) - GATE_WINDOWS + 1, GATE_WINDOWS)]
    c2_bytes = (args.buckets + 1) * int(args.bucket_mib * MiB)
    gate_bytes = (args.buckets + 1) * 256 * MiB
    summary = {"source": "rocprofv3 --kernel-trace of bench.py's trace child (%d C2 launches, %d gate calls "
                         "of %d windows, after %d warm-up calls each)" % (len(c2), len(gate), GATE_WINDOWS, TRACE_WARM),
               "kernel": TREE_KERNEL + ", 256>",
               "C2": {"dispatches": len(c2), "avg_us": round(statistics.fmean(c2), 2),
                      "median_us": round(statistics.median(c2), 2), "algo_bytes": c2_bytes,
                      "frac_of_8TBs": round(c2_bytes / (statistics.fmean(c2) * 1e-6) / 8e12, 4)},
               "gate_8x256MiB": {"calls": len(gate), "avg_us": round(statistics.fmean(gate), 2),
                                 "median_us": round(statistics.median(gate), 2), "algo_bytes": gate_bytes,
                                 "frac_of_8TBs": round(gate_bytes / (statistics.fmean(gate) * 1e-6) / 8e12, 4)}}
    with open(os.path.join(ROOT, "gpurun_out", "bench_kernel_trace_split.json"), "w") as f:
        json.dump(summary, f, indent=1)
    return summary


def run_local(args, esgd, dev):
    """N = 1: k staged buckets -> 1 output (config C2)."""
    from esgd import _lib
    k = args.buckets
    dt = _lib.FLOAT if args.dtype == "fp32" else _lib.BF16
    es = _lib.dtype_size(dt)
    count = int(args.bucket_mib * MiB) // es
    s = dev.Stream()
    bufs = [dev.DeviceBuffer(count, dt) for _ in range(k)]
    for r, b in enumerate(bufs):
        dev.fill_uniform(b, SEED, r, stream=s)
    out = dev.DeviceBuffer(count, dt)
    ptrs = [b.ptr for b in bufs]
    s.synchronize()

    if args.pmc_child == "trace":
        trace_child(dev, dt, ptrs, out, count, k, s)
        return None
    if args.pmc_child:
        args.no_gate = True
        for _ in range(PMC_CALLS):
            dev.reduce(dt, ptrs, out, count, stream=s)
        s.synchronize()
        return None

    # The gate leg (8 x 256 MiB) runs first: ~50 ms of streaming that leaves the GPU at its
    # steady clocks before the C2 warm-up and timed steps.  Measured cold, the first 40 C2
    # launches of a process averaged 95.7 us against 91.8 us over 120 launches of a longer
    # run on the same box (profiles/r03, r03ak).
    gate = None
    if not args.no_gate:
        gate = gate_256(dev, dt, es, k, s)

    for _ in range(args.warmup):
        dev.reduce(dt, ptrs, out, count, stream=s)
    s.synchronize()

    # HIP events on the launch stream inside the timed region: the average launch duration
    # including the dispatch gap between back-to-back launches (a pair around single
    # launches adds its marker packets' cost to every measured launch: 96.2 us per launch
    # against rocprof's 92.5 us on one box).  The region starts on an idle GPU (the sync
    # that brackets it), so its first launch also carries the host's submit latency and
    # the clock ramp; `kernel_ms` averages launches 2..K (event e1 follows launch 1 in
    # stream order), `kernel_ms_all` all K.
    e0, e1, e2 = dev.Event(), dev.Event(), dev.Event()
    dev.device_synchronize()
    t0 = time.perf_counter()
    e0.record(s)
    for i in range(args.steps):
        dev.reduce(dt, ptrs, out, count, stream=s)
        if i == 0:
            e1.record(s)
    e2.record(s)
    s.synchronize()
    dev.device_synchronize()
    wall = time.perf_counter() - t0
    per_launch_all_ms = e0.elapsed_ms(e2) / args.steps
    per_launch_ms = e1.elapsed_ms(e2) / (args.steps - 1) if args.steps > 1 else per_launch_all_ms

    # parity spot-check outside the timed region: first 1 Mi elements vs the oracle
    parity = "skipped"
    if dt == _lib.FLOAT:
        from oracle import ffref
        import numpy as np
        m = min(count, 1 << 20)
        got = out.download()[:m]
        want = ffref.tree_sum([ffref.fill_uniform(SEED, r, m) for r in range(k)])
        parity = "bitwise" if np.array_equal(got.view(np.uint32), want.view(np.uint32)) else "MISMATCH"

    e2e = host_e2e(dev, k, count, s) if (dt == _lib.FLOAT and not args.no_gate) else None
    bucket_bytes = count * es
    algo_bytes = (k + 1) * bucket_bytes        # k reads + 1 write per launch
    achieved = algo_bytes / (per_launch_ms * 1e-3) / 1e9
    return {
        "value": k * bucket_bytes * args.steps / wall / 1e9,
        "ms_per_step": wall * 1e3 / args.steps,
        "kernel_ms": per_launch_ms,
        "kernel_ms_all": per_launch_all_ms,
        "achieved_gbs": achieved,
        "algo_bytes": algo_bytes,
        "count": count,
        "bucket_bytes": bucket_bytes,
        "k": k,
        "parity": parity,
        "gate": gate,
        "host_e2e": e2e,
    }


def host_e2e(dev, k, count, s, iters=5):
    """The reference's contract: buckets start and end in (pinned) host memory.
    esgd_reduce_host: the tree kernel reads the pinned host buckets and writes the pinned
    output through their device views (zero-copy: PCIe in both directions at once).  Timed
    beside the plain sequence (all H2D, one tree launch, one D2H on one stream).  Reported beside the
    device-resident number, never as `value`."""
    import ctypes as C

    import numpy as np

    from esgd import _lib
    from esgd._lib import check, lib
    nbytes = count * 4
    hosts = []
    for _ in range(k + 1):
        p = C.c_void_p()
        check(lib().esgd_host_alloc(C.byref(p), nbytes))
        hosts.append(p.value)
    for j in range(k):
        np.frombuffer((C.c_char * nbytes).from_address(hosts[j]), dtype=np.float32)[:] = j
    bufs = [dev.DeviceBuffer(count) for _ in range(k)]
    out = dev.DeviceBuffer(count)
    res = np.frombuffer((C.c_char * nbytes).from_address(hosts[k]), dtype=np.float32)

    def serial():
        for j in range(k):
            check(lib().esgd_memcpy_async(bufs[j].ptr, hosts[j], nbytes, 0, s.handle))
        dev.reduce(_lib.FLOAT, [b.ptr for b in bufs], out, count, stream=s)
        check(lib().esgd_memcpy_async(hosts[k], out.ptr, nbytes, 1, s.handle))
        s.synchronize()

    def pipelined():
        dev.reduce_host(_lib.FLOAT, hosts[:k], hosts[k], count, stream=s)
        s.synchronize()

    def timed(fn):
        fn()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        return (time.perf_counter() - t0) / iters

    ts, tp = [], []
    for _ in range(2):   # interleaved
        ts.append(timed(serial))
        res[:] = -1.0
        tp.append(timed(pipelined))
    t, t_serial = min(tp), min(ts)
    ok = bool(np.all(res == float(sum(range(k)))))
    for p in hosts:
        lib().esgd_host_free(p)
    for b in bufs:
        b.close()
    out.close()
    return {"workload": f"{k} pinned host buckets of {nbytes / MiB:g} MiB -> 1 pinned host bucket "
                        "(esgd_reduce_host: tree kernel over the buckets' device views)",
            "ms": round(t * 1e3, 3), "GBs_bucket_bytes": round(k * nbytes / t / 1e9, 2),
            "pcie_bytes_per_step": (k + 1) * nbytes, "correct": ok,
            "serial_ms": round(t_serial * 1e3, 3), "serial_GBs_bucket_bytes": round(k * nbytes / t_serial / 1e9, 2)}


def gate_256(dev, dt, es, k, s, iters=20, avg_iters=100):
    """BASELINE.json's 1-GPU gate shape (k x 256 MiB buckets, no Infinity-Cache reuse
    possible): per-launch time from HIP event pairs on the launch stream."""
    count = (256 * MiB) // es
    bufs = [dev.DeviceBuffer(count, dt) for _ in range(k)]
    for r, b in enumerate(bufs):
        dev.fill_uniform(b, SEED, r, stream=s)
    out = dev.DeviceBuffer(count, dt)
    ptrs = [b.ptr for b in bufs]
    for _ in range(10):
        dev.reduce(dt, ptrs, out, count, stream=s)
    # per-launch event pairs (each adds its marker packets to the launch it brackets) ...
    ev = [dev.Event() for _ in range(2 * iters)]
    for i in range(iters):
        ev[2 * i].record(s)
        dev.reduce(dt, ptrs, out, count, stream=s)
        ev[2 * i + 1].record(s)
    s.synchronize()
    ts = sorted(ev[2 * i].elapsed_ms(ev[2 * i + 1]) for i in range(iters))
    med = ts[iters // 2]
    # ... and, like the headline roofline, one pair around `avg_iters` back-to-back calls
    # (38 ms of work: 20 calls were too short to average out run-to-run noise, 373 vs
    # 380 us on one box)
    e0, e1 = dev.Event(), dev.Event()
    e0.record(s)
    for _ in range(avg_iters):
        dev.reduce(dt, ptrs, out, count, stream=s)
    e1.record(s)
    s.synchronize()
    avg = e0.elapsed_ms(e1) / avg_iters
    algo = (k + 1) * count * es
    # also k = 2 in place, the reference's own step rb = tmp + rb
    # (ffallreduce.c:155-162; tmp is operand a): B = 3 S per call
    e0.record(s)
    for _ in range(avg_iters):
        dev.reduce(dt, [ptrs[0], ptrs[1]], ptrs[0], count, stream=s)
    e1.record(s)
    s.synchronize()
    avg2 = e0.elapsed_ms(e1) / avg_iters
    algo2 = 3 * count * es
    for b in bufs:
        b.close()
    out.close()
    return {"workload": f"{k} x 256 MiB -> 1", "kernel_ms_avg": round(avg, 4),
            "kernel_ms_median_per_launch_pairs": round(med, 4),
            "achieved_GBs": round(algo / (avg * 1e-3) / 1e9, 1),
            "frac": round(algo / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "k2_inplace": {"workload": "rb = tmp + rb, 2 x 256 MiB, in place", "kernel_ms_avg": round(avg2, 4),
                           "algo_bytes": algo2, "achieved_GBs": round(algo2 / (avg2 * 1e-3) / 1e9, 1),
                           "frac": round(algo2 / (avg2 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}}


# N > 1: schedules (and their buckets) stay alive until every leg has run, then are
# deleted together -- persistent, like the reference's.  Deleting one closes the peers'
# IPC mappings of its bucket, after which every later peer-reading kernel of the process
# is slower; nothing is closed while a leg is being timed.
_DEFERRED = []


def _defer(sch, *bufs):
    _DEFERRED.append((sch, bufs))


def _delete_deferred():
    while _DEFERRED:
        sch, bufs = _DEFERRED.pop(0)
        sch.delete()
        for b in bufs:
            b.close()


def _max_over_ranks(x: float) -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sweep_c5(comm, dev, world, dt, es):
    """C5: majority-allreduce of one bucket per rank, 64 KiB .. 1 GiB (every 2x).  Per
    size: 20 warm-up rounds, then 50 back-to-back rounds, each timed
    post -> wait on every rank; a round's time is its max over ranks; reported: the
    median round and the mean round."""
    import statistics

    import torch
    import torch.distributed as dist
    out = []
    for lg in range(16, 31):   # the 15 sizes of SURVEY.md §8(d), 64 KiB .. 1 GiB
        nbytes = 1 << lg
        iters = 50
        count = nbytes // es
        buf = dev.DeviceBuffer(count, dt)
        dev.fill_uniform(buf, SEED, comm.rank())
        dev.synchronize()
        sch = comm.Schedule(comm.MAJORITY, None, buf, count, dtype=dt, seed=6545343,
                            buf=comm.BUF_DEVICE)
        for _ in range(20):
            sch.post(); sch.wait()
        comm.barrier()
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            sch.post(); sch.wait()
            ts.append(time.perf_counter() - t0)
        tt = torch.tensor(ts, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        ts = tt.tolist()
        t, mean = statistics.median(ts), statistics.fmean(ts)
        stages = _stages_us(sch.timeline()[-iters:])
        _defer(sch, buf)
        t_min = 2 * nbytes / (world * XGMI_LINK_GBS * 1e9)
        out.append({"bytes": nbytes, "us": round(t * 1e6, 1), "mean_us": round(mean * 1e6, 1),
                    "algbw_GBs": round(nbytes / t / 1e9, 2),
                    "busbw_GBs": round(nbytes / t / 1e9 * 2 * (world - 1) / world, 2),
                    "xgmi_frac": None if SHARED_GPU else round(t_min / t, 4), "rounds": iters,
                    "rank0_stages_us": stages})
    return out


def _round_us(comm, dev, count, kind, warm=10, iters=30, dt=None):
    """Median (and mean) round time of a fresh schedule over a device bucket: `warm`
    rounds, then `iters` post -> wait rounds back to back, each round's time the max over
    ranks (as sweep_c5).  Uses whatever esgd_set_config the caller set."""
    import statistics

    import torch
    import torch.distributed as dist

    from esgd import _lib
    dt = _lib.FLOAT if dt is None else dt
    buf = dev.DeviceBuffer(count, dt)
    dev.fill_uniform(buf, SEED, comm.rank())
    dev.synchronize()
    sch = comm.Schedule(kind, None, buf, count, dtype=dt, seed=6545343, buf=comm.BUF_DEVICE)
    for _ in range(warm):
        sch.post(); sch.wait()
    comm.barrier()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        sch.post(); sch.wait()
        ts.append(time.perf_counter() - t0)
    tt = torch.tensor(ts, dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    ts = tt.tolist()
    _defer(sch, buf)
    return statistics.median(ts) * 1e6, statistics.fmean(ts) * 1e6


def ab_one_launch_threshold(comm, dev, world, sizes_mib=(1, 2, 4, 8, 16)):
    """The one-launch threshold (esgd_set_config "small_round_bytes", default 4 MiB)
    A/B'd on this node: majority-allreduce rounds of each size run both ways -- ONE
    k_round_small launch (pairing + reduce-scatter + pairing + all-gather inside one
    kernel) and the five-launch round -- in the same job.  `best_threshold_MiB` is the
    largest size where the one-launch round is still faster (what the default should be
    on this topology)."""
    out = {"sizes": []}
    best = 0
    try:
        for mib in sizes_mib:
            count = int(mib * MiB) // 4
            comm.set_config("small_round_bytes", count * 4)
            one, one_mean = _round_us(comm, dev, count, comm.MAJORITY)
            comm.set_config("small_round_bytes", 0)
            five, five_mean = _round_us(comm, dev, count, comm.MAJORITY)
            out["sizes"].append({"bytes": count * 4, "one_launch_us": round(one, 1), "five_launch_us": round(five, 1),
                                 "one_launch_mean_us": round(one_mean, 1), "five_launch_mean_us": round(five_mean, 1)})
            if one < five:
                best = mib
    finally:
        comm.set_config("small_round_bytes", -1)
    out["default_MiB"] = 4
    out["best_threshold_MiB"] = best
    return out


def ab_flag_pages(comm, dev, world, sizes=(65536, 16 << 20)):
    """Where the rank-pairing flags live (esgd_set_config "device_flags"): 0 pinned host
    memory (default; polled over PCIe), 1 uncached HBM pages, 2 fine-grained HBM pages
    (peers' words written over xGMI), each at a one-launch size (64 KiB) and a
    five-launch size (16 MiB), median majority round."""
    out = {}
    try:
        for mode, name in ((0, "host"), (1, "hbm_uncached"), (2, "hbm_finegrained")):
            comm.set_config("device_flags", mode)
            out[name] = {}
            for nbytes in sizes:
                med, mean = _round_us(comm, dev, nbytes // 4, comm.MAJORITY)
                out[name][str(nbytes)] = {"us": round(med, 1), "mean_us": round(mean, 1)}
    finally:
        comm.set_config("device_flags", -1)
    return out


def _timed_steps(comm, fn, steps):
    """Median over `steps` of fn()'s wall time, each step's time the max over ranks."""
    import statistics

    import torch
    import torch.distributed as dist
    ts = []
    for _ in range(steps):
        comm.barrier()
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    tt = torch.tensor(ts, dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return statistics.median(tt.tolist())


def c4_resnet50_161(comm, dev, rank, world, steps=8):
    """C4 as the reference runs it: one majority schedule per ResNet-50 gradient tensor
    (161 buckets, opt_esgd_solo_imagenet_imbalance.py:86-248; tests/golden/
    resnet50_buckets.json), reduced one after another every step like the op chain of
    :24-44 -- against the same 25 559 081 fp32 as ONE fused bucket
    (EagerSGDOptimizer(fuse=True)), and the 161 rounds all posted before the first wait
    (EagerSGDOptimizer's per-tensor default).  All ranks post every bucket (no straggler)."""
    with open(os.path.join(ROOT, "tests", "golden", "resnet50_buckets.json")) as f:
        lengths = json.load(f)["lengths"]
    total = sum(lengths)
    bufs = [dev.DeviceBuffer(n) for n in lengths]
    for b in bufs:
        dev.fill_uniform(b, SEED, rank)
    fused = dev.DeviceBuffer(total)
    dev.fill_uniform(fused, SEED, rank)
    dev.synchronize()
    scheds = [comm.Schedule(comm.MAJORITY, None, b, b.count, seed=6545343, buf=comm.BUF_DEVICE)
              for b in bufs]
    one = comm.Schedule(comm.MAJORITY, None, fused, total, seed=6545343, buf=comm.BUF_DEVICE)

    def chain():
        for s in scheds:
            s.post()
            s.wait()

    def pipelined():   # EagerSGDOptimizer's default: every round posted, then waited
        for s in scheds:
            s.post()
        for s in scheds:
            s.wait()

    def fused_step():
        one.post()
        one.wait()

    for _ in range(2):
        chain()
        pipelined()
        fused_step()
    t161 = _timed_steps(comm, chain, steps)
    chain_stages = _round_stages_us(scheds)
    l0, p0 = comm.get_config("launches"), comm.profile()
    t161p = _timed_steps(comm, pipelined, steps)
    launches = (comm.get_config("launches") - l0) / steps
    prof = _profile_per_step(p0, comm.profile(), steps)
    breakdown = _step_breakdown_us(scheds)
    # A/B: the same pipelined step with one launch per round (k_round_small), no sharing
    comm.set_config("batch_rounds", 0)
    try:
        pipelined()
        p0 = comm.profile()
        t161u = _timed_steps(comm, pipelined, steps)
        prof_u = _profile_per_step(p0, comm.profile(), steps)
        breakdown_u = _step_breakdown_us(scheds)
    finally:
        comm.set_config("batch_rounds", -1)
    t1 = _timed_steps(comm, fused_step, steps)
    variants = _op_like_variants(comm, dev, lengths, steps)
    launch_shape = _launch_shape_ab(comm, bufs, lengths, steps)
    for s, b in zip(scheds, bufs):
        _defer(s, b)
    _defer(one, fused)
    return {"buckets": len(lengths), "fp32_elements": total,
            "step_ms_161_buckets": round(t161 * 1e3, 3),
            "step_ms_161_buckets_pipelined": round(t161p * 1e3, 3),
            "rank0_chain_round_stages_us": chain_stages,
            "step_ms_one_fused_bucket": round(t1 * 1e3, 3),
            "fused_speedup": round(t161 / t1, 2), "steps": steps,
            "rank0_launches_per_pipelined_step": launches,
            "rank0_pipelined_step_us": breakdown,
            "rank0_progress_thread_per_step": prof,
            "step_ms_161_buckets_pipelined_one_launch_per_round": round(t161u * 1e3, 3),
            "rank0_pipelined_step_us_one_launch_per_round": breakdown_u,
            "rank0_progress_thread_per_step_one_launch_per_round": prof_u,
            "op_like_pipelined_variants": variants,
            "launch_shape_ab": launch_shape}


def _launch_shape_ab(comm, bufs, lengths, steps):
    """The pipelined 161-bucket step over schedules created with every ResNet-50 bucket a
    one-launch round (small_round_bytes 16 MiB: the 9 buckets above 4 MiB too, no five-launch
    rounds) and shared launches of up to 256 workers (batch_workers_max) -- against the
    defaults (4 MiB, 64) measured above.  On the 1-GPU rehearsal this took the optimizer's
    step from 1.48 to 1.14-1.23 ms at P = 2 and left P = 4 unchanged
    (profiles/r05/threshold_workers_ab/); a GPU per rank decides the defaults."""
    comm.set_config("small_round_bytes", 16 << 20)
    comm.set_config("batch_workers_max", 256)
    try:
        scheds = [comm.Schedule(comm.MAJORITY, None, b, b.count, seed=6545343, buf=comm.BUF_DEVICE) for b in bufs]

        def pipelined():
            for s in scheds:
                s.post()
            for s in scheds:
                s.wait()

        for _ in range(2):
            pipelined()
        t = _timed_steps(comm, pipelined, steps)
        breakdown = _step_breakdown_us(scheds)
        workers = comm.get_config("batch_workers")
    finally:
        comm.set_config("small_round_bytes", -1)
        comm.set_config("batch_workers_max", -1)
    for s in scheds:
        _defer(s)
    return {"small_round_bytes": 16 << 20, "batch_workers_max": 256,
            "step_ms_161_buckets_pipelined": round(t * 1e3, 3), "rank0_step_us": breakdown,
            "last_launch_workers": workers}


def _op_like_variants(comm, dev, lengths, steps):
    """The pipelined 161-bucket step with the deep500 op's schedule properties added one at
    a time (what separates this leg's step from the optimizer's): HOLD | FRESH_ONLY with
    group post / release; a separate send bucket (the snapshot copies it into rb); both;
    both with the legacy NULL stream as the producer and consumer stream (torch's default).
    Per variant: ms per step, rank 0's timeline breakdown and progress-thread profile."""
    import torch
    out = {}
    hf = comm.HOLD | comm.FRESH_ONLY
    for name, sep, flags, stream, rstream in (
            ("hold_fresh_group", False, hf, None, None),
            ("separate_sb", True, 0, None, None),
            ("separate_sb_hold_fresh_group", True, hf, None, None),
            ("separate_sb_hold_fresh_group_null_stream", True, hf, 0, 0)):
        # (producer-only / consumer-only NULL-stream variants: profiles/r04/extra_queues_ab/;
        # every variant is 161 more schedules of the job's 2048)
        rbs = [dev.DeviceBuffer(n) for n in lengths]
        sbs = [dev.DeviceBuffer(n) for n in lengths] if sep else [None] * len(lengths)
        for b in (sbs if sep else rbs):
            dev.fill_uniform(b, SEED, comm.rank())
        dev.synchronize()
        scheds = [comm.Schedule(comm.MAJORITY, sb, rb, rb.count, seed=6545343, buf=comm.BUF_DEVICE, flags=flags)
                  for sb, rb in zip(sbs, rbs)]
        hold = bool(flags & comm.HOLD)

        def step():
            if hold:
                comm.post_group(scheds, stream)
            else:
                for sc in scheds:
                    sc.post()
            for sc in scheds:
                sc.wait()
            if hold:
                comm.release_group(scheds, rstream)
            if stream is not None or rstream is not None:
                torch.cuda.synchronize()

        for _ in range(2):
            step()
        p0 = comm.profile()
        t = _timed_steps(comm, step, steps)
        out[name] = {"step_ms": round(t * 1e3, 3), "rank0_step_us": _step_breakdown_us(scheds),
                     "rank0_progress_thread_per_step": _profile_per_step(p0, comm.profile(), steps)}
        for sc, rb, sb in zip(scheds, rbs, sbs):
            _defer(sc, *([rb] if sb is None else [rb, sb]))
    return out


def _profile_per_step(p0, p1, steps):
    """esgd_comm_profile differences per step: busy passes, us inside them, us launching
    (issue-ring pumps), joins and us joining, launches and us flushing shared launches."""
    d = {k: (p1[k] - p0[k]) / steps for k in p0}
    return {"passes": round(d["passes"], 1), "pass_us": round(d["pass_ns"] / 1e3, 1),
            "launch_us": round(d["launch_ns"] / 1e3, 1), "joins": round(d["joins"], 1),
            "join_us": round(d["join_ns"] / 1e3, 1), "launches": round(d["launches"], 2),
            "flush_us": round(d["flush_ns"] / 1e3, 1)}


def _timeline_of(handle):
    """esgd_schedule_timeline of a raw schedule handle (a deep500 op's, esgd_op_schedule)."""
    import ctypes as C

    import numpy as np

    from esgd._lib import check, lib
    n = C.c_uint32()
    check(lib().esgd_schedule_timeline(C.c_uint64(handle), None, 0, C.byref(n)))
    out = np.zeros((max(1, n.value), 12), np.uint64)
    check(lib().esgd_schedule_timeline(C.c_uint64(handle), out.ctypes.data_as(C.POINTER(C.c_uint64)), n.value,
                                       C.byref(n)))
    return out[: n.value]


def _step_breakdown_us(scheds):
    """Where the last pipelined step's time went on this rank, from every schedule's host
    timeline (esgd_schedule_timeline) of its last round: stamps relative to the first post,
    in us -- the last post / join / launch queued / completion seen / wait returned, the
    host time spent inside launches summed over the buckets."""
    import numpy as np
    rows = []
    for s in scheds:
        tl = (s.timeline() if hasattr(s, "timeline") else _timeline_of(s)).astype(np.int64)
        tl = tl[(tl[:, 0] > 0) & (tl[:, 5] > 0)]
        if len(tl):
            rows.append(tl[-1])
    if not rows:
        return None
    tl = np.array(rows)
    t0 = tl[:, 0].min()
    rel = lambda i: round(float(tl[:, i].max() - t0) / 1e3, 1)   # noqa: E731
    return {"last_post": rel(0), "last_join": rel(1), "last_launch_queued": rel(3), "last_completion": rel(4),
            "last_wait": rel(5), "launch_host_sum": round(float((tl[:, 3] - tl[:, 2]).sum()) / 1e3, 1),
            "first_launch": round(float(tl[:, 2].min() - t0) / 1e3, 1),
            "gpu_us_per_bucket": round(float(tl[:, 4].max() - tl[:, 2].min()) / 1e3 / len(tl), 2)}


def _round_stages_us(scheds):
    """A chain of rounds, one at a time (the reference's blocking pattern): where a round's
    time goes on this rank, the median over the schedules' last rounds of each stage of the
    host timeline (esgd_schedule_timeline), in us -- post -> join -> launch start -> launch
    queued -> completion seen -> wait returned; and the median time from one round's post
    to the next one's (the chain's cycle: what the caller does between rounds included)."""
    import numpy as np
    rows = []
    for s in scheds:
        tl = (s.timeline() if hasattr(s, "timeline") else _timeline_of(s)).astype(np.int64)
        tl = tl[(tl[:, 0] > 0) & (tl[:, 5] > 0) & (tl[:, 1] > 0) & (tl[:, 2] > 0)]
        if len(tl):
            rows.append(tl[-1])
    if len(rows) < 2:
        return None
    tl = np.array(rows)
    tl = tl[np.argsort(tl[:, 0])]
    med = lambda a: round(float(np.median(a)) / 1e3, 2)   # noqa: E731
    return {"post_to_join": med(tl[:, 1] - tl[:, 0]), "join_to_launch": med(tl[:, 2] - tl[:, 1]),
            "launch_host": med(tl[:, 3] - tl[:, 2]), "launch_to_completion": med(tl[:, 4] - tl[:, 3]),
            "completion_to_wait": med(tl[:, 5] - tl[:, 4]), "post_to_wait": med(tl[:, 5] - tl[:, 0]),
            "cycle": med(np.diff(tl[:, 0])), "rounds": len(tl)}


def optimizer_resnet50_161(comm, rank, world, steps=8):
    """The drop-in caller path at C4's shape: EagerSGDOptimizer (majority, the reference's
    seed) over 161 torch parameters with the ResNet-50 bucket lengths
    (opt_esgd_majority_imagenet_imbalance.py:6-44; tests/golden/resnet50_buckets.json), the
    gradients already on the device; one step = apply_gradients() (copy-in with the /P,
    the rounds, the copy-out, the wrapped SGD step), max over ranks.  Per tensor pipelined
    (the default; shared launches on and off), per tensor blocking (the reference's chain),
    fused."""
    import torch

    import ctypes as C

    from esgd._lib import check, lib
    from esgd.optim import EagerSGDOptimizer
    with open(os.path.join(ROOT, "tests", "golden", "resnet50_buckets.json")) as f:
        lengths = json.load(f)["lengths"]
    d = C.c_int()
    check(lib().esgd_get_device(C.byref(d)))
    torch.cuda.set_device(d.value)   # the rank's GPU (esgd_set_device chose it)
    dev_t = torch.device("cuda", d.value)
    gen = torch.Generator(device=dev_t)
    gen.manual_seed(SEED + rank)
    out = {}
    opts = []
    # (round 6: the A/B variants whose alternative lost -- rounds waited for on the GPU, the
    # ops on the data plane's round stream, copy kernels instead of the rounds' own I/O, the
    # caller on a side stream, idle-stream skips, snapshot worker caps -- are gone with their
    # switches; their numbers are in profiles/r05/)
    for name, kw in (("per_tensor_pipelined", dict(fuse=False)),
                     ("per_tensor_blocking", dict(pipeline=False)),
                     ("fused", dict(fuse=True))):
        params = [torch.zeros(n, device=dev_t, requires_grad=True) for n in lengths]
        for p in params:
            p.grad = torch.rand(p.numel(), device=dev_t, generator=gen) - 0.5
        opt = EagerSGDOptimizer(torch.optim.SGD(params, lr=1e-3), world, mode="majority", **kw)
        opts.append(opt)

        def step(opt=opt):
            opt.step()
            torch.cuda.synchronize()

        step()   # creates the ops' schedules (collective, first step)
        step()
        p0 = comm.profile()
        out[name + "_ms"] = round(_timed_steps(comm, step, steps) * 1e3, 3)
        out[name + "_progress_thread_per_step"] = _profile_per_step(p0, comm.profile(), steps)
        if name != "fused":
            out[name + "_breakdown_us"] = _optimizer_breakdown(opt, steps, None)
            out[name + "_rank0_step_us"] = _step_breakdown_us([op.schedule() for op in opt._ops.values()])
        else:
            out["fused_breakdown_us"] = _fused_breakdown(comm, opt, params, steps)
        if name == "per_tensor_blocking":
            out[name + "_round_stages_us"] = _round_stages_us([op.schedule() for op in opt._ops.values()])
        if name == "per_tensor_pipelined":
            # the same step with one launch per round (no shared launches; process-local)
            for key, vals, what in (("batch_rounds", {"batch_rounds": 0}, "_one_launch_per_round_ms"),):
                for k, v in vals.items():
                    comm.set_config(k, v)
                try:
                    step()
                    out[name + what] = round(_timed_steps(comm, step, steps) * 1e3, 3)
                finally:
                    for k in vals:
                        comm.set_config(k, -1)
    _OPTS.extend(opts)   # their schedules stay alive until the end, like every leg's
    out["grad_view_backward_us"] = _grad_view_backward_us(params, steps)
    out["tensors"] = len(lengths)
    out["steps"] = steps
    return out


_OPTS = []


def _grad_view_backward_us(params, steps):
    """What gradients as views into the buckets (DDP's gradient_as_bucket_view; VERDICT r05
    item 4) would add to backward, per step on this rank's GPU: with
    p.grad a persistent view, zero_grad zeroes it (one foreach launch, S written) and
    AccumulateGrad adds the fresh gradient into it (one launch per tensor, 2S read, S
    written) -- where today's path takes the fresh gradient as p.grad and the round's I/O
    moves it.  Median GPU time over `steps` (torch events on the current stream); set this
    against caller_vs_data_plane's op-like minus in-place rounds, the most views could
    remove from the step."""
    import statistics

    import torch
    views = [p.grad for p in params]
    fresh = [torch.empty_like(v).copy_(v) for v in views]
    zero_us, acc_us = [], []
    for _ in range(steps + 1):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        torch._foreach_zero_(views)
        e1.record()
        for v, g in zip(views, fresh):
            v.add_(g)
        e2.record()
        e2.synchronize()
        zero_us.append(e0.elapsed_time(e1) * 1e3)
        acc_us.append(e1.elapsed_time(e2) * 1e3)
    zero_us, acc_us = zero_us[1:], acc_us[1:]     # the first pass warms the kernels
    total_bytes = sum(v.numel() for v in views) * 4
    return {"zero_grad": round(statistics.median(zero_us), 1),
            "accumulate_161": round(statistics.median(acc_us), 1),
            "total": round(statistics.median(z + a for z, a in zip(zero_us, acc_us)), 1),
            "hbm_bytes": 4 * total_bytes}


def _fused_breakdown(comm, opt, params, steps):
    """Where the fused optimizer step's time goes (EagerSGDOptimizer(fuse=True)): each part
    timed alone on this rank, median over `steps`, against the whole step -- the pack of the
    161 gradients (divided by P) into a bucket and the unpack back (torch events on the
    caller's stream around one launch group each: what the round's own copy-in / copy-out
    cost), the fused bucket's round alone (post -> wait, wall, max over ranks), the round as
    the step runs it (esgd_schedule_post_iov: pack + round + unpack on the round stream), the
    wrapped SGD step (events), and apply_gradients + synchronize (wall, max over ranks).  The
    step against (round with pack / unpack + SGD) is the host / launch overhead."""
    import statistics

    import torch

    from esgd import _lib
    from esgd import device as dev
    from esgd._lib import check, lib
    layout, op = opt._fused
    total = sum(n for _, n in layout)
    grads = [p.grad for p in reversed(params)]
    bucket = torch.empty(total, device=grads[0].device)
    counts = [g.numel() for g in grads]
    stream = torch.cuda.current_stream()

    def gpu_ms(fn):
        ts = []
        for _ in range(steps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            fn()
            b.record(stream)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return statistics.median(ts)

    pack = gpu_ms(lambda: dev.pack_div(grads, counts, bucket, float(comm.world()), stream.cuda_stream or 1))
    unpack = gpu_ms(lambda: dev.unpack(grads, counts, bucket, stream.cuda_stream or 1))
    sgd = gpu_ms(lambda: opt.optimizer.step())
    h = C_u64(op.schedule())

    def one_round():
        check(lib().esgd_schedule_post(h, None, None), "post")
        check(lib().esgd_schedule_wait(h), "wait")
        check(lib().esgd_schedule_release(h, None), "release")

    import ctypes as C
    n = len(grads)
    ptrs = _lib.ptr_array([g.data_ptr() for g in grads])
    cnt = (C.c_uint64 * n)(*counts)
    sh = stream.cuda_stream or 1   # ESGD_STREAM_NULL: torch's legacy stream

    def one_round_iov():   # what the step's round is: pack (/ P) + round + unpack, on the round stream
        check(lib().esgd_schedule_post_iov(h, n, ptrs, ptrs, cnt, float(comm.world()), sh, None), "post_iov")
        check(lib().esgd_schedule_wait(h), "wait")
        check(lib().esgd_schedule_release(h, None), "release")

    rnd = _timed_steps(comm, one_round, steps)
    rnd_io = _timed_steps(comm, one_round_iov, steps)
    whole = _timed_steps(comm, lambda: (opt.step(), torch.cuda.synchronize()), steps)
    parts = sgd + rnd_io * 1e3
    return {"pack_div_gpu": round(pack * 1e3, 1), "round_wall": round(rnd * 1e6, 1),
            "unpack_gpu": round(unpack * 1e3, 1), "round_with_pack_unpack_wall": round(rnd_io * 1e6, 1),
            "sgd_step_gpu": round(sgd * 1e3, 1),
            "step_wall": round(whole * 1e6, 1), "parts_sum": round(parts * 1e3, 1),
            "overhead": round((whole * 1e3 - parts) * 1e3, 1), "fp32_elements": total}


def C_u64(v):
    import ctypes as C
    return C.c_uint64(v)


def _optimizer_breakdown(opt, steps, stream=None):
    """Median host time per step inside apply_gradients (rank 0's view, untimed steps):
    the wrapper's Python loop over the tensors, post_many_io, wait_many (or the blocking
    per-tensor forward calls), the wrapped SGD step and the closing synchronize."""
    import contextlib
    import statistics

    import torch

    from esgd import deep500
    Op = deep500.AllreduceOp
    acc = {}

    def timed(key, f):
        def g(*a, **k):
            t0 = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                acc[key] = acc.get(key, 0.0) + time.perf_counter() - t0
        return g

    saved = (Op.wait_many, Op.forward_cuda_div, opt.optimizer.step, Op.post_many_io)
    Op.wait_many = staticmethod(timed("wait_many", saved[0]))
    Op.forward_cuda_div = timed("forward_cuda_div", saved[1])
    opt.optimizer.step = timed("sgd_step", saved[2])
    Op.post_many_io = staticmethod(timed("post_many_io", saved[3]))
    rows = []
    try:
        for _ in range(steps):
            acc.clear()
            t0 = time.perf_counter()
            with (torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()):
                opt.step()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            row = dict(acc)
            row["apply_gradients"] = t1 - t0
            row["python_loop"] = row["apply_gradients"] - sum(v for k, v in acc.items())
            row["synchronize"] = t2 - t1
            rows.append(row)
    finally:
        Op.wait_many = staticmethod(saved[0])
        Op.forward_cuda_div = saved[1]
        Op.post_many_io = staticmethod(saved[3])
        del opt.optimizer.step   # the instance attribute; the class method shows again
    keys = sorted({k for r in rows for k in r})
    return {k: round(statistics.median(r.get(k, 0.0) for r in rows) * 1e6, 1) for k in keys}


def c3_over_rccl(comm, dev, rank, world, count, steps=20):
    """C3 (solo-allreduce, 256 MiB per rank) through the RCCL transport: grouped
    ncclSend/ncclRecv over xGMI, arrived chunks folded by the tree kernel on a side
    stream.  Needs one GPU per rank (RCCL refuses duplicate GPUs)."""
    import numpy as np

    import esgd
    from oracle import ffref
    if world > esgd.device_count():
        return {"skipped": "ranks share a GPU; RCCL refuses duplicate GPUs"}
    comm.set_transport("rccl")
    try:
        rb = dev.DeviceBuffer(count)
        dev.fill_uniform(rb, SEED, rank)
        dev.synchronize()
        sch = comm.Schedule(comm.SOLO, None, rb, count, async_=32, seed=6545343, buf=comm.BUF_DEVICE)

        def step():
            sch.post()
            sch.wait()

        for _ in range(3):
            step()
        t = _timed_steps(comm, step, steps)
        dev.fill_uniform(rb, SEED + 1, rank)
        dev.synchronize()
        comm.barrier()
        step()
        m = min(count, 1 << 18)
        got = rb.download()[:m]
        want = ffref.tree_sum([ffref.fill_uniform(SEED + 1, r, m) for r in range(world)])
        ok = bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
        sch.delete()
        # the same round with bf16 on the wire (half the RCCL bytes; the oracle's bf16
        # convention, as for the IPC wire leg)
        sw = comm.Schedule(comm.SOLO, None, rb, count, async_=32, seed=6545343, buf=comm.BUF_DEVICE,
                           flags=comm.WIRE_BF16)

        def wstep():
            sw.post()
            sw.wait()

        for _ in range(3):
            wstep()
        tw = _timed_steps(comm, wstep, steps)
        dev.fill_uniform(rb, SEED + 1, rank)
        dev.synchronize()
        comm.barrier()
        wstep()
        got = rb.download()[:m]
        want = ffref.bf16_to_f32(ffref.tree_sum_bf16(
            [ffref.f32_to_bf16(ffref.fill_uniform(SEED + 1, r, m)) for r in range(world)]))
        okw = bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
        sw.delete()
        rb.close()
    finally:
        comm.set_transport("ipc")
    S = count * 4
    t_min = 2 * S / (world * XGMI_LINK_GBS * 1e9)
    return {"bucket_bytes": S, "round_ms_median": round(t * 1e3, 4),
            "value_GBs": round(world * S / t / 1e9, 2), "algbw_GBs": round(S / t / 1e9, 2),
            "xgmi_frac": round(t_min / t, 4), "parity_rank_slice": "bitwise" if ok else "MISMATCH",
            "wire_bf16": {"round_ms_median": round(tw * 1e3, 4), "value_GBs": round(world * S / tw / 1e9, 2),
                          "xgmi_frac": round(t_min / 2 / tw, 4),
                          "parity_rank_slice": "bitwise" if okw else "MISMATCH"}}


def rccl_as_default_c3_c4(comm, dev, rank, world, count, ipc_c3_ms, ipc_c4, steps=10):
    """C3 and C4 with RCCL P2P as the transport every schedule of the leg is created with
    (esgd_set_transport("rccl")) -- the data plane the north star names -- head to head with
    the IPC pull numbers of this job: C3 = solo rounds of one 256 MiB fp32 bucket per GPU
    (the headline's shape), C4 = majority rounds of the ResNet-50 fused gradient with the
    last rank 0.2 T late (straggler_c4's shape and contributor check).  One GPU per rank."""
    import numpy as np

    from oracle import ffref
    if SHARED_GPU:
        return {"skipped": "ranks share a GPU (a 1-GPU rehearsal): RCCL refuses two ranks on one device, so "
                           "RCCL cannot be any schedule's transport here; the leg runs with one GPU per rank"}
    comm.set_transport("rccl")
    try:
        rb = dev.DeviceBuffer(count)
        dev.fill_uniform(rb, SEED, rank)
        dev.synchronize()
        sch = comm.Schedule(comm.SOLO, None, rb, count, async_=32, seed=6545343, buf=comm.BUF_DEVICE)

        def step():
            sch.post()
            sch.wait()

        for _ in range(3):
            step()
        t = _timed_steps(comm, step, steps)
        dev.fill_uniform(rb, SEED + 3, rank)
        dev.synchronize()
        comm.barrier()
        step()
        m = min(count, 1 << 18)
        got = rb.download()[:m]
        ok = bool(np.array_equal(got.view(np.uint32),
                                 ffref.tree_sum([ffref.fill_uniform(SEED + 3, r, m) for r in range(world)]).view(
                                     np.uint32)))
        sch.delete()
        rb.close()
        c4 = straggler_c4(comm, dev, rank, world, rounds=8, delay_fracs=(0.2,))
    finally:
        comm.set_transport("ipc")
    S = count * 4
    t_min = 2 * S / (world * XGMI_LINK_GBS * 1e9)
    ipc4 = (ipc_c4 or {}).get("delay_0.2T", {})
    return {"c3": {"round_ms_median": round(t * 1e3, 4), "value_GBs": round(world * S / t / 1e9, 2),
                   "xgmi_frac": round(t_min / t, 4), "parity_head_slice": "bitwise" if ok else "MISMATCH",
                   "ipc_pull_round_ms": ipc_c3_ms,
                   "rccl_over_ipc_time": round(t * 1e3 / ipc_c3_ms, 3) if ipc_c3_ms else None},
            "c4": {"T_no_straggler_ms": c4["T_no_straggler_ms"], "delay_0.2T": c4["delay_0.2T"],
                   "ipc_pull_T_no_straggler_ms": (ipc_c4 or {}).get("T_no_straggler_ms"),
                   "ipc_pull_on_time_ranks_median_ms": ipc4.get("on_time_ranks_median_ms")}}


def c3_wire_bf16(comm, dev, rank, world, count, steps=20):
    """C3 (solo-allreduce, 256 MiB fp32 per rank) with bf16 on the wire
    (ESGD_SCHED_WIRE_BF16): peers read a bf16 copy of every
    bucket, half the xGMI bytes of the fp32 headline, for one more local pass.  Measured
    A/B against the fp32 round in the same leg, the same way (median of per-step max over
    ranks).  The result is the bf16-rounded tree (an extension; parity vs the oracle's
    convention on head/tail slices).  xgmi_frac is against the wire bytes:
    t_min = 2 (S/2) / (P x 153 GB/s)."""
    import numpy as np

    from oracle import ffref
    rb = dev.DeviceBuffer(count)
    dev.fill_uniform(rb, SEED, rank)
    dev.synchronize()
    sw = comm.Schedule(comm.SOLO, None, rb, count, async_=32, seed=6545343, buf=comm.BUF_DEVICE,
                       flags=comm.WIRE_BF16)
    sf = comm.Schedule(comm.SOLO, None, rb, count, async_=32, seed=6545343, buf=comm.BUF_DEVICE)

    def stepper(sch):
        def step():
            sch.post()
            sch.wait()
        return step

    for _ in range(3):
        stepper(sw)()
        stepper(sf)()
    tw, tf = [], []
    for _ in range(4):   # interleaved A/B blocks
        tw.append(_timed_steps(comm, stepper(sw), steps // 4))
        tf.append(_timed_steps(comm, stepper(sf), steps // 4))
    t, t32 = float(np.median(tw)), float(np.median(tf))
    stages = _stages_us(sw.timeline()[-(steps // 4):])
    dev.fill_uniform(rb, SEED + 1, rank)
    dev.synchronize()
    comm.barrier()
    stepper(sw)()
    got = rb.download()
    m = min(count, 1 << 18)
    ok = True
    for start in (0, count - m):
        xs = [ffref.f32_to_bf16(ffref.fill_uniform(SEED + 1, r, m, start=start)) for r in range(world)]
        want = ffref.bf16_to_f32(ffref.tree_sum_bf16(xs))
        ok &= bool(np.array_equal(got[start:start + m].view(np.uint32), want.view(np.uint32)))
    _defer(sw, rb)
    _defer(sf)
    S = count * 4
    t_min = 2 * (S / 2) / (world * XGMI_LINK_GBS * 1e9)
    return {"bucket_bytes": S, "wire_bytes": S // 2, "round_ms_median": round(t * 1e3, 4),
            "fp32_round_ms_median": round(t32 * 1e3, 4), "speedup_vs_fp32": round(t32 / t, 3),
            "value_GBs": round(world * S / t / 1e9, 2), "algbw_GBs": round(S / t / 1e9, 2),
            "xgmi_frac": None if SHARED_GPU else round(t_min / t, 4), "rank0_stages_us": stages,
            "parity_head_tail": "bf16 convention, bitwise" if ok else "MISMATCH"}


def c1_host_majority(comm, dev, rank, world, count=262144, warmup=20, iters=50):
    """BASELINE's C1 shape on the GPU path and the reference's contract: majority-allreduce
    of a 1 MiB fp32 HOST bucket (calloc'd in the wrapper, opt_esgd_majority...py:288-298;
    pinned here at creation), seed 6545343 (:252), every rank posting every round: each
    round is H2D -> one-launch round -> D2H.  Timed post -> wait, max over ranks, median
    of `iters` rounds; the CPU restatement of the same shape is `cpu_baseline_c1`."""
    import statistics

    import numpy as np
    import torch
    import torch.distributed as dist

    from oracle import ffref
    host = np.zeros(count, np.float32)
    sch = comm.Schedule(comm.MAJORITY, None, host, count, seed=6545343, buf=comm.BUF_HOST)
    x = ffref.fill_uniform(SEED, rank, count)
    for _ in range(warmup):
        host[:] = x
        sch.post(); sch.wait()
    ts = []
    for _ in range(iters):
        host[:] = x
        comm.barrier()
        t0 = time.perf_counter()
        sch.post(); sch.wait()
        ts.append(time.perf_counter() - t0)
    tt = torch.tensor(ts, dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    t = statistics.median(tt.tolist())
    want = ffref.tree_sum([ffref.fill_uniform(SEED, r, count) for r in range(world)])
    ok = bool(np.array_equal(host.view(np.uint32), want.view(np.uint32)))
    stages = _stages_us(sch.timeline()[-iters:])
    _defer(sch)
    S = count * 4
    return {"bucket_bytes": S, "round_us_median": round(t * 1e6, 1),
            "value_GBs": round(world * S / t / 1e9, 3), "rounds": iters,
            "parity": "bitwise" if ok else "MISMATCH", "rank0_stages_us": stages}


def small_round_after_idle(comm, dev, rank, world, count=16384, iters=30, idle_s=0.002):
    """A 64 KiB majority round after every rank has been idle for `idle_s` (the training
    pattern: buckets are posted once per backward pass, the progress threads sleep in
    between), post -> wait, max over ranks, median.  Compare with C5's back-to-back
    64 KiB round: the difference is the cost of waking up."""
    import statistics

    import torch
    import torch.distributed as dist
    buf = dev.DeviceBuffer(count)
    dev.fill_uniform(buf, SEED, rank)
    dev.synchronize()
    sch = comm.Schedule(comm.MAJORITY, None, buf, count, seed=6545343, buf=comm.BUF_DEVICE)
    for _ in range(5):
        sch.post(); sch.wait()
    ts = []
    for _ in range(iters):
        comm.barrier()
        time.sleep(idle_s)
        t0 = time.perf_counter()
        sch.post(); sch.wait()
        ts.append(time.perf_counter() - t0)
    tt = torch.tensor(ts, dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    stages = _stages_us(sch.timeline()[-iters:])
    _defer(sch, buf)
    return {"bucket_bytes": count * 4, "idle_ms": idle_s * 1e3,
            "us": round(statistics.median(tt.tolist()) * 1e6, 1), "rounds": iters,
            "rank0_stages_us": stages}


def c3_host_buckets(comm, dev, rank, world, count, steps=8):
    """C3 on the reference's own contract: the bucket lives in host memory (the wrapper's
    calloc'd buckets, opt_esgd_solo_imagenet_imbalance.py:288-298), so each round is
    H2D -> reduce-scatter -> all-gather -> D2H.  The caller's array is pinned at schedule
    creation (hipHostRegister), so both copies are DMA."""
    import numpy as np

    from esgd._lib import check, lib
    from oracle import ffref
    host = np.empty(count, np.float32)
    sch = comm.Schedule(comm.SOLO, None, host, count, async_=32, seed=6545343, buf=comm.BUF_HOST)
    src = dev.DeviceBuffer(count)

    def refill(seed):
        dev.fill_uniform(src, seed, rank)
        check(lib().esgd_memcpy_async(host.ctypes.data, src.ptr, count * 4, 1, None))
        dev.synchronize()

    def step():
        sch.post()
        sch.wait()

    refill(SEED)
    for _ in range(2):
        step()
    t = _timed_steps(comm, step, steps)
    refill(SEED + 2)
    comm.barrier()
    step()
    m = min(count, 1 << 18)
    want = ffref.tree_sum([ffref.fill_uniform(SEED + 2, r, m, start=count - m) for r in range(world)])
    ok = bool(np.array_equal(host[count - m:].view(np.uint32), want.view(np.uint32)))
    _defer(sch, src)          # the schedule object keeps `host` alive
    S = count * 4
    return {"bucket_bytes": S, "round_ms_median": round(t * 1e3, 3),
            "value_GBs": round(world * S / t / 1e9, 2), "pcie_bytes_per_rank": 2 * S,
            "parity_tail_slice": "bitwise" if ok else "MISMATCH"}


def _stages_us(tl):
    """Median per-round host timeline of this rank (esgd_schedule_timeline), in us:
    post->join, join->launch, launch (host), launched->completion seen, ->wait returned."""
    import numpy as np
    tl = tl.astype(np.int64)
    tl = tl[(tl[:, 0] > 0) & (tl[:, 5] > 0)]
    if not len(tl):
        return None
    names = ["post_join", "join_launch", "launch_host", "gpu_round", "wake"]
    d = [tl[:, i + 1] - tl[:, i] for i in range(5)]
    out = {n: round(float(np.median(x)) / 1e3, 1) for n, x in zip(names, d)}
    if tl[:, 11].any():   # ESGD_GPU_TRACE=1: spans measured on the GPU
        gn = ["g_wait_ready", "g_rs", "g_wait_reduced", "g_ag", "g_wait_done"]
        out.update({n: round(float(np.median(tl[:, 6 + i])) / 1e3, 1) for i, n in enumerate(gn)})
    return out


def straggler_c4(comm, dev, rank, world, rounds=16, delay_fracs=(0.2, 2.0)):
    """C4: majority-allreduce of the ResNet-50 fused gradient (25 559 081 fp32,
    opt_esgd_solo_imagenet_imbalance.py:86-248 summed) with the last rank late every
    round by f x T (T = median no-straggler round; f = 0.2 is BASELINE.json's "delayed
    20 %", f = 2 a straggler slower than a whole round).  Gradients are 1.0, zeroed after
    use (evaluation/rsgd.c:87,100), so a round's result counts its fresh contributors.
    On-time ranks write theirs before the round's barrier, the straggler f x T after it.
    Reported per f: the contributor histogram over rounds, how many rounds the straggler
    activated (rand_r(6545343) % P, ffrand_allreduce.c:88) -- exactly those should take
    all P -- and the on-time ranks' post -> wait latency."""
    import collections
    import ctypes as C
    import statistics

    import numpy as np

    from esgd import _lib
    from esgd._lib import check, lib
    count = 25559081
    ones = dev.DeviceBuffer(count)
    ones.upload(np.ones(count, np.float32))
    sb, rb = dev.DeviceBuffer(count), dev.DeviceBuffer(count)
    sb.zero(); rb.zero()
    dev.synchronize()
    sch = comm.Schedule(comm.MAJORITY, sb, rb, count, dtype=_lib.FLOAT, seed=6545343,
                        buf=comm.BUF_DEVICE)
    hp = C.c_void_p()   # pinned result cell
    check(lib().esgd_host_alloc(C.byref(hp), 64))
    cell = np.ctypeslib.as_array(C.cast(hp, C.POINTER(C.c_float)), shape=(1,))
    late = rank == world - 1

    def fill():
        check(lib().esgd_memcpy_async(sb.ptr, ones.ptr, count * 4, 2, None))
        dev.synchronize()

    def one(delay):
        """-> (post-to-wait seconds, contributors, the straggler's achieved delay).  The
        delay is a spin to a perf_counter deadline (time.sleep cannot do tens of us) and then
        the late gradient's write; the achieved one is measured from the barrier to the post."""
        if not (late and delay):
            fill()
        comm.barrier()
        tb = time.perf_counter()
        if late and delay:   # wait to the deadline (asleep but for the last 2 ms, then a spin:
            while True:      # a spinning thread would starve this rank's progress thread),
                left = tb + delay - time.perf_counter()   # then the late gradient is written
                if left <= 0:
                    break
                if left > 2e-3:
                    time.sleep(left - 2e-3)
            fill()
        t0 = time.perf_counter()
        achieved = t0 - tb
        sch.post()
        sch.wait()
        dt_ = time.perf_counter() - t0
        check(lib().esgd_memcpy_async(cell.ctypes.data, rb.ptr, 4, 1, None))
        check(lib().esgd_memset_async(sb.ptr, 0, count * 4, None))
        dev.synchronize()
        c = float(cell[0])
        comm.barrier()
        return dt_, c, achieved

    base = [one(0.0)[0] for _ in range(12)]
    T = _max_over_ranks(statistics.median(base))
    out = {"bucket_fp32": count, "world": world, "T_no_straggler_ms": round(T * 1e3, 3)}
    for f in delay_fracs:
        first = sch.stats()["joined"] + 1
        lat, contrib, ach = [], [], []
        for _ in range(rounds):
            d, c, a = one(f * T)
            lat.append(d); contrib.append(c); ach.append(a)
        log = [e for e in sch.log() if first <= e["round"] < first + rounds]
        by_straggler = sum(1 for e in log if e["activator"] == world - 1)
        want = [world if e["activator"] == world - 1 else world - 1 for e in log]
        on_time = _max_over_ranks(statistics.median(lat) if not late else 0.0)
        out[f"delay_{f:g}T"] = {
            "straggler_delay_requested_ms": round(f * T * 1e3, 3),
            # the straggler's own measurement (the median over its rounds), shared by all ranks
            "straggler_delay_achieved_ms": round(_max_over_ranks(statistics.median(ach) if late else 0.0) * 1e3, 3),
            "contributors_histogram": {str(int(k)): v for k, v in sorted(collections.Counter(contrib).items())},
            "mean_contributors": round(float(np.mean(contrib)), 3),
            "rounds": rounds, "rounds_activated_by_straggler": by_straggler,
            "rounds_matching_partial_semantics": int(sum(int(a == b) for a, b in zip(want, contrib))),
            "on_time_ranks_median_ms": round(on_time * 1e3, 3)}
    _defer(sch, ones, sb, rb)
    check(lib().esgd_host_free(hp))
    return out


def run_allreduce(args, rank, world):
    """N > 1: one persistent schedule per rank over a device-resident bucket (config C3:
    256 MiB fp32, solo-allreduce), in place, all ranks posting every step.  Timed
    region: barrier + device sync, K x (post, wait), device sync, barrier; the MAX over
    ranks is the step time."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from esgd import _lib, comm
    from esgd import device as dev
    from oracle import ffref

    import datetime
    os.environ.setdefault("ESGD_TIMEOUT_S", "60")    # a stuck peer fails the run, not hangs it
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=180))
    comm.init(rank=rank, world=world)            # job id broadcast over gloo
    if args.transport:
        comm.set_transport(args.transport)
    # ranks sharing a GPU (a 1-GPU rehearsal of the N > 1 path) move HBM bytes, not xGMI
    # bytes: no xGMI fraction or roofline can be claimed for them
    import ctypes as C
    from esgd._lib import check, lib
    mydev = C.c_int()
    check(lib().esgd_get_device(C.byref(mydev)))
    devs = [None] * world
    dist.all_gather_object(devs, mydev.value)
    global SHARED_GPU
    SHARED_GPU = len(set(devs)) < world
    dt = _lib.FLOAT if args.dtype == "fp32" else _lib.BF16
    es = _lib.dtype_size(dt)
    count = int(args.bucket_mib * MiB) // es
    kind = {"solo": comm.SOLO, "majority": comm.MAJORITY, "allreduce": comm.ALLREDUCE}[args.schedule]

    def headline():
        """The timed C3 rounds on the current transport, then a parity round."""
        rb = dev.DeviceBuffer(count, dt)
        dev.fill_uniform(rb, SEED, rank)
        dev.synchronize()
        sched = comm.Schedule(kind, None, rb, count, dtype=dt, async_=32, seed=6545343,
                              buf=comm.BUF_DEVICE)

        def step():
            sched.post()
            sched.wait()

        for _ in range(args.warmup):
            step()
        dist.barrier(); comm.barrier(); dev.device_synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        dev.device_synchronize()
        dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        wall = float(el.item())
        out = {"wall": wall, "stats": sched.stats(), "stages": _stages_us(sched.timeline()[-args.steps:])}
        # parity outside the timed region: fresh inputs, one round, slices vs the oracle
        out["parity"] = "skipped"
        if dt == _lib.FLOAT:
            dev.fill_uniform(rb, SEED + 1, rank)
            dev.synchronize()
            comm.barrier()
            step()
            got = rb.download()
            m = min(count, 1 << 18)
            ok = True
            for start in (0, count - m):
                xs = [ffref.fill_uniform(SEED + 1, r, m, start=start) for r in range(world)]
                want = ffref.tree_sum(xs)
                ok &= bool(np.array_equal(got[start:start + m].view(np.uint32), want.view(np.uint32)))
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            out["parity"] = "bitwise (head+tail slices, every rank)" if flag.item() else "MISMATCH"
        _defer(sched, rb)
        return out

    # The headline runs on the default transport (IPC pull).  Should it fail on this node
    # (the IPC data plane has not crossed xGMI before the driver's first 8-GPU run), every
    # rank learns it through gloo and the line is measured over RCCL instead, saying so,
    # rather than ending the run without a line.
    transport = args.transport or os.environ.get("ESGD_TRANSPORT") or "ipc"
    fallback = None
    try:
        h, failed = headline(), 0
    except Exception as e:   # noqa: BLE001 -- reported in the line
        import traceback
        traceback.print_exc()
        h, failed, err = None, 1, f"rank {rank}: {e!r}"[:300]
    flag = torch.tensor([failed], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    if flag.item():
        import esgd
        if transport == "rccl" or world > esgd.device_count():
            raise RuntimeError("C3 headline failed on " + transport)
        errs = [None] * world
        dist.all_gather_object(errs, err if failed else None)
        fallback = {"from": transport, "errors": [e for e in errs if e]}
        comm.set_transport("rccl")
        transport = "rccl"
        h = headline()
    wall, stats, stages, parity = h["wall"], h["stats"], h["stages"], h["parity"]
    t_step = wall / args.steps

    S = count * es
    algbw = S / t_step / 1e9
    busbw = algbw * 2 * (world - 1) / world
    t_min = 2 * S / (world * XGMI_LINK_GBS * 1e9)
    link_in = 2 * (world - 1) / world * S / t_step / 1e9     # bytes each GPU pulls per second
    line = {
        "metric": "GB/s grad-bucket reduced (device-resident), solo/majority-allreduce 1-8 GPU",
        "value": round(world * S * args.steps / wall / 1e9, 2),
        "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.dtype == "fp32" else "bf16 (f32 accumulate)",
        "data": "synthetic (splitmix64 uniform [-1,1), generated on device)",
        "config": {"workload": f"C3: {args.schedule}-allreduce of one {args.bucket_mib:g} MiB "
                               f"{args.dtype} bucket per GPU, in place",
                   "bucket_bytes": S,
                   # what ran, from the ranks' devices: a 1-GPU rehearsal is labelled as one
                   **run_labels(world, devs, transport)},
        "algbw_GBs": round(algbw, 2), "busbw_GBs": round(busbw, 2),
        "xgmi_frac": None if SHARED_GPU else round(t_min / t_step, 4),
        "roofline": None if SHARED_GPU else {
            "bound": "xgmi", "achieved": round(link_in, 2), "peak": XGMI_LINK_GBS * (world - 1),
            "unit": "GB/s", "frac": round(link_in / (XGMI_LINK_GBS * (world - 1)), 4), "traffic": None},
        "devices": devs,
        "launcher": ("bench.py (self-launched torch.distributed.run)" if os.environ.get("ESGD_BENCH_SELF_LAUNCHED")
                     else "torch.distributed.run"),
        "rounds": {"fresh": stats["fresh_rounds"], "auto": stats["auto_rounds"],
                   "activations_rank0": stats["activations"]},
        "rank0_stages_us": stages,
        "parity": parity,
    }
    if fallback:
        line["headline_fallback"] = fallback
        args.no_extras = True   # the extra legs run on the IPC data plane that just failed
    if SHARED_GPU:
        line["rehearsal"] = "ranks share a GPU (HBM, not xGMI): no xGMI fraction or roofline"

    # The extra legs (C5 sweeps, C4, RCCL) run under a watchdog: if one hangs, rank 0
    # still prints the headline line with the legs finished so far, and every rank leaves.
    extras = {}
    if not args.no_extras:
        import threading

        def give_up(leg):
            if rank == 0:
                out = dict(line)
                out.update(extras)
                out["extras_timeout"] = leg[0]
                emit(out)
            os._exit(0)

        leg = ["none"]
        budget = float(os.environ.get("ESGD_BENCH_EXTRAS_S", "420"))
        dog = threading.Timer(budget, give_up, args=(leg,))
        dog.daemon = True
        dog.start()
        # both C5 sweeps first: the C4 legs leave 160+ schedules (and their peer mappings)
        # alive until the end, and small rounds measured after them were bimodal
        legs = [("sweep_c5_majority", lambda: sweep_c5(comm, dev, world, dt, es)),
                ("sweep_c5_majority_bf16", lambda: sweep_c5(comm, dev, world, _lib.BF16, 2)),
                ("ab_one_launch_threshold", lambda: ab_one_launch_threshold(comm, dev, world)),
                ("c3_wire_bf16", lambda: c3_wire_bf16(comm, dev, rank, world, int(args.bucket_mib * MiB) // 4)),
                ("c1_host_majority", lambda: c1_host_majority(comm, dev, rank, world)),
                ("small_round_after_idle", lambda: small_round_after_idle(comm, dev, rank, world)),
                ("straggler_c4_majority", lambda: straggler_c4(comm, dev, rank, world)),
                ("c4_resnet50_161_vs_fused", lambda: c4_resnet50_161(comm, dev, rank, world)),
                ("optimizer_resnet50_161", lambda: optimizer_resnet50_161(comm, rank, world)),
                ("c3_host_buckets", lambda: c3_host_buckets(comm, dev, rank, world,
                                                                  int(args.bucket_mib * MiB) // 4))]
        if os.environ.get("ESGD_BENCH_RCCL", "1") == "1":
            legs.append(("c3_rccl_transport", lambda: c3_over_rccl(comm, dev, rank, world, count)))
            legs.append(("rccl_as_default_c3_c4", lambda: rccl_as_default_c3_c4(
                comm, dev, rank, world, count, round(t_step * 1e3, 4), extras.get("straggler_c4_majority"))))
        # last: device flag pages have never run across GPUs; a hang there costs the
        # round timeout, and no other leg is lost to it
        legs.append(("ab_flag_pages", lambda: ab_flag_pages(comm, dev, world)))
        only = os.environ.get("ESGD_BENCH_LEGS")   # comma-separated subset, in this order
        if only:
            pick = only.split(",")
            legs = sorted((lg for lg in legs if lg[0] in pick), key=lambda lg: pick.index(lg[0]))
        legs_s = extras["legs_s"] = {}      # wall time of each leg on rank 0's clock
        for name, fn in legs:
            leg[0] = name
            t_leg = time.perf_counter()
            try:
                extras[name] = fn()
            except Exception as e:   # keep the headline line; report what failed
                import traceback
                traceback.print_exc()
                extras[name + "_error"] = f"rank {rank}: " + repr(e)[:300]
                break                # peers may be inside this leg: do not start another
            finally:
                legs_s[name] = round(time.perf_counter() - t_leg, 2)
        leg[0] = "teardown"
        if not any(k.endswith("_error") for k in extras):
            _delete_deferred()       # collective; after a failed leg finalize frees them
        comm.finalize()
        dog.cancel()
    else:
        _delete_deferred()
        comm.finalize()
    line.update(extras)
    opt_leg, c4_leg = extras.get("optimizer_resnet50_161"), extras.get("c4_resnet50_161_vs_fused")
    if isinstance(opt_leg, dict) and isinstance(c4_leg, dict) and c4_leg.get("step_ms_161_buckets_pipelined"):
        # the drop-in caller path against the data plane beneath it, same job (VERDICT r04
        # item 2): the bare in-place rounds, and the rounds with the op's schedule properties
        # (separate send bucket, HOLD, FRESH_ONLY, group calls)
        bare = c4_leg["step_ms_161_buckets_pipelined"]
        op_like = (c4_leg.get("op_like_pipelined_variants", {}).get("separate_sb_hold_fresh_group") or {}).get("step_ms")
        pt = opt_leg.get("per_tensor_pipelined_ms")
        line["caller_vs_data_plane"] = {
            "per_tensor_pipelined_ms": pt, "rounds_161_in_place_ms": bare, "rounds_161_op_like_ms": op_like,
            "per_tensor_over_in_place": round(pt / bare, 3) if pt else None,
            "per_tensor_over_op_like": round(pt / op_like, 3) if pt and op_like else None,
            "fused_ms": opt_leg.get("fused_ms")}
    dist.destroy_process_group()
    return line


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.pmc_child:
        sys.exit(launch_ranks(args))   # before any HIP call in this process
    if args.bucket_mib is None:
        args.bucket_mib = 64.0 if args.gpus == 1 else 256.0
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not args.pmc_child:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    if world > 1:
        _quiet_stdout()

    import esgd
    from esgd import device as dev
    ndev = esgd.device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no HIP device visible")
    # one rank per GPU; extra ranks wrap around (1-GPU rehearsal of the N>1 path)
    esgd.check(esgd.lib().esgd_set_device(local_rank % ndev), "esgd_set_device")

    if world > 1:
        res = run_allreduce(args, rank, world)
        if rank == 0:
            emit(res)
        return

    res = run_local(args, esgd, dev)
    if args.pmc_child:
        return
    line = {
        "metric": "GB/s grad-bucket reduced (device-resident), solo/majority-allreduce 1-8 GPU",
        "value": round(res["value"], 2),
        "unit": "GB/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(res["ms_per_step"], 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.dtype == "fp32" else "bf16 (f32 accumulate)",
        "data": "synthetic (splitmix64 uniform [-1,1), generated on device)",
        "config": {"workload": f"C2: local reduction of {res['k']} staged "
                               f"{args.bucket_mib:g} MiB {args.dtype} buckets -> 1 (tree order)",
                   "buckets": res["k"], "bucket_bytes": res["bucket_bytes"],
                   "parallelism": "single GPU", "kernel": "esgd_reduce (k_tree_sum)"},
        "parity": res["parity"],
    }
    if res.get("gate"):
        line["gate_256MiB"] = res["gate"]
    if res.get("host_e2e"):
        line["host_e2e"] = res["host_e2e"]
    traffic = None
    if _under_profiler():
        # an outer rocprofv3 already traces this process: a nested profiler child would
        # inherit its environment (a profiler-preloaded launcher re-exec'ing python, which
        # this pool forbids) and its data would be meaningless
        args.no_pmc = args.no_trace = True
        line["profiler_passes"] = "skipped: bench.py runs under a profiler"
    if not args.no_pmc:
        try:
            traffic = pmc_traffic(args, args.bucket_mib)
            if res.get("gate"):
                res["gate"]["traffic"] = pmc_traffic(args, 256.0)
        except Exception as e:  # profiler missing or refused: report, keep the line
            line["pmc_error"] = str(e)[:200]
    trace = None
    if not args.no_trace:
        try:
            trace = kernel_trace(args)
        except Exception as e:  # profiler missing or refused: report, keep the line
            line["trace_error"] = str(e)[:200]
    if trace and res.get("gate"):
        res["gate"]["rocprof_call_us"] = trace["gate_8x256MiB"]["avg_us"]
        res["gate"]["rocprof_frac"] = trace["gate_8x256MiB"]["frac_of_8TBs"]
    line["roofline"] = {
        "bound": "hbm", "achieved": round(res["achieved_gbs"], 1), "peak": HBM_PEAK_GBS,
        "unit": "GB/s", "frac": round(res["achieved_gbs"] / HBM_PEAK_GBS, 4),
        "traffic": traffic, "algo_bytes_per_launch": res["algo_bytes"],
        "kernel_ms": round(res["kernel_ms"], 5),
        "kernel_ms_all_launches": round(res["kernel_ms_all"], 5),
        # the north star's 1-GPU gate: 8 x 256 MiB fp32 buckets, same kernel, same timing
        "gate_256MiB_frac": res["gate"]["frac"] if res.get("gate") else None,
        # the same kernel's average dispatch on this box from rocprofv3 --kernel-trace
        # (profiles/r03/: bench_kernel_trace_split.json); the event pair above also holds
        # the dispatch gap between back-to-back launches
        "rocprof_kernel_us": trace["C2"]["avg_us"] if trace else None,
        "rocprof_frac": trace["C2"]["frac_of_8TBs"] if trace else None,
    }
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(res["k"], res["count"] if args.dtype == "fp32"
                                            else res["count"])
        line["cpu_baseline_c1"] = cpu_baseline_c1()
    emit(line)


if __name__ == "__main__":
    main()
