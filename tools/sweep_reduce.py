#!/usr/bin/env python3
"""Interleaved A/B sweep of the reduction launch parameters in ONE process
(cdna_hip_programming.md §5.4 rule 24): every variant is timed once per round, for
several rounds, and the median/min per-launch time from HIP event pairs is reported.
The variants live in the tools-only library tools/bin/libesgd_sweeps.so (`make sweeps`,
tools/sweeps/reduce_sweeps.hip: fp32, fan-in 8); libesgd.so carries only the production
launch (policy -1 here).

  python tools/sweep_reduce.py [--mib 64] [--rounds 7] [--iters 30] [--policies -1,0,17]
"""
import argparse
import ctypes as C
import itertools
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "eager-sgd_amd"))
sys.path.insert(0, ROOT)

import esgd  # noqa: E402
from esgd import device as dev  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=8, choices=[8], help="fan-in (the sweep library is k = 8 only)")
ap.add_argument("--mib", type=float, default=64)
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--grids", default="0,1024,2048,4096,8192,16384")
ap.add_argument("--unrolls", default="2,4")
ap.add_argument("--nts", default="0,1")
ap.add_argument("--policies", default="-1")
ap.add_argument("--stagger", type=int, default=0,
                help="bytes between consecutive buckets in one arena (0 = separate allocations)")
a = ap.parse_args()
dt, es = esgd.FLOAT, 4
sw = C.CDLL(os.path.join(ROOT, "tools", "bin", "libesgd_sweeps.so"))
sw.esgd_sweep_reduce.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p), C.c_void_p,
                                 C.c_uint64, C.c_void_p]
sw.esgd_sweep_last_error.restype = C.c_char_p
count = int(a.mib * (1 << 20)) // es
s = dev.Stream()
if a.stagger:
    pitch = count * es + a.stagger
    arena = dev.DeviceBuffer((pitch * (a.k + 1)) // es + 1, dt)
    ptrs = [arena.ptr + r * pitch for r in range(a.k)]
    out = arena.ptr + a.k * pitch
    for r, p in enumerate(ptrs):
        esgd.check(esgd.lib().esgd_fill_uniform_f32(0x5EEDE56D, r, p, count, s.handle))
else:
    bufs = [dev.DeviceBuffer(count, dt) for _ in range(a.k)]
    for r, b in enumerate(bufs):
        dev.fill_uniform(b, 0x5EEDE56D, r, stream=s)
    out = dev.DeviceBuffer(count, dt)
    ptrs = [b.ptr for b in bufs]
s.synchronize()
variants = list(itertools.product([int(x) for x in a.unrolls.split(",")],
                                  [int(x) for x in a.nts.split(",")],
                                  [int(x) for x in a.grids.split(",")],
                                  [int(x) for x in a.policies.split(",")]))
# every variant's output must be the production variant's, bit for bit
import numpy as np  # noqa: E402
pa = (C.c_void_p * 8)(*ptrs)
optr = out if a.stagger else out.ptr


def run(v):
    u, nt, g, pol = v
    if sw.esgd_sweep_reduce(pol, u, nt, g, pa, optr, count, s.handle):
        raise RuntimeError(sw.esgd_sweep_last_error().decode())


# Every variant's output is checked against the ORACLE (ffref.tree_sum of the same
# splitmix buckets) before anything is timed; a variant that differs is reported with its
# bad byte count and never timed -- no sweep number can come from a wrong answer.
from oracle import ffref  # noqa: E402
want = ffref.tree_sum([ffref.fill_uniform(0x5EEDE56D, r, count) for r in range(a.k)])


def download_out():
    if not a.stagger:
        return out.download()
    host = np.empty(count, np.float32)
    esgd.check(esgd.lib().esgd_memcpy_async(host.ctypes.data, out, count * es, 1, s.handle), "d2h")
    s.synchronize()
    return host


bad = {}
for v in variants:
    esgd.check(esgd.lib().esgd_memset_async(optr, 0, count * es, s.handle), "memset")
    run(v)
    s.synchronize()
    nbad = int(np.count_nonzero(download_out().view(np.uint8) != want.view(np.uint8)))
    if nbad:
        bad[v] = nbad
good = [v for v in variants if v not in bad]
ev = [dev.Event() for _ in range(2 * a.iters)]
times = {v: [] for v in good}
for rnd in range(a.rounds):
    for v in good:
        for _ in range(3):
            run(v)
        for i in range(a.iters):
            ev[2 * i].record(s)
            run(v)
            ev[2 * i + 1].record(s)
        s.synchronize()
        times[v].extend(ev[2 * i].elapsed_ms(ev[2 * i + 1]) for i in range(a.iters))
algo = (a.k + 1) * count * es
rows = [{"unroll": v[0], "nt": v[1], "grid": v[2], "policy": v[3], "bad_bytes": n, "timed": False}
        for v, n in bad.items()]
for v, t in times.items():
    med, mn = statistics.median(t), min(t)
    rows.append({"unroll": v[0], "nt": v[1], "grid": v[2], "policy": v[3], "bad_bytes": bad.get(v, 0),
                 "median_us": round(med * 1e3, 2),
                 "min_us": round(mn * 1e3, 2), "median_GBs": round(algo / (med * 1e-3) / 1e9, 1),
                 "frac_of_8TBs": round(algo / (med * 1e-3) / 8e12, 4)})
rows.sort(key=lambda r: r.get("median_us", float("inf")))
for r in rows:
    r.update(k=a.k, mib=a.mib, stagger=a.stagger)
    print(json.dumps(r))
