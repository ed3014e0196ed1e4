#!/usr/bin/env python3
"""Interleaved A/B in ONE process: the production tree kernel (8 inputs -> 1, fp32) over
separately allocated buckets vs the same buckets carved out of one allocation at a pitch
of S + stagger bytes (so that the k inputs' same-index bytes fall on different HBM
channels / banks).  Every layout's result is checked bit-exact against the first.
  python tools/stagger_ab.py [--mib 64] [--staggers 0,256,4096,65536,1052672]"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "eager-sgd_amd"))

import numpy as np  # noqa: E402

import esgd  # noqa: E402
from esgd import device as dev  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mib", type=float, default=64)
ap.add_argument("--k", type=int, default=8)
ap.add_argument("--staggers", default="256,4096,65536,1052672")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--inplace", type=int, default=1)
a = ap.parse_args()
k, count = a.k, int(a.mib * (1 << 20)) // 4
S = count * 4
s = dev.Stream()
layouts = {}
sep = [dev.DeviceBuffer(count) for _ in range(k + 1)]
layouts["separate"] = ([b.ptr for b in sep[:k]], sep[k].ptr)
if a.inplace:
    # the output is input 0 (the reference's rb = tmp + rb): its inputs change every launch,
    # so it is refilled before each timed block and not compared bitwise
    inp = [dev.DeviceBuffer(count) for _ in range(k)]
    layouts["inplace"] = ([b.ptr for b in inp], inp[0].ptr)
arenas = []
for st in [int(x) for x in a.staggers.split(",")]:
    pitch = S + st
    ar = dev.DeviceBuffer((pitch * (k + 1)) // 4 + 1024)
    arenas.append(ar)
    base = (ar.ptr + 255) // 256 * 256
    layouts[f"pitch+{st}"] = ([base + j * pitch for j in range(k)], base + k * pitch)
for name, (ins, out) in layouts.items():
    for r, p in enumerate(ins):
        esgd.check(esgd.lib().esgd_fill_uniform_f32(0x5EEDE56D, r, p, count, s.handle))
s.synchronize()
ref = None
bad = {}
for name, (ins, out) in layouts.items():
    if name == "inplace":
        bad[name] = -1
        continue
    dev.reduce(esgd.FLOAT, ins, out, count, stream=s)
    s.synchronize()
    host = np.empty(count, np.float32)
    esgd.check(esgd.lib().esgd_memcpy_async(host.ctypes.data, out, S, 1, s.handle))
    s.synchronize()
    if ref is None:
        ref = host
    bad[name] = int(np.count_nonzero(host.view(np.uint32) != ref.view(np.uint32)))
ev = [dev.Event() for _ in range(2 * a.iters)]
times = {n: [] for n in layouts}
for _ in range(a.rounds):
    for name, (ins, out) in layouts.items():
        if name == "inplace":
            esgd.check(esgd.lib().esgd_fill_uniform_f32(0x5EEDE56D, 0, ins[0], count, s.handle))
        for _ in range(3):
            dev.reduce(esgd.FLOAT, ins, out, count, stream=s)
        for i in range(a.iters):
            ev[2 * i].record(s)
            dev.reduce(esgd.FLOAT, ins, out, count, stream=s)
            ev[2 * i + 1].record(s)
        s.synchronize()
        times[name].extend(ev[2 * i].elapsed_ms(ev[2 * i + 1]) for i in range(a.iters))
algo = (k + 1) * S
print(json.dumps({"separate_ptr_deltas_bytes": [p - sep[0].ptr for p in layouts["separate"][0]]
                  + [layouts["separate"][1] - sep[0].ptr]}))
for name, t in times.items():
    med = statistics.median(t)
    print(json.dumps({"layout": name, "k": k, "mib": a.mib, "bad_bytes": bad[name],
                      "median_us": round(med * 1e3, 2), "min_us": round(min(t) * 1e3, 2),
                      "frac_of_8TBs": round(algo / (med * 1e-3) / 8e12, 4)}))
