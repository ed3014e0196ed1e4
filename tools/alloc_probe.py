#!/usr/bin/env python3
"""Why do 8 x 1 GiB buckets reduce slower (~75 % of 8 TB/s) than 8 x 256 MiB (~81 %)?

Both run as the same 64 MiB window launches, so each launch touches the same 576 MiB.
This probe separates the allocation from the bytes touched: the production reduction
over `use` MiB of each of 9 buffers of `alloc` MiB, at byte offset `off` MiB inside
them, every case timed by one HIP event pair around back-to-back calls, interleaved over
rounds (median per call).

  python tools/alloc_probe.py
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "eager-sgd_amd"))

import esgd  # noqa: E402
from esgd import device as dev  # noqa: E402

MiB = 1 << 20
# (alloc MiB, use MiB, offset MiB); alloc < 0: the 9 buckets carved at a `use` pitch out
# of ONE allocation of -alloc MiB
CASES = [
    (256, 256, 0),
    (1024, 256, 0),
    (1024, 256, 768),
    (1024, 1024, 0),
    (512, 512, 0),
    (64, 64, 0),
    (256, 64, 0),
    (1024, 64, 0),
    (-576, 64, 0),
    (-1024, 64, 0),
    (-4096, 256, 0),
]
if len(sys.argv) > 1 and sys.argv[1] == "--c2":
    CASES = [c for c in CASES if c[1] == 64]
dt, k = esgd.FLOAT, 8
s = dev.Stream()
sets = {}
for alloc in sorted({c[0] for c in CASES if c[0] > 0}):
    bufs = [dev.DeviceBuffer(alloc * MiB // 4, dt) for _ in range(k + 1)]
    for r, b in enumerate(bufs[:k]):
        dev.fill_uniform(b, 0x5EEDE56D, r, stream=s)
    sets[alloc] = [b.ptr for b in bufs]
    sets[("keep", alloc)] = bufs
for alloc, use, _ in CASES:
    if alloc < 0 and alloc not in sets:
        one = dev.DeviceBuffer(-alloc * MiB // 4, dt)
        assert (k + 1) * use <= -alloc
        ptrs = [one.ptr + i * use * MiB for i in range(k + 1)]
        for r in range(k):
            esgd.check(esgd.lib().esgd_fill_uniform_f32(0x5EEDE56D, r, ptrs[r], use * MiB // 4, s.handle))
        sets[alloc] = ptrs
        sets[("keep", alloc)] = [one]
s.synchronize()
e0, e1 = dev.Event(), dev.Event()
times = {c: [] for c in CASES}
for _ in range(7):
    for c in CASES:
        alloc, use, off = c
        base = sets[alloc]
        ptrs = [p + off * MiB for p in base[:k]]
        out = base[k] + off * MiB
        count = use * MiB // 4
        calls = max(4, 2048 // use)
        for _ in range(2):
            dev.reduce(dt, ptrs, out, count, stream=s)
        e0.record(s)
        for _ in range(calls):
            dev.reduce(dt, ptrs, out, count, stream=s)
        e1.record(s)
        s.synchronize()
        times[c].append(e0.elapsed_ms(e1) * 1e3 / calls)
for c, t in times.items():
    alloc, use, off = c
    med = statistics.median(t)
    algo = (k + 1) * use * MiB
    print(json.dumps({"alloc_MiB": alloc, "use_MiB": use, "offset_MiB": off, "per_call_us": round(med, 1),
                      "per_64MiB_window_us": round(med * 64 / use, 2),
                      "frac_of_8TBs": round(algo / (med * 1e-6) / 8e12, 4)}))
