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
CASES = [  # (alloc MiB, use MiB, offset MiB)
    (256, 256, 0),
    (1024, 256, 0),
    (1024, 256, 768),
    (1024, 1024, 0),
    (512, 512, 0),
]
dt, k = esgd.FLOAT, 8
s = dev.Stream()
sets = {}
for alloc in sorted({c[0] for c in CASES}):
    bufs = [dev.DeviceBuffer(alloc * MiB // 4, dt) for _ in range(k + 1)]
    for r, b in enumerate(bufs[:k]):
        dev.fill_uniform(b, 0x5EEDE56D, r, stream=s)
    sets[alloc] = bufs
s.synchronize()
e0, e1 = dev.Event(), dev.Event()
times = {c: [] for c in CASES}
for _ in range(7):
    for c in CASES:
        alloc, use, off = c
        bufs = sets[alloc]
        ptrs = [b.ptr + off * MiB for b in bufs[:k]]
        out = bufs[k].ptr + off * MiB
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
