#!/usr/bin/env python3
"""Does a hipGraph close the dispatch gap between back-to-back C2 launches?

C2 (8 x 64 MiB fp32 -> 1) launched K times back to back on one stream, timed by one HIP
event pair around the K launches, against the same K launches captured once into a
hipGraph (stream capture, relaxed mode) and replayed.  Interleaved, several rounds; every
replay's output is checked against the stream launches' bit for bit.

  python tools/graph_probe.py [--launches 40] [--rounds 7]
"""
import argparse
import ctypes as C
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
ap.add_argument("--launches", type=int, default=40)
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--mib", type=float, default=64)
a = ap.parse_args()

hip = C.CDLL("libamdhip64.so")
for f in ("hipStreamBeginCapture", "hipStreamEndCapture", "hipGraphInstantiate", "hipGraphLaunch",
          "hipGraphExecDestroy", "hipGraphDestroy"):
    getattr(hip, f).restype = C.c_int


def ok(rc, what):
    if rc:
        raise RuntimeError(f"{what}: hip error {rc}")


dt, k = esgd.FLOAT, 8
count = int(a.mib * (1 << 20)) // 4
s = dev.Stream()
bufs = [dev.DeviceBuffer(count, dt) for _ in range(k)]
for r, b in enumerate(bufs):
    dev.fill_uniform(b, 0x5EEDE56D, r, stream=s)
out = dev.DeviceBuffer(count, dt)
ptrs = [b.ptr for b in bufs]
s.synchronize()
dev.reduce(dt, ptrs, out, count, stream=s)
s.synchronize()
ref = out.download()

graph, gexec = C.c_void_p(), C.c_void_p()
ok(hip.hipStreamBeginCapture(C.c_void_p(s.handle), 2), "hipStreamBeginCapture")
for _ in range(a.launches):
    dev.reduce(dt, ptrs, out, count, stream=s)
ok(hip.hipStreamEndCapture(C.c_void_p(s.handle), C.byref(graph)), "hipStreamEndCapture")
ok(hip.hipGraphInstantiate(C.byref(gexec), graph, None, None, C.c_size_t(0)), "hipGraphInstantiate")

out.zero(stream=s)
ok(hip.hipGraphLaunch(gexec, C.c_void_p(s.handle)), "hipGraphLaunch")
s.synchronize()
graph_bitwise = bool(np.array_equal(out.download().view(np.uint32), ref.view(np.uint32)))


def stream_launches():
    for _ in range(a.launches):
        dev.reduce(dt, ptrs, out, count, stream=s)


def graph_launch():
    ok(hip.hipGraphLaunch(gexec, C.c_void_p(s.handle)), "hipGraphLaunch")


e0, e1 = dev.Event(), dev.Event()
times = {"stream": [], "graph": []}
for _ in range(a.rounds):
    for name, fn in (("stream", stream_launches), ("graph", graph_launch)):
        fn()                       # warm
        s.synchronize()
        e0.record(s)
        fn()
        e1.record(s)
        s.synchronize()
        times[name].append(e0.elapsed_ms(e1) * 1e3 / a.launches)
# the floor: the same back-to-back launches over a 4 KiB bucket (one block, the kernel's
# own work ~nil) -- what every launch pays for dispatch, completion and cache maintenance
tiny = 1024
for _ in range(3):
    for _ in range(a.launches):
        dev.reduce(dt, ptrs, out, tiny, stream=s)
    s.synchronize()
    e0.record(s)
    for _ in range(a.launches):
        dev.reduce(dt, ptrs, out, tiny, stream=s)
    e1.record(s)
    s.synchronize()
    times.setdefault("stream_4KiB", []).append(e0.elapsed_ms(e1) * 1e3 / a.launches)
algo = (k + 1) * count * 4
for name, t in times.items():
    med = statistics.median(t)
    print(json.dumps({"mode": name, "launches": a.launches, "per_launch_us_median": round(med, 2),
                      "per_launch_us_min": round(min(t), 2), "frac_of_8TBs": None if name == "stream_4KiB" else round(algo / (med * 1e-6) / 8e12, 4),
                      "graph_bitwise": graph_bitwise}))
hip.hipGraphExecDestroy(gexec)
hip.hipGraphDestroy(graph)
