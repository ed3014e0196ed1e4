#!/usr/bin/env python3
"""esgd_reduce_host at the C2 shape (8 pinned 64 MiB host buckets -> 1) for the chunk
size in ESGD_HOST_REDUCE_CHUNK (read once per process): one JSON line.
  for c in 1 2 4 8 16; do ESGD_HOST_REDUCE_CHUNK=$((c<<20)) python tools/host_reduce_sweep.py; done"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "eager-sgd_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from esgd import device as dev  # noqa: E402

s = dev.Stream()
r = bench.host_e2e(dev, 8, (64 << 20) // 4, s, iters=5)
r["mode"] = os.environ.get("ESGD_HOST_REDUCE_MODE", "auto (zero-copy)")
r["chunk"] = int(os.environ.get("ESGD_HOST_REDUCE_CHUNK", 4 << 20))
print(json.dumps(r))
