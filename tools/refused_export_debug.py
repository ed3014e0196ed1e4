#!/usr/bin/env python3
"""One-off diagnostics for a refused export on one rank (ESGD_FAIL_EXPORTS on rank 1):
every round's first wrong element with got / want / inputs, for the batched and the
one-launch-per-round data plane, with ESGD_DEBUG=1 tracing the setup path.
  python tools/refused_export_debug.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eager-sgd_amd"), os.path.join(ROOT, "tests")]

import mp_workers  # noqa: E402

if __name__ == "__main__":
    os.environ["ESGD_DEBUG"] = "1"
    for count in (1, 17, 4099):
        for batch in (None, 0):
            for fails in ((0, 2), (0, 1), (2, 0)):
                outs = mp_workers.run("gpu_allreduce", 2, count=count, rounds=3, fail_exports=fails, batch=batch,
                                      detail=True)
                print(json.dumps({"count": count, "batch": batch, "fails": fails, "verdicts": outs}), flush=True)
