#!/usr/bin/env python3
"""Host-side cost of the per-tensor call pattern, no GPU: P processes (gloo rendezvous on
127.0.0.1), 161 control-plane-only schedules (ESGD_BUF_NONE: the engine's join / ticket /
issue-ring / completion path with a transport that moves nothing), every step posts all
of them and then waits for all (EagerSGDOptimizer's pipelined per-tensor order).  Prints
the median step and the last step's timeline on rank 0 (same fields as bench.py's
rank0_pipelined_step_us).

  python tools/host_engine_probe.py [--world 2] [--steps 50] [--kind 2]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--kind", type=int, default=2)
    ap.add_argument("--n", type=int, default=161)
    ap.add_argument("--idle", type=int, default=0, help="schedules kept alive and never posted")
    a = ap.parse_args()
    import mp_workers
    outs = mp_workers.run("cp_pipelined_steps", a.world, steps=a.steps, kind=a.kind, n=a.n, idle=a.idle)
    print(json.dumps(outs[0]))
