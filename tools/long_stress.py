#!/usr/bin/env python3
"""Long runs of the randomized activation stress (tests/mp_workers.gpu_stress_fresh):
HOLD | FRESH_ONLY schedules, gradients written in the wrapper's racy order, random delays,
no barriers; every round checked (shares = tag iff the rank had posted the round, else 0;
no torn buckets; every rank sees the same result).  One JSON line per configuration.
  python tools/long_stress.py [--rounds 5000]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eager-sgd_amd"), os.path.join(ROOT, "tests")]

from mp_workers import run  # noqa: E402

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5000)
    ap.add_argument("--device-flags", default=None, help="ESGD_DEVICE_FLAGS for every rank (1 or 2)")
    ap.add_argument("--configs", default=None, help="world:count:buf,... (default: the four of the suite)")
    ap.add_argument("--pipelined", default=None,
                    help="world:batch,... -- the batched per-tensor stress (mp_workers.gpu_stress_pipelined: "
                         "8 HOLD | FRESH_ONLY schedules posted at once every step; batch: rounds per shared "
                         "launch, 'mix' = 64/0/5/2 by rank) instead of the one-schedule stress")
    ap.add_argument("--strict", type=int, default=0, help="ESGD_STRICT_HANDOFFS for every rank")
    ap.add_argument("--fail-exports", default=None,
                    help="per rank, comma-separated: that many of its first chunk exports fail (the runtime's refusals)")
    ap.add_argument("--kinds", default="solo,majority")
    ap.add_argument("--diag-dir", default=os.path.join(ROOT, "gpurun_out", "long_stress_diag"),
                    help="every rank's step every 50 steps (progress.txt) and Python stacks every 60 s "
                         "(stacks/): a stall leaves evidence, and a slow run keeps writing")
    a = ap.parse_args()
    os.environ["ESGD_STRICT_HANDOFFS"] = str(a.strict)
    if a.diag_dir:   # inherited by the spawned ranks (r06p: a run silent for 180 s left nothing)
        os.makedirs(a.diag_dir, exist_ok=True)
        os.environ.setdefault("ESGD_PROGRESS_FILE", os.path.join(a.diag_dir, "progress.txt"))
        os.environ.setdefault("ESGD_HANG_DUMP_DIR", os.path.join(a.diag_dir, "stacks"))
        os.environ.setdefault("ESGD_HANG_DUMP_S", "60")
    if a.pipelined:
        return pipelined(a)
    if a.device_flags:
        os.environ["ESGD_DEVICE_FLAGS"] = a.device_flags   # inherited by the spawned ranks
    configs = ((3, 65536, "device"), (3, (1 << 20) + 3, "device"), (8, 65536, "device"), (3, 65536, "host"))
    if a.configs:   # world:count:buf,...
        configs = tuple((int(w), int(c), b) for w, c, b in (x.split(":") for x in a.configs.split(",")))
    for world, count, buf in configs:
        for kind, kname in ((1, "solo"), (2, "majority")):
            t0 = time.time()
            outs = run("gpu_stress_fresh", world, kind=kind, count=count, rounds=a.rounds, buf=buf, timeout=900)
            bits = outs[0]["bits"]
            bad = sum(len(o["torn"]) for o in outs) + sum(o["vals"] != outs[0]["vals"] for o in outs)
            for t in range(1, a.rounds + 1):
                v = outs[0]["vals"][t - 1]
                for q in range(world):
                    want = t % (1 << bits) if outs[q]["fresh"][t - 1] else 0
                    bad += ((v >> (bits * q)) & ((1 << bits) - 1)) != want
            print(json.dumps({"world": world, "count": count, "buf": buf, "kind": kname, "rounds": a.rounds,
                              "device_flags": a.device_flags or "0 (host flags)",
                              "bad": int(bad), "auto_rounds": sum(o["stats"]["auto_rounds"] for o in outs),
                              "fresh_rounds": sum(o["stats"]["fresh_rounds"] for o in outs),
                              "wall_s": round(time.time() - t0, 1)}), flush=True)


def pipelined(a):
    for cfg in a.pipelined.split(","):
        w, b = cfg.split(":")
        world = int(w)
        batch = None if b == "default" else ([64, 0, 5, 2] * 2)[:world] if b == "mix" else int(b)
        fails = [int(x) for x in a.fail_exports.split(",")][:world] if a.fail_exports else None
        for kind, kname in ((1, "solo"), (2, "majority")):
            if kname not in a.kinds.split(","):
                continue
            t0 = time.time()
            outs = run("gpu_stress_pipelined", world, kind=kind, rounds=a.rounds, batch=batch, timeout=900,
                       fail_exports=fails)
            bits = outs[0]["bits"]
            bad = sum(len(o["torn"]) for o in outs) + sum(o["vals"] != outs[0]["vals"] for o in outs)
            for i in range(len(outs[0]["vals"])):
                for t in range(1, len(outs[0]["vals"][i]) + 1):
                    v = outs[0]["vals"][i][t - 1]
                    for q in range(world):
                        want = t % (1 << bits) if outs[q]["fresh"][i][t - 1] else 0
                        bad += ((v >> (bits * q)) & ((1 << bits) - 1)) != want
            print(json.dumps({"stress": "pipelined", "world": world, "batch": b, "kind": kname,
                              "steps": a.rounds, "rounds": a.rounds * len(outs[0]["vals"]),
                              "strict": a.strict, "fail_exports": a.fail_exports, "bad": int(bad), "auto_rounds": sum(o["auto_rounds"] for o in outs),
                              "wall_s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":   # spawned workers re-import this module
    main()
