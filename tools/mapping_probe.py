#!/usr/bin/env python3
"""Which IPC mapping goes wrong after a refused export (round 5, r05b: a simulated refusal on
rank 0 -- seal written, runtime call refused -- and then rank 0's mapping of rank 1's
first slab showed rank 0's OWN next exported chunk; the seal caught it).  Runs small
2-rank jobs (mp_workers.gpu_allreduce) over a grid of (count, batching, refusals) a few
times each, every export / open logged with its 64 handle bytes (ESGD_IPC_TRACE_FILE, one
file per job), and prints one JSON line per job: the outcome and the handles each rank
exported and opened, decoded into 8-byte words.
  python tools/mapping_probe.py <outdir> [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eager-sgd_amd"), os.path.join(ROOT, "tests")]

import mp_workers  # noqa: E402


def words(h):
    b = bytes.fromhex(h)
    return [hex(int.from_bytes(b[i:i + 8], "little")) for i in range(0, 64, 8)]


def parse(path):
    rows = []
    if not os.path.exists(path):
        return rows
    with open(path) as f:
        for line in f:
            p = line.split()
            if len(p) < 12 or p[0] != "esgd-ipc":
                continue
            rows.append({"pid": int(p[2]), "what": p[3], "peer": int(p[5]), "ptr": p[7], "bytes": int(p[9]),
                         "handle": words(p[11])})
    return rows


if __name__ == "__main__":
    out = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    os.makedirs(out, exist_ok=True)
    grid = [(17, 0, (1, 0)), (17, None, (1, 0)), (1, 0, (1, 0)), (4099, 0, (1, 0)), (17, 0, (0, 1)),
            (17, 0, (0, 0)), (17, 0, (2, 0))]
    for rep in range(reps):
        for count, batch, fails in grid:
            tag = f"{rep}_{count}_{batch}_{fails[0]}{fails[1]}"
            trace = os.path.join(out, f"trace_{tag}.log")
            os.environ["ESGD_IPC_TRACE_FILE"] = trace
            try:
                v = mp_workers.run("gpu_allreduce", 2, count=count, rounds=2, fail_exports=fails, batch=batch,
                                   timeout=120)
                status = "ok" if all(all(x) for x in v) else "wrong: " + json.dumps(v)[:400]
            except AssertionError as e:
                s = str(e)
                status = ("seal_mismatch: " if "other memory" in s else "error: ") + s.splitlines()[-1][:300]
            print(json.dumps({"rep": rep, "count": count, "batch": batch, "fails": fails, "status": status,
                              "ipc": parse(trace)}), flush=True)
