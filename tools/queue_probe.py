#!/usr/bin/env python3
"""Which hardware queue does each dispatch of the blocking per-tensor path use?  Runs
mp_workers.op_queue_probe at 2 ranks under AMD_LOG_LEVEL=4 with and without one extra
torch stream (round 4: a third hardware queue per process made this path 2x faster on a
GPU shared by the ranks); each rank's runtime log goes to
<out>/log_side<0|1>.txt, and per kernel name the distinct HWq values are printed.
  python tools/queue_probe.py <out>"""
import collections
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    for side in (0, 1):
        log = os.path.join(out, f"log_side{side}.txt")
        code = ("import sys; sys.path[:0] = ['tests', 'eager-sgd_amd']\n"
                "from mp_workers import run\n"
                f"print(run('op_queue_probe', 2, side={bool(side)}, timeout=300))\n")
        env = dict(os.environ, AMD_LOG_LEVEL="4")
        with open(log, "w") as f:
            r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                               stderr=f, text=True, timeout=400)
        queues = collections.defaultdict(set)
        pat = re.compile(r"HWq=(0x[0-9a-f]+).*")
        last_q = None
        for line in open(log, errors="replace"):
            m = pat.search(line)
            if m:
                last_q = m.group(1)
            k = re.search(r"ShaderName : (\S+)", line)
            if k and last_q:
                queues[k.group(1)[:60]].add(last_q)
        print(json.dumps({"side": side, "result": r.stdout.strip()[-300:],
                          "kernel_queues": {k: sorted(v) for k, v in queues.items()}}), flush=True)


if __name__ == "__main__":
    main()
