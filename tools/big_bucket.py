"""ff.h's largest bucket (2^31 - 1 fp32 = 8 GiB per rank) through a schedule at 2 ranks
on the box's GPU: where creation spends its time (ESGD_DEBUG=1 prints the phases)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from mp_workers import run  # noqa: E402

if __name__ == "__main__":
    for count in (1 << 28, (1 << 31) - 1):
        outs = run("gpu_big", 2, count=count, rounds=2, timeout=600)
        print(json.dumps({"count": count, "ranks": outs}), flush=True)
