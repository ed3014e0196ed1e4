"""Scratch: reproduce the C5 mismatch after schedule churn with details."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from mp_workers import run  # noqa: E402

MAJ = 2

if __name__ == "__main__":
    sizes = [(1 << lg) // 4 for lg in (24, 28)]
    outs = run("gpu_config", 8, kind=MAJ, counts=sizes, rounds=1, timeout=300, detail=True)
    print("free", "->", [[v[3] for v in per] for per in outs], flush=True)
