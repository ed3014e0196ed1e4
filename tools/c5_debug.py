"""Scratch: the C5 churn pattern (buckets freed and re-allocated between schedules)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from mp_workers import run  # noqa: E402

MAJ = 2

if __name__ == "__main__":
    sizes = [(1 << lg) // 4 for lg in (24, 28)]
    for name, kw in [("base", {}), ("norounds_first", {"rounds": [0, 2]}),
                     ("p4_norounds", {"rounds": [0, 2], "world": 4}),
                     ("torch_like_shadow", {"env": {"ESGD_SHADOW": "1"}})]:
        kw.setdefault("counts", sizes)
        kw.setdefault("rounds", 2)
        world = kw.pop("world", 8)
        outs = run("gpu_config", world, kind=MAJ, timeout=300, **kw)
        print(name, "->", [[v[3] for v in per] for per in outs], flush=True)
