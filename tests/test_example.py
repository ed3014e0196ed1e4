"""examples/resnet50_eager_sgd.py's CPU-checkable pieces: the model is the reference's
ResNet-50 -- 161 trainable tensors holding exactly the 25 559 081 parameters of the bucket
table in opt_esgd_solo_imagenet_imbalance.py:86-248 -- and the straggler draw follows
resnet_run_loop_solo_imagenet_300.py:290-294."""
import os
import sys

import numpy as np

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "examples"))
import resnet50_eager_sgd as ex  # noqa: E402


def _reference_table():
    # the `length` list of the reference wrapper, summed (file read as data, not code)
    import re
    path = "/root/reference/test-models/tf-models-r1.11/official/utils/opt_esgd_solo_imagenet_imbalance.py"
    if not os.path.exists(path):
        return None
    text = open(path).read()
    m = re.search(r"int length\[OPS\]\s*=\s*\{([^}]*)\}", text)
    if not m:
        return None
    vals = [int(v) for v in re.findall(r"\d+", m.group(1))]
    assert len(vals) == 161
    return vals


def test_model_is_the_reference_bucket_table():
    params = [p for p in ex.resnet50().parameters() if p.requires_grad]
    assert len(params) == 161
    assert sum(p.numel() for p in params) == 25559081
    import json
    with open(os.path.join(ROOT, "tests", "golden", "resnet50_buckets.json")) as f:
        golden = json.load(f)["lengths"]   # the table as committed data (bench's C4 leg)
    assert sorted(golden) == sorted(p.numel() for p in params)
    table = _reference_table()   # and straight from the reference where it is present
    if table is not None:
        assert table == golden
    if table is not None:
        assert sum(table) == 25559081
        # the same 161 bucket sizes (the reference lists them in TF's variable order)
        assert sorted(table) == sorted(p.numel() for p in params)


def test_straggler_draw_matches_the_reference_loop():
    # the same two seeded draws on every rank; a rank sleeps if it is the first draw or,
    # failing that, the second
    for world in (2, 4, 8):
        for step in range(20):
            np.random.seed(step)
            a = np.random.randint(world)
            b = np.random.randint(world)
            want = {a, b}
            got = {r for r in range(world) if ex.straggles(step, r, world)}
            assert got == want, (world, step, got, want)
