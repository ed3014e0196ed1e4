"""The drop-in callers on the GPU: the deep500 op ABI (host buckets, the reference's
contract) and the PyTorch EagerSGDOptimizer (device path), multi-rank on one device."""
import pytest

from mp_workers import run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["allreduce", "solo", "majority"])
def test_deep500_op_host_path(mode):
    # with every rank posting behind a barrier, solo / majority rounds see every rank's
    # fresh gradient (evaluation/{solo,rand}_allreduce_correctness.c known answer)
    outs = run("op_host", 2, mode=mode, steps=3, count=5000)
    for o in outs:
        assert o["cuda"] and o["report"] == 3 * 5000 * 4
        if mode == "allreduce":
            assert all(o["ok"]), o


@pytest.mark.parametrize("fuse", [False, True])
@pytest.mark.parametrize("mode", ["allreduce", "solo"])
def test_eager_sgd_optimizer(mode, fuse):
    # fuse=True packs every gradient into one bucket (one round per step): the same
    # bits as one round per tensor
    outs = run("optimizer_step", 2, mode=mode, steps=2, fuse=fuse)
    for o in outs:
        if mode == "allreduce":
            assert all(o["ok"]), o["ok"]
        assert o["bytes"] > 0
    if mode == "allreduce":   # synchronous averaging keeps the replicas identical
        assert outs[0]["params_digest"] == outs[1]["params_digest"]
