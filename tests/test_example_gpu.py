"""examples/resnet50_eager_sgd.py on the GPU: the reference's training loop (ResNet-50,
its 161 gradient tensors = the 25 559 081-parameter bucket table of
opt_esgd_solo_imagenet_imbalance.py:86-248, the random-straggler sleep of
resnet_run_loop_solo_imagenet_300.py:287-296) driving EagerSGDOptimizer, launched the way
the reference launches its ranks (torch.distributed.run here, srun there).  Small images
and batches keep it to seconds; the synchronous mode must leave every rank with
bit-identical weights."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run(world, *args):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "examples", "resnet50_eager_sgd.py"),
           "--image", "64", "--batch", "4", "--warmup", "1", *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", ESGD_TIMEOUT_S="60"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["tensors"] == 161 and out["parameters"] == 25559081, out
    return out


@pytest.mark.parametrize("overlap", [False, True], ids=["after_backward", "during_backward"])
def test_resnet50_synchronous_rounds_keep_ranks_identical(overlap):
    # overlap: the 161 rounds posted from the gradient hooks while backward runs
    out = _run(2, "--mode", "allreduce", "--steps", "3", "--delay", "0", *(["--overlap"] if overlap else []))
    assert out["weights_identical_on_every_rank"], out


@pytest.mark.parametrize("mode,fuse,overlap", [("solo", True, False), ("majority", False, False),
                                               ("solo", False, True), ("majority", True, True)])
def test_resnet50_eager_sgd_with_stragglers(mode, fuse, overlap):
    # up to two drawn ranks sleep before each forward pass; the job runs through, and the
    # replicas stay identical: a partial round gives every rank the same sum (overlap: the
    # rounds posted from the gradient hooks during backward)
    out = _run(2, "--mode", mode, "--steps", "4", "--delay", "0.05", *(["--fuse"] if fuse else []),
               *(["--overlap"] if overlap else []))
    assert out["images_per_s"] > 0, out
    assert out["weights_identical_on_every_rank"], out
