#!/usr/bin/env python3
"""ResNet-50 trained with eager-SGD on PyTorch-ROCm: the reference's use of the path.

The reference trains ResNet-50 on ImageNet with TF 1.x and swaps its optimizer for
EagerSGDOptimizer (test-models/tf-models-r1.11/official/resnet/resnet_run_loop_solo_
imagenet_300.py:46), with a synthetic load imbalance: every step, seeded by the step
counter, up to two randomly drawn ranks sleep 0.32 s before the forward pass (:287-296).
This script runs the same loop on MI355X -- a ResNet-50 whose 161 trainable tensors hold
the reference's 25 559 081 parameters (1001 classes, the model garden's ImageNet head;
the bucket table of opt_esgd_solo_imagenet_imbalance.py:86-248), synthetic images,
fp32 -- with one of:
  --mode solo | majority   eager-SGD (esgd.optim.EagerSGDOptimizer, per tensor or --fuse)
  --mode allreduce         the same optimizer, every round synchronous
  --mode ddp               torch.distributed all_reduce of each gradient over RCCL, divided
                           after (opt_sgd_mpi.py:40-44's synchronous baseline; needs one
                           GPU per rank)
One JSON line from rank 0: step time, images/s over all ranks, and whether every rank
ended with bit-identical weights -- in every mode: a partial round delivers the same sum
to every rank (a late rank's gradient is left out of it, not applied on that rank alone),
so the replicas never drift apart.  With P ranks each step puts 1/P + (P-1)/P^2 of them
to sleep (0.75 at P = 2, 0.23 at P = 8), which bounds what eager-SGD can gain at small P.

  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
      examples/resnet50_eager_sgd.py --mode solo --steps 50
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "eager-sgd_amd"))


def resnet50(classes: int = 1001):
    """ResNet-50 v1.5 (stride in the 3x3 conv of each bottleneck): 53 convolutions, 53
    batch norms (scale + shift) and the dense head = 161 trainable tensors."""
    import torch.nn as nn
    import torch.nn.functional as F

    class Bottleneck(nn.Module):
        def __init__(self, cin, width, stride, project):
            super().__init__()
            self.conv1, self.bn1 = nn.Conv2d(cin, width, 1, bias=False), nn.BatchNorm2d(width)
            self.conv2, self.bn2 = nn.Conv2d(width, width, 3, stride, 1, bias=False), nn.BatchNorm2d(width)
            self.conv3, self.bn3 = nn.Conv2d(width, 4 * width, 1, bias=False), nn.BatchNorm2d(4 * width)
            self.project = nn.Sequential(nn.Conv2d(cin, 4 * width, 1, stride, bias=False),
                                         nn.BatchNorm2d(4 * width)) if project else None

        def forward(self, x):
            skip = x if self.project is None else self.project(x)
            y = F.relu(self.bn1(self.conv1(x)))
            y = F.relu(self.bn2(self.conv2(y)))
            return F.relu(self.bn3(self.conv3(y)) + skip)

    layers = [nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
              nn.MaxPool2d(3, 2, 1)]
    cin = 64
    for width, blocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for b in range(blocks):
            layers.append(Bottleneck(cin, width, stride if b == 0 else 1, b == 0))
            cin = 4 * width
    layers += [nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(cin, classes)]
    return nn.Sequential(*layers)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["solo", "majority", "allreduce", "ddp"], default="solo")
    ap.add_argument("--fuse", action="store_true", help="eager-SGD: one fused bucket per step")
    ap.add_argument("--overlap", action="store_true",
                    help="eager-SGD: post the rounds from the gradient hooks during backward (per tensor; "
                         "with --fuse one fused round per bucket of --bucket-mb)")
    ap.add_argument("--bucket-mb", type=float, default=25.0, help="--fuse --overlap: bucket size in MiB")
    ap.add_argument("--wire", choices=["fp32", "bf16"], default="fp32",
                    help="eager-SGD: what the ranks exchange (bf16: fp32 buckets, bf16 copies on the wire)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="images per rank per step")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--delay", type=float, default=0.32,
                    help="seconds a drawn rank sleeps before its forward pass (0: balanced)")
    ap.add_argument("--trace-grads", action="store_true",
                    help="digest every step's reduced gradients on every rank; report the first step "
                         "whose reduced gradients differ between ranks (slow: host copies)")
    return ap.parse_args()


def straggles(step: int, rank: int, world: int) -> bool:
    """resnet_run_loop_solo_imagenet_300.py:290-294: seeded by the step counter, the rank
    sleeps if it equals the first draw or (failing that) a second draw."""
    import numpy as np
    np.random.seed(step)
    return rank == np.random.randint(world) or rank == np.random.randint(world)


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    import esgd
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = esgd.device_count()
    if ndev < 1:
        raise SystemExit("resnet50_eager_sgd.py: no HIP device")
    dev = torch.device("cuda", local % ndev)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    if a.mode == "ddp":
        if world > ndev:
            raise SystemExit("--mode ddp needs one GPU per rank (RCCL refuses ranks sharing a GPU)")
        group = dist.new_group(backend="nccl") if world > 1 else None
    else:
        from esgd import comm
        from esgd.optim import EagerSGDOptimizer
        esgd.check(esgd.lib().esgd_set_device(local % ndev), "esgd_set_device")
        comm.init()

    torch.manual_seed(42)   # the same initial weights on every rank
    model = resnet50().to(dev)
    params = [p for p in model.parameters() if p.requires_grad]
    sgd = torch.optim.SGD(params, lr=0.1, momentum=0.9)
    # the fused buckets' size (fuse + overlap) is a class attribute of the optimizer
    cls = type("Opt", (EagerSGDOptimizer,), {"bucket_mb": a.bucket_mb})
    opt = sgd if a.mode == "ddp" else cls(sgd, world, mode=a.mode, fuse=a.fuse, wire=a.wire, overlap=a.overlap)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.randn(a.batch, 3, a.image, a.image, device=dev, generator=g)
    y = torch.randint(0, 1001, (a.batch,), device=dev, generator=g)

    traced = []   # (step, slept, digest of the reduced gradients) with --trace-grads

    def step(t):
        if a.delay > 0 and world > 1 and straggles(t, rank, world):
            time.sleep(a.delay)
        loss = torch.nn.functional.cross_entropy(model(x), y)
        if a.mode == "ddp":
            sgd.zero_grad()
            loss.backward()
            for p in params:   # opt_sgd_mpi.py: allreduce every gradient, then divide
                if group is not None:
                    dist.all_reduce(p.grad, group=group)
                p.grad.div_(world)
            sgd.step()
        else:
            opt.zero_grad()
            opt.apply_gradients(opt.compute_gradients(loss))
        torch.cuda.synchronize()
        if a.trace_grads:
            h = hashlib.sha256()
            for p in params:
                h.update(p.grad.detach().cpu().numpy().tobytes())
            # zero fraction per rank-shard of the fused bucket (its order: reversed params)
            flat = torch.cat([p.grad.detach().reshape(-1) for p in reversed(params)]).cpu().numpy()
            per = -(-flat.size // world)
            zeros = [round(float((flat[q * per:(q + 1) * per] == 0).mean()), 4) for q in range(world)]
            traced.append((t, straggles(t, rank, world) if a.delay > 0 and world > 1 else False,
                           h.hexdigest()[:16], zeros))

    for t in range(a.warmup):
        step(t)
    # one barrier before the timed steps, none between them: a rank that was not drawn
    # runs ahead (eager-SGD) or waits inside the collective (synchronous modes), as in
    # the reference's run loop
    if world > 1:
        dist.barrier()
    times = []
    t_all = time.perf_counter()
    for t in range(a.warmup, a.warmup + a.steps):
        t0 = time.perf_counter()
        step(t)
        times.append(time.perf_counter() - t0)
    wall = time.perf_counter() - t_all

    digest = hashlib.sha256()
    for p in params:
        digest.update(p.detach().cpu().numpy().tobytes())
    mine = {"digest": digest.hexdigest(), "wall": wall, "device": local % ndev, "traced": traced}
    alls = [mine]
    if world > 1:
        alls = [None] * world
        dist.all_gather_object(alls, mine)
    if rank == 0:
        wall_max = max(o["wall"] for o in alls)
        print(json.dumps({
            "model": "resnet50 (1001 classes)", "tensors": len(params),
            "parameters": sum(p.numel() for p in params), "mode": a.mode, "fuse": a.fuse, "wire": a.wire,
            "overlap": a.overlap,
            "world": world, "batch_per_rank": a.batch, "image": a.image, "dtype": "f32",
            "data": "synthetic", "straggler_delay_s": a.delay, "steps": a.steps,
            "step_ms_median": round(statistics.median(times) * 1e3, 2),
            "images_per_s": round(world * a.batch * a.steps / wall_max, 1),
            "weights_identical_on_every_rank": len({o["digest"] for o in alls}) == 1,
            "devices": [o["device"] for o in alls],
            **({"first_step_with_different_reduced_gradients": next(
                (st[0][0] for st in zip(*[o["traced"] for o in alls]) if len({x[2] for x in st}) > 1), None),
                "traced": [o["traced"] for o in alls]} if a.trace_grads else {}),
        }), flush=True)
    if a.mode != "ddp":
        comm.finalize()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
