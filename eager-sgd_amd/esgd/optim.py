"""EagerSGDOptimizer for PyTorch-ROCm: the optimizer-wrapper surface of eager-SGD.

Reference (TF 1.x): test-models/tf-models-r1.11/official/utils/
  opt_esgd_solo_imagenet_imbalance.py:6-44       (solo, LIMITER 32)
  opt_esgd_majority_imagenet_imbalance.py:6-44   (majority, seed 6545343)
  opt_sgd_mpi.py:6-47                            (synchronous MPI_Allreduce baseline)

Same protocol: compute_gradients() passes through to the wrapped optimizer's gradient
computation; apply_gradients() walks the (grad, var) list in reverse (:28), feeds every
gradient divided by the comm size (:40) through one eager-SGD op instance per tensor,
and hands the partially reduced gradients to the wrapped optimizer.  The op runs on the
device (allreducef_forward_cuda_div): the gradient never leaves HBM, unlike the
reference's CPU-only TF kernel (deep500/frameworks/tensorflow/custom_operators/tf.py:80).
The division is fused into the op's copy-in (same IEEE fp32 division, same bits) and the
reduced gradient is written back into p.grad in place: per tensor and step 3 HBM passes
of the gradient (copy-in with the divide; the move with the zeroing fused; copy-out)
instead of 5 (divide, copy-in, move, copy-out, memset); with the fused round I/O below, 1
(the round's own snapshot reads the gradient; its phases write the result back).

pipeline=True (the per-tensor default): every tensor's round is posted before the first
is waited for, so the 161 host round trips overlap instead of running one after another as
the reference's blocking ops do (:304-307); the same rounds over the same operands, so the
same bits.  The posts and the waits each go through ONE call
(allreducef_forward_cuda_post_many_io / _wait_many, one producer event), and the data plane
runs the rounds that come due together in shared launches, each round reading grad /
comm_size and writing the reduced gradient back into p.grad itself (no copy-in or copy-out
launch on the caller's stream, 2 HBM passes of the gradient fewer -- only a round a peer
carried this rank through before its post is copied out of the op's bucket).
pipeline=False keeps the blocking chain (each op fused the same way).
When the caller works on the legacy default stream (torch's default), the ops' posts, waits
and copies go through a stream of the optimizer's own, ordered after the caller's stream on
entry and before it on exit (the ops on the legacy stream cost 1.3-1.6x per step on the
1-GPU rehearsal: profiles/r05/README.md).

Not here, by design (round 6): gradients as views into the ops' buckets.  A
solo / majority round a peer activates while this rank is still in backward must read a
send bucket backward is not writing -- the move sb -> rb that opens every round of the
reference (F/src/colls/ffallreduce.c:126-130) is the algorithm, not overhead -- and with
p.grad a persistent view, autograd accumulates into it (zero + read-add-write, 4 passes
of the gradient and a kernel per tensor in backward) instead of stealing the fresh
gradient: more HBM traffic than the snapshot it would save.

fuse=True (SURVEY.md §8(f) "bucket fusion"): the reference runs one schedule per tensor,
161 per ResNet-50 step (opt_esgd_solo_imagenet_imbalance.py:85-248), each a
host-blocking post/wait.  Fused, the scaled gradients are packed in the same reversed
order into ONE persistent HBM bucket, reduced by one round and unpacked.  The reduction
is element-wise, so every element meets the same operands in the same tree order: the
result is bit-identical to the per-tensor path.
"""
from __future__ import annotations

from typing import Iterable

from . import deep500


def _nullcontext():
    import contextlib
    return contextlib.nullcontext()


class EagerSGDOptimizer:
    # fuse=True with overlap=True: gradients go in buckets of about this many MiB (DDP's
    # default bucket_cap_mb); a subclass or the class attribute changes it before construction
    bucket_mb = 25.0
    # overlap=True: the hooks post in groups of this many tensors (one call, one producer
    # event each): a post per tensor from Python cost ~15 us of host time apiece, on the
    # backward's host path (r05t)
    overlap_group = 16

    def __init__(self, optimizer, comm_size: int, mode: str = "solo", async_: int = 32,
                 seed: int = 6545343, fuse: bool = False, wire: str = "fp32",
                 pipeline: bool = True, overlap: bool = False):
        if mode not in deep500.MODES:
            raise ValueError(f"mode must be one of {sorted(deep500.MODES)}")
        if wire not in deep500.WIRES:
            raise ValueError(f"wire must be one of {sorted(deep500.WIRES)}")
        if comm_size < 1:
            raise ValueError("comm_size must be >= 1")
        self.optimizer = optimizer
        self.comm_size = int(comm_size)
        self.mode, self.async_, self.seed = mode, int(async_), int(seed)
        self.fuse = bool(fuse)
        self.pipeline = bool(pipeline)
        # overlap=True: every tensor's round is posted from a post-accumulate-grad hook, as
        # soon as backward has written that gradient -- the way TF's dataflow runs the
        # reference's ops as their inputs become ready -- and apply_gradients waits for them.
        # With fuse=True the gradients go in buckets of about bucket_mb MiB (reversed
        # parameter order, the order backward produces them), one fused round per bucket,
        # posted once its last gradient exists.  One backward per step: a gradient's round is
        # posted once per step (a second backward before apply_gradients -- gradient
        # accumulation -- is refused by a clear error)
        self.overlap = bool(overlap)
        self._buckets = None    # fuse + overlap: [[param, ...], ...] in reversed order
        self._bucket_of = {}    # id(param) -> bucket index
        self._bucket_ops = []   # one AllreduceOp per bucket (created at its first post)
        self._bucket_left = []  # gradients each bucket still waits for in this backward
        self._bucket_posted = []
        self._conv = []         # (param, its gradient, the fp32 copy the bucket reduces)
        self._ready = []        # (op, grad, param) whose gradient exists, not yet posted
        self._seen = set()      # id(param) whose gradient the hooks saw since the last step
        self._bwd = []          # (op, grad, param) posted by the hooks since the last step
        self._hooks = []
        if self.overlap:
            self._attach()
        self._side = None
        self.wire = wire        # "bf16": bf16 copies between ranks
        # id(parameter) -> op instance (one bucket per tensor); by id: a Parameter's own
        # __hash__ is a Python call, 161 of them a step (the parameters live in param_groups)
        self._ops = {}
        self._fused = None      # (layout, op, packed bucket, reduced bucket)
        self._configured = False

    # -- the reference's two-call protocol ------------------------------------------
    def compute_gradients(self, loss) -> list:
        """Backpropagate `loss`; returns [(grad, param)] like tf.train.Optimizer."""
        loss.backward()
        return [(p.grad, p) for g in self.optimizer.param_groups for p in g["params"]]

    def apply_gradients(self, grads_and_vars: Iterable, global_step=None):
        import torch
        if not self._configured:
            deep500.configure(self.mode, self.async_, self.seed, self.wire)
            self._configured = True
        self._seen = set()   # the next backward's hooks start afresh
        caller = torch.cuda.current_stream()
        side = None
        if caller.cuda_stream == 0:
            if self._side is None or self._side.device != caller.device:
                self._side = torch.cuda.Stream(device=caller.device)
            side = self._side
            side.wait_stream(caller)       # the gradients were written on the caller's stream
        with (torch.cuda.stream(side) if side is not None else _nullcontext()):
            made = self._reduce(list(grads_and_vars), torch.cuda.current_stream().cuda_stream)
        if side is not None:
            caller.wait_stream(side)       # the wrapped step reads what the ops wrote there
            for t in made:                 # gradients converted on the side stream: the
                t.record_stream(caller)    # caller's stream uses them too
        r = self.optimizer.step()
        if global_step is not None and hasattr(global_step, "add_"):
            global_step.add_(1)
        return r

    def _attach(self):
        params = [p for group in self.optimizer.param_groups for p in group["params"] if p.requires_grad]
        if self.fuse:
            cap = max(1.0, self.bucket_mb * (1 << 20))
            self._buckets, cur, size = [], [], 0
            for p in reversed(params):
                cur.append(p)
                size += p.numel() * 4
                if size >= cap:
                    self._buckets.append(cur)
                    cur, size = [], 0
            if cur:
                self._buckets.append(cur)
            self._bucket_of = {id(p): b for b, bk in enumerate(self._buckets) for p in bk}
            self._bucket_ops = [None] * len(self._buckets)
            self._bucket_posted = [False] * len(self._buckets)
            self._bucket_left = [len(bk) for bk in self._buckets]
        for p in params:
            self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    def _post_bucket(self, b, stream, made=None):
        """The fused round of bucket b, its pieces the parameters' gradients (converted to
        contiguous fp32 if they are not: only from apply_gradients, `made` given)."""
        import torch
        bk = self._buckets[b]
        gs = []
        for p in bk:
            g = p.grad
            if g is None:
                raise RuntimeError("EagerSGDOptimizer(fuse=True, overlap=True): a parameter of a bucket has no "
                                   "gradient, but the bucket's schedule is persistent")
            if g.dtype != torch.float32 or not g.is_contiguous():
                if made is None:
                    return False   # apply_gradients posts it
                g32 = g.float().contiguous()
                self._conv.append((p, g, g32))   # written back after the wait
                g = g32
            gs.append(g)
        if not self._configured:
            deep500.configure(self.mode, self.async_, self.seed, self.wire)
            self._configured = True
        if self._bucket_ops[b] is None:
            self._bucket_ops[b] = deep500.AllreduceOp((sum(g.numel() for g in gs),))
        self._bucket_ops[b].post_packed(gs, gs, self.comm_size, stream)
        self._bucket_posted[b] = True
        return True

    def _on_grad(self, p):
        """Backward has accumulated p.grad: post its round now (read grad / P, result back
        into grad), ordered after the backward's stream.  A gradient the fused round I/O cannot
        take (not fp32 contiguous and 16-B aligned) waits for apply_gradients.  fuse=True: the
        bucket's round once its last gradient is there."""
        import torch
        if id(p) in self._seen:   # a second backward of this step (gradient accumulation)
            raise RuntimeError("EagerSGDOptimizer(overlap=True) posts each gradient's round during the step's one "
                               "backward; a second backward before apply_gradients (gradient accumulation) would "
                               "change a gradient whose round is already posted -- use overlap=False for it")
        self._seen.add(id(p))
        if self.fuse:
            b = self._bucket_of.get(id(p))
            if b is not None and not self._bucket_posted[b]:
                self._bucket_left[b] -= 1
                if self._bucket_left[b] == 0:
                    self._post_bucket(b, torch.cuda.current_stream().cuda_stream)
            return
        g = p.grad
        if g is None or g.dtype != torch.float32 or not g.is_contiguous() or g.data_ptr() % 16:
            return
        if not self._configured:
            deep500.configure(self.mode, self.async_, self.seed, self.wire)
            self._configured = True
        op = self._ops.get(id(p))
        if op is None:
            op = self._ops[id(p)] = deep500.AllreduceOp(tuple(g.shape))
        self._ready.append((op, g, p))
        if len(self._ready) >= self.overlap_group:
            self._post_ready(torch.cuda.current_stream().cuda_stream)

    def _post_ready(self, stream):
        group, self._ready = self._ready, []
        if group:
            self._bwd.extend(group)   # waited for in apply_gradients even if the post failed part-way
            gs = [g for _, g, _ in group]
            deep500.AllreduceOp.post_many_io([o for o, _, _ in group], gs, gs, self.comm_size, stream)

    def detach(self):
        """Remove the overlap hooks (posts go back to apply_gradients)."""
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self.overlap = False

    def _reduce(self, gvs, stream):
        """The ops' rounds over every gradient, results back in p.grad; returns the
        gradients it had to replace (converted to contiguous fp32 and back)."""
        import torch
        made = []
        if self.fuse:
            self._apply_fused(gvs, stream, made)
        else:
            if self._ready:   # the hooks' last, partial group
                self._post_ready(stream)
            early, self._bwd = self._bwd, []
            if early:   # posted by the backward hooks (overlap): wait for those first
                done = {id(p) for _, _, p in early}
                err = None
                try:
                    deep500.AllreduceOp.wait_many([o for o, _, _ in early], [g for _, g, _ in early], stream)
                except Exception as e:   # noqa: BLE001 -- re-raised after the rest
                    err = e
                gvs = [(g, v) for g, v in gvs if id(v) not in done]
                if err is not None:
                    raise err
            posted = []
            ops_of, f32 = self._ops, torch.float32
            for grad, var in reversed(gvs):
                if grad is None:      # the reference would still feed None (:35-42); skip
                    continue
                op = ops_of.get(id(var))
                if op is None:
                    op = ops_of[id(var)] = deep500.AllreduceOp(tuple(grad.shape))
                g = grad if (grad.dtype is f32 and grad.is_contiguous()) else grad.float().contiguous()
                if self.pipeline:
                    posted.append((op, g, grad, var))
                else:
                    op.forward_cuda_div(g, g, self.comm_size, stream)      # :40 fused, in place
                    if g is not grad:
                        var.grad = g.to(grad.dtype).view_as(grad)
                        made.append(var.grad)
            if posted:
                ops, gs = [p[0] for p in posted], [p[1] for p in posted]
                err = None
                try:   # :40 and the copy-in / copy-out fused into the rounds themselves
                    deep500.AllreduceOp.post_many_io(ops, gs, gs, self.comm_size, stream)
                except Exception as e:   # noqa: BLE001 -- re-raised below
                    err = e
                try:   # every posted round is waited for, even after a failed post
                    deep500.AllreduceOp.wait_many(ops, gs, stream)
                except Exception as e:   # noqa: BLE001
                    err = err or e
                if err is not None:
                    raise err
                for op, g, grad, var in posted:
                    if g is not grad:
                        var.grad = g.to(grad.dtype).view_as(grad)
                        made.append(var.grad)
        return made

    def _apply_fused(self, gvs, stream, made):
        import torch
        if self._buckets is not None:   # overlap: the buckets' rounds, posted by the hooks or now
            err = None
            for b in range(len(self._buckets)):
                if not self._bucket_posted[b]:
                    try:
                        self._post_bucket(b, stream, made)
                    except Exception as e:   # noqa: BLE001 -- the posted ones are waited for first
                        err = err or e
            for b, op in enumerate(self._bucket_ops):
                if self._bucket_posted[b]:
                    try:
                        op.wait_packed(stream)
                    except Exception as e:   # noqa: BLE001
                        err = err or e
            self._bucket_posted = [False] * len(self._buckets)
            self._bucket_left = [len(bk) for bk in self._buckets]
            conv, self._conv = self._conv, []
            if err is not None:
                raise err
            for p, g, g32 in conv:
                p.grad = g32.to(g.dtype).view_as(g)
                made.append(p.grad)
            return
        live = [(g, v) for g, v in reversed(gvs) if g is not None]
        if not live:
            return
        layout = tuple((id(v), g.numel()) for g, v in live)
        if self._fused is None:
            total = sum(n for _, n in layout)
            # one persistent schedule over the op's own bucket, created collectively at
            # the first step (the reference creates its bucket schedules lazily too,
            # :288-298)
            self._fused = (layout, deep500.AllreduceOp((total,)))
        elif self._fused[0] != layout:
            raise RuntimeError("EagerSGDOptimizer(fuse=True): the set of gradients changed, "
                               "but the fused bucket's schedule is persistent")
        _, op = self._fused
        gs = [g if (g.dtype == torch.float32 and g.is_contiguous()) else g.float().contiguous()
              for g, _ in live]
        # pack (divided as in :40) -> one round -> unpack into the same tensors
        op.forward_cuda_packed(gs, gs, self.comm_size, stream)
        for g32, (g, v) in zip(gs, live):
            if g32 is not g:
                v.grad = g32.to(g.dtype).view_as(g)
                made.append(v.grad)

    # -- torch.optim-style convenience ---------------------------------------------
    def step(self, closure=None):
        if closure is not None:
            closure()
        gvs = [(p.grad, p) for g in self.optimizer.param_groups for p in g["params"]]
        return self.apply_gradients(gvs)

    def zero_grad(self, set_to_none: bool = True):
        self.optimizer.zero_grad(set_to_none=set_to_none)

    @property
    def param_groups(self):
        return self.optimizer.param_groups

    def bytes_reduced(self) -> int:
        n = sum(op.report() for op in self._ops.values())
        if self._fused is not None:
            n += self._fused[1].report()
        n += sum(op.report() for op in self._bucket_ops if op is not None)
        return n
