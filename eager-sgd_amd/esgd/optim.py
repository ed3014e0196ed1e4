"""EagerSGDOptimizer for PyTorch-ROCm: the optimizer-wrapper surface of eager-SGD.

Reference (TF 1.x): test-models/tf-models-r1.11/official/utils/
  opt_esgd_solo_imagenet_imbalance.py:6-44       (solo, LIMITER 32)
  opt_esgd_majority_imagenet_imbalance.py:6-44   (majority, seed 6545343)
  opt_sgd_mpi.py:6-47                            (synchronous MPI_Allreduce baseline)

Same protocol: compute_gradients() passes through to the wrapped optimizer's gradient
computation; apply_gradients() walks the (grad, var) list in reverse (:28), feeds every
gradient divided by the comm size (:40) through one eager-SGD op instance per tensor,
and hands the partially reduced gradients to the wrapped optimizer.  The op runs on the
device (allreducef_forward_cuda): the gradient never leaves HBM, unlike the reference's
CPU-only TF kernel (deep500/frameworks/tensorflow/custom_operators/tf.py:80).
"""
from __future__ import annotations

from typing import Iterable

from . import deep500


class EagerSGDOptimizer:
    def __init__(self, optimizer, comm_size: int, mode: str = "solo", async_: int = 32,
                 seed: int = 6545343):
        if mode not in deep500.MODES:
            raise ValueError(f"mode must be one of {sorted(deep500.MODES)}")
        if comm_size < 1:
            raise ValueError("comm_size must be >= 1")
        self.optimizer = optimizer
        self.comm_size = int(comm_size)
        self.mode, self.async_, self.seed = mode, int(async_), int(seed)
        self._ops = {}          # parameter -> op instance (one bucket per tensor)
        self._configured = False

    # -- the reference's two-call protocol ------------------------------------------
    def compute_gradients(self, loss) -> list:
        """Backpropagate `loss`; returns [(grad, param)] like tf.train.Optimizer."""
        loss.backward()
        return [(p.grad, p) for g in self.optimizer.param_groups for p in g["params"]]

    def apply_gradients(self, grads_and_vars: Iterable, global_step=None):
        import torch
        if not self._configured:
            deep500.configure(self.mode, self.async_, self.seed)
            self._configured = True
        stream = torch.cuda.current_stream().cuda_stream
        for grad, var in reversed(list(grads_and_vars)):
            if grad is None:          # the reference would still feed None (:35-42); skip
                continue
            op = self._ops.get(var)
            if op is None:
                op = self._ops[var] = deep500.AllreduceOp(tuple(grad.shape))
            scaled = (grad.float() / self.comm_size).contiguous()        # :40
            out = torch.empty_like(scaled)
            op.forward_cuda(scaled, out, stream)
            var.grad = out.to(grad.dtype).view_as(grad)
        r = self.optimizer.step()
        if global_step is not None and hasattr(global_step, "add_"):
            global_step.add_(1)
        return r

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
        return sum(op.report() for op in self._ops.values())
