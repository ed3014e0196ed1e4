"""deep500-style custom-operator bridge for the prebuilt eager-SGD gradient op.

The reference compiles the op from a C++ string at run time
(deep500/lv0/operators/op_compiler.py:57-114 -> CMake -> .so) and loads it with ctypes
(lv0/operators/operator_interface.py:48-91).  Here the op is part of libesgd.so; this
module keeps the same handle protocol: descriptors -> create_new_op -> forward ->
report -> delete_op (include/esgd_deep500.h).
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np

from . import _lib
from ._lib import lib

TT_FLOAT = 10          # deep500.h:16-34 tensortype_t
MODES = {"allreduce": 0, "solo": 1, "majority": 2}


class tensor_t(C.Structure):
    """deep500::tensor_t (deep500.h:43-49; utils/tensor_desc.py:6-11)."""
    _fields_ = [("type", C.c_int), ("order", C.c_int), ("dims", C.c_uint8),
                ("sizes", C.POINTER(C.c_uint32))]


class TensorDesc:
    def __init__(self, shape: Sequence[int], ttype: int = TT_FLOAT):
        self._sizes = (C.c_uint32 * max(1, len(shape)))(*[int(s) for s in shape])
        self.t = tensor_t(ttype, 0, len(shape), self._sizes)
        self.shape = tuple(int(s) for s in shape)


def _bind(h):
    vp = C.c_void_p
    h.esgd_op_configure.restype, h.esgd_op_configure.argtypes = C.c_int, [C.c_int, C.c_int, C.c_uint]
    h.esgd_op_configure_wire.restype, h.esgd_op_configure_wire.argtypes = C.c_int, [C.c_int]
    h.esgd_op_on_error.restype, h.esgd_op_on_error.argtypes = C.c_int, [C.c_int]
    h.esgd_op_status.restype, h.esgd_op_status.argtypes = C.c_int, [C.c_void_p]
    h.esgd_op_schedule.restype, h.esgd_op_schedule.argtypes = C.c_uint64, [C.c_void_p]
    h.create_new_op.restype = vp
    h.create_new_op.argtypes = [C.POINTER(tensor_t), C.c_int, C.POINTER(tensor_t), C.c_int]
    h.allreducef_forward.restype, h.allreducef_forward.argtypes = None, [vp, vp, vp, vp]
    h.allreducef_forward_host.restype = C.c_int
    h.allreducef_forward_host.argtypes = [vp, vp, vp]
    h.allreducef_forward_cuda.restype = None
    h.allreducef_forward_cuda.argtypes = [vp, vp, vp, vp, vp]
    h.allreducef_forward_cuda_div.restype = C.c_int
    h.allreducef_forward_cuda_div.argtypes = [vp, vp, vp, C.c_float, vp]
    h.allreducef_forward_cuda_packed.restype = C.c_int
    h.allreducef_forward_cuda_packed.argtypes = [vp, C.c_int, C.POINTER(vp), C.POINTER(C.c_uint64),
                                                 C.POINTER(vp), C.c_float, vp]
    h.allreducef_forward_cuda_wait_many.restype = C.c_int
    h.allreducef_forward_cuda_wait_many.argtypes = [C.POINTER(vp), C.c_int, C.POINTER(vp), vp]
    h.allreducef_forward_cuda_packed_post.restype = C.c_int
    h.allreducef_forward_cuda_packed_post.argtypes = [vp, C.c_int, C.POINTER(vp), C.POINTER(C.c_uint64),
                                                      C.POINTER(vp), C.c_float, vp]
    h.allreducef_forward_cuda_packed_wait.restype = C.c_int
    h.allreducef_forward_cuda_packed_wait.argtypes = [vp, vp]
    h.allreducef_forward_cuda_post_many_io.restype = C.c_int
    h.allreducef_forward_cuda_post_many_io.argtypes = [C.POINTER(vp), C.c_int, C.POINTER(vp), C.POINTER(vp),
                                                       C.c_float, vp]
    h.is_cuda_supported.restype, h.is_cuda_supported.argtypes = C.c_bool, [vp]
    h.report.restype, h.report.argtypes = C.c_int64, [vp, vp]
    h.delete_op.restype, h.delete_op.argtypes = None, [vp]


_lib.register_signatures(_bind)


WIRES = {"fp32": _lib.FLOAT, "bf16": _lib.BF16}


def configure(mode: str = "solo", async_: int = 32, seed: int = 6545343, wire: str = "fp32"):
    """Mode of the ops created afterwards (solo LIMITER 32 / majority seed 6545343 as
    in opt_esgd_{solo,majority}_imagenet_imbalance.py).  wire="bf16": device ops exchange
    bf16 copies of their fp32 buckets (half the xGMI bytes; an extension, the result is
    the bf16-rounded tree)."""
    _lib.check(lib().esgd_op_configure(MODES[mode], int(async_), int(seed) & 0xFFFFFFFF),
               "esgd_op_configure")
    _lib.check(lib().esgd_op_configure_wire(WIRES[wire]), "esgd_op_configure_wire")


def on_error(policy: str):
    """What the deep500-shaped void entry points do on a failed round: "abort" (default)
    or "local" (carry on with this rank's own gradient; AllreduceOp.status() keeps the
    first failure).  The Python methods below use the status variants and raise."""
    _lib.check(lib().esgd_op_on_error({"abort": 0, "local": 1, "default": -1}[policy]), "esgd_op_on_error")


class AllreduceOp:
    """One allreducef instance (one gradient tensor)."""

    def __init__(self, shape: Sequence[int]):
        self.inputs = [TensorDesc(shape), TensorDesc(shape)]   # (gradient, unused last)
        self.outputs = [TensorDesc(shape)]
        ins = (tensor_t * 2)(self.inputs[0].t, self.inputs[1].t)
        outs = (tensor_t * 1)(self.outputs[0].t)
        self.handle = lib().create_new_op(ins, 2, outs, 1)
        if not self.handle:
            raise _lib.EsgdError(_lib.ERROR, "create_new_op: " + _lib.last_error())
        self.numel = int(np.prod(shape)) if len(shape) else 1

    def forward(self, grad: np.ndarray, last: np.ndarray | None = None) -> np.ndarray:
        """Host path (the reference's CPU-registered kernel); allreducef_forward's status
        variant, so a failed round raises EsgdError instead of aborting the process."""
        g = np.ascontiguousarray(grad, dtype=np.float32)
        assert g.size == self.numel
        out = np.empty_like(g)
        _lib.check(lib().allreducef_forward_host(self.handle, g.ctypes.data, out.ctypes.data),
                   "allreducef_forward_host")
        return out

    def forward_cuda(self, grad, out, stream: int | None = None):
        """Device path: grad / out are device pointers or torch tensors.  Runs
        allreducef_forward_cuda's round through its status variant (a divisor of 1 is the
        plain copy-in), so a failed round raises EsgdError instead of aborting."""
        from .device import as_ptr
        _lib.check(lib().allreducef_forward_cuda_div(self.handle, as_ptr(grad), as_ptr(out), 1.0, stream),
                   "allreducef_forward_cuda")
        return out

    def forward_cuda_div(self, grad, out, divisor: float, stream: int | None = None):
        """Device path with the wrapper's grad / comm_size (:40) fused into the copy-in;
        `out` may be `grad` itself.  Raises EsgdError instead of aborting."""
        from .device import as_ptr
        _lib.check(lib().allreducef_forward_cuda_div(self.handle, as_ptr(grad), as_ptr(out),
                                                     float(divisor), stream),
                   "allreducef_forward_cuda_div")
        return out

    def forward_cuda_packed(self, grads, outs, divisor: float = 1.0, stream: int | None = None):
        """Bucket fusion: the tensors `grads` (fp32, contiguous, sizes summing to this op's
        size) packed in order, divided, reduced in one round and unpacked into `outs`."""
        from .device import ptr_array_of
        n = len(grads)
        counts = (C.c_uint64 * max(1, n))(*[int(g.numel()) if hasattr(g, "numel") else int(g.size)
                                             for g in grads])
        src = ptr_array_of(grads)
        dst = src if outs is grads else ptr_array_of(outs)
        _lib.check(lib().allreducef_forward_cuda_packed(self.handle, n, src, counts, dst, float(divisor),
                                                        stream), "allreducef_forward_cuda_packed")
        return outs

    def post_packed(self, grads, outs, divisor: float = 1.0, stream: int | None = None):
        """First half of forward_cuda_packed (allreducef_forward_cuda_packed_post): the round
        of the fused bucket posted with the pieces as its own data; wait_packed() finishes it.
        The tensors must stay alive until then.  Raises EsgdError."""
        from .device import ptr_array_of
        n = len(grads)
        counts = (C.c_uint64 * max(1, n))(*[int(g.numel()) for g in grads])
        src = ptr_array_of(grads)
        dst = src if outs is grads else ptr_array_of(outs)
        _lib.check(lib().allreducef_forward_cuda_packed_post(self.handle, n, src, counts, dst, float(divisor), stream),
                   "allreducef_forward_cuda_packed_post")

    def wait_packed(self, stream: int | None = None):
        """Second half: wait for the fused bucket's round (results in the outputs)."""
        _lib.check(lib().allreducef_forward_cuda_packed_wait(self.handle, stream), "allreducef_forward_cuda_packed_wait")

    @staticmethod
    def post_many_io(ops, grads, outs, divisor: float = 1.0, stream: int | None = None):
        """The rounds of many ops posted in one call (allreducef_forward_cuda_post_many_io), in
        this order, with one producer event: each round reads grads[i] / divisor itself and
        writes its result into outs[i] (may be grads[i]) -- no copy-in or copy-out launch on the
        caller's stream.  wait_many(ops, outs) then copies out only the rounds a peer carried
        this rank through before the post.  Unaligned tensors or a bf16 wire make the group go
        the copy-in way.  Raises EsgdError; the ops before a failed post stay posted."""
        from .device import ptr_array_of
        n = len(ops)
        hs = _lib.ptr_array([op.handle for op in ops])
        gs = ptr_array_of(grads)
        os_ = gs if outs is grads else ptr_array_of(outs)
        _lib.check(lib().allreducef_forward_cuda_post_many_io(hs, n, gs, os_, float(divisor), stream),
                   "allreducef_forward_cuda_post_many_io")

    @staticmethod
    def wait_many(ops, outs, stream: int | None = None):
        """The other half (allreducef_forward_cuda_wait_many): every posted op's round waited
        for in order, the copy-outs a round did not do itself in one launch per 48 ops, one
        release event; ops not posted are skipped.  Raises EsgdError (the first failure)
        after every round was waited for."""
        from .device import ptr_array_of
        n = len(ops)
        hs = _lib.ptr_array([op.handle for op in ops])
        os_ = ptr_array_of(outs)
        _lib.check(lib().allreducef_forward_cuda_wait_many(hs, n, os_, stream),
                   "allreducef_forward_cuda_wait_many")

    def forward_void(self, grad: np.ndarray) -> np.ndarray:
        """The reference ABI's void allreducef_forward verbatim (host buffers): on a failed
        round it aborts, or, under on_error("local"), returns this rank's own gradient."""
        g = np.ascontiguousarray(grad, dtype=np.float32)
        out = np.empty_like(g)
        lib().allreducef_forward(self.handle, g.ctypes.data, None, out.ctypes.data)
        return out

    def status(self) -> int:
        """First failure of a void entry point under on_error("local"), 0 while none."""
        return int(lib().esgd_op_status(self.handle))

    def schedule(self) -> int:
        """The op's esgd schedule handle (esgd_op_schedule), 0 before its first round."""
        return int(lib().esgd_op_schedule(self.handle))

    def supports_cuda(self) -> bool:
        return bool(lib().is_cuda_supported(self.handle))

    def report(self) -> int:
        return int(lib().report(self.handle, None))

    def close(self):
        if self.handle:
            lib().delete_op(self.handle)
            self.handle = None


def custom_op(shape: Sequence[int]) -> AllreduceOp:
    return AllreduceOp(shape)


# ---- the op as a registered PyTorch operator -------------------------------------------
# The reference's PyTorch bridge compiles forward_op / backward_op around the op's handle
# and wraps them in a torch.autograd.Function inside an nn.Module
# (D/frameworks/pytorch/custom_operators/pytorch.tmpl.cpp:30-56, pytorch.py:71-114,
# CustomPytorchCPPModule).  Here the same op is a torch.library operator, esgd::allreducef,
# so it can sit inside a traced (torch.fx) or exported graph: a fake (meta) implementation
# gives its output's shape without running a round, and its backward is the reference op's
# -- allreducef::backward writes nothing (opt_esgd_solo_imagenet_imbalance.py:321-326), so
# the inputs' gradients are the zeros the bridge's buffers start as.

_LIVE = {}   # handle -> AllreduceOp: the registered operator names ops by handle


def _register_torch_op():
    import torch

    # the schema spelled out: this module's annotations are strings (postponed evaluation)
    @torch.library.custom_op("esgd::allreducef", mutates_args=(),
                             schema="(Tensor grad, Tensor last, int handle, float divisor) -> Tensor")
    def allreducef(grad, last, handle, divisor):
        op = _LIVE.get(handle)
        if op is None:
            raise RuntimeError(f"esgd::allreducef: no live op with handle {handle:#x} (AllreduceModule holds one)")
        g = grad.detach().to(torch.float32).contiguous()
        if g.is_cuda:   # the device path, ordered on the caller's current stream
            out = torch.empty_like(g)
            op.forward_cuda_div(g, out, divisor, torch.cuda.current_stream(g.device).cuda_stream or None)
            return out
        x = g.numpy() if divisor == 1.0 else (g / divisor).numpy()
        return torch.from_numpy(op.forward(x)).view_as(g)   # the reference's host contract

    @allreducef.register_fake
    def _(grad, last, handle, divisor):
        return torch.empty_like(grad, dtype=torch.float32)

    def setup_context(ctx, inputs, output):
        ctx.shapes = (inputs[0], inputs[1])

    def backward(ctx, g_out):
        grad, last = ctx.shapes
        return torch.zeros_like(grad), torch.zeros_like(last), None, None

    allreducef.register_autograd(backward, setup_context=setup_context)
    return allreducef


_TORCH_OP = None


def torch_op():
    """torch.ops.esgd.allreducef(grad, last, handle, divisor) (registered on first use)."""
    global _TORCH_OP
    if _TORCH_OP is None:
        _TORCH_OP = _register_torch_op()
    return _TORCH_OP


def _module_base():
    import torch
    return torch.nn.Module


class AllreduceModule(_module_base()):
    """CustomPytorchCPPModule for the eager-SGD op: forward(grad, last) returns grad's
    partial allreduce (divided by `divisor` first: the wrapper's grad / comm_size, :40) through
    the registered operator esgd::allreducef -- the same round as AllreduceOp.forward_cuda_div
    (device tensors) or AllreduceOp.forward (host tensors)."""

    def __init__(self, shape: Sequence[int], divisor: float = 1.0):
        super().__init__()
        self.op = AllreduceOp(shape)
        self.divisor = float(divisor)
        _LIVE[self.op.handle] = self.op
        torch_op()

    def is_cuda_supported(self) -> bool:
        return self.op.supports_cuda()

    def close(self):
        """Unregister the op and delete it (its schedule: collective once a round ran, so every
        rank closes its modules in the same order, as AllreduceOp.close)."""
        if self.op.handle:
            _LIVE.pop(self.op.handle, None)
            self.op.close()

    def forward(self, grad, last=None):
        import torch
        return torch.ops.esgd.allreducef(grad, grad if last is None else last, self.op.handle, self.divisor)
