"""CPU checks of the caller-side surface (no device needed)."""
import ctypes

import pytest

from esgd import deep500
from esgd.optim import EagerSGDOptimizer


def test_tensor_t_layout_matches_deep500():
    # deep500.h:43-49: {tensortype_t type; tensororder_t order; uint8_t dims; uint32_t *sizes}
    assert ctypes.sizeof(deep500.tensor_t) == 24
    assert deep500.tensor_t.sizes.offset == 16
    d = deep500.TensorDesc((7, 3, 2))
    assert d.t.dims == 3 and [d.t.sizes[i] for i in range(3)] == [7, 3, 2] and d.t.type == 10


def test_optimizer_validation():
    with pytest.raises(ValueError):
        EagerSGDOptimizer(object(), 2, mode="ring")
    with pytest.raises(ValueError):
        EagerSGDOptimizer(object(), 0)


def test_configure_rejects_bad_mode():
    with pytest.raises(KeyError):
        deep500.configure("ring")


def test_overlap_refuses_a_second_backward_before_the_step():
    # with overlap=True the hooks post each gradient's round during backward; a
    # second backward before apply_gradients (gradient accumulation) would change gradients
    # whose rounds are already posted -- a clear error instead of autograd's deep one
    import torch
    model = torch.nn.Linear(4, 3)
    opt = EagerSGDOptimizer(torch.optim.SGD(model.parameters(), lr=0.1), 2, mode="allreduce", overlap=True)
    x = torch.randn(5, 4)
    model(x).sum().backward()   # two tensors: below the hooks' posting group, nothing posted
    with pytest.raises(RuntimeError, match="gradient accumulation"):
        model(x).sum().backward()
    opt.detach()


def test_registered_torch_op_sits_in_traced_graphs():
    # the reference's PyTorch bridge wraps the op in an autograd Function / nn.Module
    # (pytorch.tmpl.cpp:30-56, pytorch.py:71-114); here it is the torch.library operator
    # esgd::allreducef: torch.fx and torch.export keep it as one node, and its fake
    # implementation gives the output's shape without running a round (no device needed)
    import torch
    import torch.fx
    from torch._subclasses.fake_tensor import FakeTensorMode

    ar = deep500.AllreduceModule((4, 3), divisor=2.0)

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.ar = ar

        def forward(self, x):
            return self.ar(x * 2.0) + 1.0

    gm = torch.fx.symbolic_trace(Net())
    targets = [n.target for n in gm.graph.nodes if n.op == "call_function"]
    assert torch.ops.esgd.allreducef in targets
    ep = torch.export.export(Net(), (torch.randn(4, 3),))
    assert any(getattr(n.target, "name", lambda: "")() == "esgd::allreducef" for n in ep.graph.nodes
               if n.op == "call_function")
    with FakeTensorMode():
        y = torch.ops.esgd.allreducef(torch.empty(4, 3), torch.empty(4, 3), ar.op.handle, 2.0)
    assert tuple(y.shape) == (4, 3) and y.dtype == torch.float32
    handle = ar.op.handle
    ar.close()   # unregistered: the operator no longer reaches it
    with pytest.raises(RuntimeError, match="no live op"):
        torch.ops.esgd.allreducef(torch.ones(4, 3), torch.ones(4, 3), handle, 2.0)
