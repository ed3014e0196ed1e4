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
