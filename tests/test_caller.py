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
