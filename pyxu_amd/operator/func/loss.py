"""``shift_loss`` (reference operator/func/loss.py:13-34): ``op.argshift(-data)``."""
from pyxu_amd import _dev

__all__ = ["shift_loss"]


def shift_loss(op, data=None):
    if data is None:
        return op
    from pyxu_amd.util import is_device_array

    if is_device_array(data):
        return op.argshift(_dev.axpby(-1.0, _dev.require(data, "data")))
    return op.argshift(-data)  # host tensor: construction-only (compute on it raises)
