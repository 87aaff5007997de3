"""
Backend registry (mirrors reference ``pyxu.info.deps.NDArrayInfo``, src/pyxu/info/deps.py:25-87).

``NDArrayInfo.MI355X`` is the new backend member: device arrays are torch-ROCm tensors resident on
an MI355X, and all arithmetic on them runs in this package's HIP kernels.  ``NUMPY`` is recognised
only so host arrays can be identified (and moved with :py:func:`pyxu_amd.util.to_device`);
operators in this package do not compute on host arrays.
"""
import enum

import numpy as np

__all__ = ["NDArrayInfo", "supported_array_types", "supported_array_modules"]


@enum.unique
class NDArrayInfo(enum.Enum):
    NUMPY = enum.auto()
    MI355X = enum.auto()

    @classmethod
    def default(cls) -> "NDArrayInfo":
        return cls.MI355X

    def type(self) -> type:
        if self is NDArrayInfo.NUMPY:
            return np.ndarray
        import torch

        return torch.Tensor

    @classmethod
    def from_obj(cls, obj) -> "NDArrayInfo":
        if obj is not None:
            if isinstance(obj, np.ndarray):
                return cls.NUMPY
            if type(obj).__module__.startswith("torch") and hasattr(obj, "is_cuda"):
                if obj.is_cuda:
                    return cls.MI355X
        raise ValueError(f"No known array type to match {obj}.")

    @classmethod
    def from_flag(cls, gpu: bool) -> "NDArrayInfo":
        return cls.MI355X if gpu else cls.NUMPY

    def module(self, linalg: bool = False):
        if self is NDArrayInfo.NUMPY:
            return np.linalg if linalg else np
        from pyxu_amd import xp

        return xp.linalg if linalg else xp


def supported_array_types():
    return tuple(n.type() for n in NDArrayInfo)


def supported_array_modules():
    return tuple(n.module() for n in NDArrayInfo)
