import numpy as np

from pyxu_amd.info.deps import NDArrayInfo

__all__ = [
    "get_array_module",
    "to_NUMPY",
    "to_device",
    "copy_if_unsafe",
    "read_only",
    "compute",
    "as_canonical_shape",
    "is_device_array",
]


def is_device_array(x) -> bool:
    return type(x).__module__.startswith("torch") and getattr(x, "is_cuda", False)


def get_array_module(x, fallback=None):
    """array-module of `x` (array_module.py:20-49)."""
    try:
        return NDArrayInfo.from_obj(x).module()
    except ValueError:
        if fallback is None:
            raise
        return fallback


def to_device(x, dtype=None, device=None):
    """Host NDArray -> MI355X tensor (the inverse of :py:func:`to_NUMPY`)."""
    import torch

    if is_device_array(x):
        if dtype is None or x.dtype == dtype:
            return x
        from pyxu_amd import _dev

        return _dev.cast(x, torch.empty((1,), dtype=dtype, device=x.device))  # device -> device: HIP cast
    a = np.ascontiguousarray(x)
    t = torch.from_numpy(a)
    if dtype is not None:
        t = t.to(dtype)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    return t.to(dev)


def to_NUMPY(x):
    """Any supported array -> numpy.ndarray (array_module.py:85-114)."""
    if isinstance(x, np.ndarray):
        return x
    if type(x).__module__.startswith("torch"):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def copy_if_unsafe(x):
    """Copy `x` if it is a view or read-only (array_module.py:194-225)."""
    if isinstance(x, np.ndarray):
        return x if (x.flags.owndata and x.flags.writeable) else x.copy()
    if type(x).__module__.startswith("torch"):
        from pyxu_amd import _dev

        return x if (x._base is None and x.is_contiguous()) else _dev.copy(x)
    return x


def read_only(x):
    if isinstance(x, np.ndarray):
        y = x.view()
        y.flags.writeable = False
        return y
    return x


def compute(*args, **kwargs):
    """No lazy backend here: identity (array_module.py:52-82)."""
    return args[0] if len(args) == 1 else args


def as_canonical_shape(x) -> tuple:
    if isinstance(x, (int, np.integer)):
        return (int(x),)
    return tuple(int(_) for _ in x)
