"""
pyxu_amd — MI355X-native backend for Pyxu's proximal-splitting hot path.

Mirrors the reference package layout for that path: ``pyxu_amd.abc`` (Operator lattice, Solver),
``pyxu_amd.operator`` (Stencil/Convolve/Gaussian, Gradient, L1/L21/SquaredL2, PositiveOrthant,
dense LinOp), ``pyxu_amd.opt.solver`` (PGD, CondatVu, PD3O, ADMM, CG, aliases),
``pyxu_amd.opt.stop``, ``pyxu_amd.runtime``, ``pyxu_amd.info.deps.NDArrayInfo`` (new member MI355X).

All arithmetic runs in hand-written HIP kernels (``libpyxu_amd.so``, C-ABI in
``include/pyxu_amd.h``); torch-ROCm tensors are only the device-array container.
"""
__version__ = "0.1.0"

from pyxu_amd._lib import BackendUnavailable, lib  # noqa: F401


def native_loaded() -> bool:
    """True if the HIP C-ABI library is loadable (it is the only compute path)."""
    return lib.loaded
