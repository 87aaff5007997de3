"""FFT LinOp (reference operator/linop/fft/fft.py:20-379), on the MI355X through pxa_fft."""
import numpy as np

import pyxu_amd.abc as pxa
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev

__all__ = ["FFT"]


def _canonical_shape(s):
    if np.isscalar(s):
        return (int(s),)
    return tuple(int(v) for v in s)


class FFT(pxa.LinOp):
    r"""Multi-dimensional DFT over ``axes`` of ``arg_shape`` (fft.py:20-210).

    ``apply``: fftn(x, axes, norm="backward"); ``adjoint``: ifftn(x, axes, norm="forward").
    Complex arrays are real views ``(..., 2 N)`` of interleaved (re, im) pairs (the reference's
    ``view_as_real``).  With ``real=True`` the input of ``apply`` (and the output of ``adjoint``) is
    real-valued ``(..., N)``.  Like the reference, this inherits from LinOp (not NormalOp): with
    ``real=True`` the operator is not square.
    """

    def __init__(self, arg_shape, axes=None, real: bool = False, **kwargs):
        arg_shape = _canonical_shape(arg_shape)
        N_dim, N = len(arg_shape), int(np.prod(arg_shape))
        if axes is None:
            axes = tuple(range(N_dim))
        axes = np.unique(np.array(_canonical_shape(axes)))  # drop duplicates (fft.py:194)
        assert np.all((-N_dim <= axes) & (axes < N_dim))
        axes = (axes + N_dim) % N_dim
        sh_op = [2 * N, 2 * N]
        sh_op[1] //= 2 if real else 1
        super().__init__(shape=tuple(sh_op))
        self._arg_shape = tuple(arg_shape)
        self._axes = tuple(int(a) for a in axes)
        self._real = bool(real)
        self.lipschitz = self.estimate_lipschitz()

    def estimate_lipschitz(self, **kwargs):
        sh = np.array(self._arg_shape, dtype=int)
        return float(np.sqrt(sh[list(self._axes)].prod()))

    def gram(self):
        from pyxu_amd.operator.linop import HomothetyOp

        return HomothetyOp(dim=self.dim, cst=self.lipschitz**2)

    def cogram(self):
        if self._real:
            return super().cogram()  # no closed form once adjoint() projects onto the reals (fft.py:232-235)
        from pyxu_amd.operator.linop import HomothetyOp

        return HomothetyOp(dim=self.codim, cst=self.lipschitz**2)

    @pxrt.enforce_precision(i=("arr", "damp"))
    def pinv(self, arr, damp, **kwargs):
        N = self.lipschitz**2
        out = self.adjoint(arr)
        return _dev.div(out, N + damp, out=out)

    def dagger(self, damp, **kwargs):
        N = self.lipschitz**2
        return self.T / (N + damp)

    @pxrt.enforce_precision()
    def svdvals(self, **kwargs):
        k = int(kwargs.get("k", 1))
        return np.full(k, self.lipschitz, dtype=pxrt.getPrecision().value)

    def _transform(self, z, inverse):
        sh = z.shape[:-1]
        stack = int(np.prod(sh)) if len(sh) else 1
        return _dev.fft(z, self._arg_shape, self._axes, stack, inverse)

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        x = _dev.require(arr, "arr")
        z = _dev.real_to_complex(x) if self._real else x
        return self._transform(z, inverse=False)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        z = _dev.require(arr, "arr")
        out = self._transform(z, inverse=True)
        return _dev.complex_real_part(out) if self._real else out
