"""Repeat FFT(arg_shape=(2048, 2048), real=True) fp64 apply / adjoint against NumPy (the test_fft_vs_numpy case
that failed once in r04zw) and report the error and where it sits; also under each PXA_TUNE_FFT_KERNEL mode."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402
from pyxu_amd.util import to_NUMPY, to_device  # noqa: E402

sh = (2048, 2048)
N = sh[0] * sh[1]
stack = 2
rng = np.random.default_rng(26)
xr = rng.standard_normal((stack, *sh))
x = xr + 1j * np.zeros_like(xr)
ref_f = np.fft.fftn(x, axes=[1, 2], norm="backward")
ref_b = np.fft.ifftn(x, axes=[1, 2], norm="forward")
view = lambda c: np.stack([c.real, c.imag], axis=-1).reshape(stack, 2 * N)  # noqa: E731
want = ref_b.real.reshape(stack, N)
modes = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 256, 512, 1]
for mode in modes:
    _dev.tuning(_dev.TUNE_FFT_KERNEL, mode)
    with pxrt.Precision(pxrt.Width.DOUBLE):
        op = pxo.FFT(arg_shape=sh, real=True)
        for it in range(3):
            y = to_NUMPY(op.apply(to_device(xr.reshape(stack, N))))
            z = to_NUMPY(op.adjoint(to_device(view(x))))
            ey = np.max(np.abs(y - view(ref_f))) / np.max(np.abs(view(ref_f)))
            ez = np.abs(z - want)
            bad = np.argwhere(ez > 1e-9 * np.max(np.abs(want)))
            print(f"mode {mode} it {it}: apply {ey:.2e} adjoint {np.max(ez) / np.max(np.abs(want)):.2e} "
                  f"bad {len(bad)} first {bad[:4].tolist()}", flush=True)
_dev.tuning(_dev.TUNE_FFT_KERNEL, 0)
