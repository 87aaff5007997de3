"""
N-D stencils (mirrors reference ``pyxu.operator.linop.stencil``: Stencil / Correlate / Convolve,
src/pyxu/operator/linop/stencil/stencil.py:26-887 and _stencil.py:99-476).

Semantics are the reference's exactly — ``apply = Trim o S_{D-1} o ... o S_0 o Pad`` with numba
``@stencil`` zeroing on the padded array, ``adjoint = Pad^T o S^bw o Trim^T`` (flipped kernels,
centers ``k - c - 1``), taps constant-folded like the code generator (``isclose(k, 0)`` dropped,
``isclose(k, 1)`` applied without a multiply) — but evaluated by HIP kernels:

* mode="constant" everywhere: one fused pass (pxa_stencil_sep / pxa_stencil_nd with zero-padding
  semantics) — the padded array is never materialised;
* any other mode: pxa_pad -> zeroed passes on the padded array -> pxa_trim (and the exact adjoint).
"""
import functools
import itertools
import operator
import warnings

import numpy as np

import pyxu_amd.abc as pxa
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev
from pyxu_amd.util import is_device_array, to_NUMPY

__all__ = ["Stencil", "Correlate", "Convolve"]

_MODES = ("constant", "wrap", "reflect", "symmetric", "edge")


class PrecisionWarning(UserWarning):
    pass


def _fold_taps(kernel, center):
    """Code-generation constant folding (_stencil.py:284-305): returns [(offset_vec, coef)] in
    itertools.product order, dropping isclose(k,0) taps and snapping isclose(k,1) taps to 1."""
    out = []
    for idx in itertools.product(*map(range, kernel.shape)):
        cst = kernel[idx]
        if np.isclose(cst, 0):
            continue
        off = tuple(int(i - c) for i, c in zip(idx, center))
        out.append((off, 1.0 if np.isclose(cst, 1) else float(cst)))
    return out


class _StencilSpec:
    """Host-side description of one stencil of the chain (kernel rank D, center rank D)."""

    def __init__(self, kernel, center):
        self.kernel = kernel
        self.center = np.asarray(center, dtype=int)
        self.taps = _fold_taps(kernel, self.center)
        nz = [d for d in range(kernel.ndim) if kernel.shape[d] > 1]
        self.axis = nz[0] if len(nz) == 1 else (0 if not nz else None)  # single-axis stencil?
        self.identity = len(self.taps) == 1 and all(o == 0 for o in self.taps[0][0]) and self.taps[0][1] == 1.0
        self._dev_taps = {}

    def axis_taps(self):
        a = self.axis
        return [t[0][a] for t in self.taps], [t[1] for t in self.taps]

    def device_taps(self, like):
        import torch

        key = (like.device, like.dtype)
        if key not in self._dev_taps:
            offs = np.array([t[0] for t in self.taps], dtype=np.int32).reshape(-1, self.kernel.ndim)
            coefs = np.array([t[1] for t in self.taps], dtype=np.float64)
            npdt = np.float32 if like.dtype == torch.float32 else np.float64
            self._dev_taps[key] = (  # host -> device uploads (the coefficients cast on the host)
                torch.from_numpy(offs).to(like.device),
                torch.from_numpy(coefs.astype(npdt)).to(like.device),
            )
            self._tap_box = (offs.min(axis=0).tolist(), offs.max(axis=0).tolist()) if len(offs) else None
        return self._dev_taps[key]

    def tap_box(self):
        """per-axis (min, max) of the tap offsets (host), for the tiled N-D kernel; None without taps"""
        return getattr(self, "_tap_box", None)


class Stencil(pxa.SquareOp):
    """Multi-dimensional stencil (stencil.py:26-789)."""

    def __init__(self, arg_shape, kernel, center, mode="constant", enable_warnings: bool = True):
        arg_shape, _kernel, _center, _mode = self._canonical_repr(arg_shape, kernel, center, mode)
        dim = int(np.prod(arg_shape))
        super().__init__(shape=(dim, dim))
        self._arg_shape = arg_shape
        self._mode = _mode
        self._pad_width = self._compute_pad_width(_kernel, _center, _mode)
        self._pad_shape = tuple(n + l + r for n, (l, r) in zip(arg_shape, self._pad_width))
        self._separable = len(_kernel) > 1
        self._st_fw = [_StencilSpec(k, c) for k, c in zip(_kernel, _center)]
        k_bw, c_bw = self._bw_equivalent(_kernel, _center)
        self._st_bw = [_StencilSpec(k, c) for k, c in zip(k_bw, c_bw)]
        self._dtype = _kernel[0].dtype
        self._enable_warnings = bool(enable_warnings)
        self.lipschitz = self.estimate_lipschitz(__rule=True)

    # ------------------------------------------------------------------ canonical forms
    @staticmethod
    def _canonical_repr(arg_shape, kernel, center, mode):
        """stencil.py:497-538: kernels coerced to the RUNTIME precision (Appendix A hazard 1)."""
        if not isinstance(arg_shape, (tuple, list)):
            arg_shape = (arg_shape,)
        arg_shape = tuple(int(n) for n in arg_shape)
        N = len(arg_shape)
        assert len(center) == N
        if isinstance(kernel, np.ndarray) or is_device_array(kernel):  # non-separable
            kernel = to_NUMPY(kernel)
            assert kernel.ndim == N
            _kernel = [pxrt.coerce(kernel)]
            _center = [np.array(center, dtype=int)]
        else:  # separable: one 1-D kernel per axis
            assert len(kernel) == N
            _kernel = []
            for i in range(N):
                sh = [1] * N
                sh[i] = -1
                _kernel.append(pxrt.coerce(np.asarray(to_NUMPY(kernel[i]))).reshape(sh))
            _center = np.zeros((N, N), dtype=int)
            _center[np.diag_indices(N)] = center
            _center = list(_center)
        if isinstance(mode, str):
            mode = (mode,) * N
        assert len(mode) == N, "arg_shape/mode are length-mismatched."
        _mode = tuple(m.strip().lower() for m in mode)
        assert set(_mode) <= set(_MODES), "Unknown mode(s) encountered."
        for k, c in zip(_kernel, _center):
            assert np.all(0 <= c) and np.all(c < k.shape)
        return arg_shape, _kernel, _center, _mode

    @staticmethod
    def _compute_pad_width(_kernel, _center, _mode):
        """stencil.py:540-561."""
        N = _kernel[0].ndim
        pw = []
        for i in range(N):
            if len(_kernel) == 1:
                c, n = _center[0][i], _kernel[0].shape[i]
            else:
                c, n = _center[i][i], _kernel[i].size
            p = max(c, n - c - 1) if _mode[i] == "constant" else n - 1
            pw.append((int(p), int(p)))
        return tuple(pw)

    @staticmethod
    def _bw_equivalent(_kernel, _center):
        """stencil.py:563-576."""
        k_bw = [np.ascontiguousarray(np.flip(k)) for k in _kernel]
        if len(_kernel) == 1:
            c_bw = [np.array(_kernel[0].shape) - _center[0] - 1]
        else:
            N = _kernel[0].ndim
            c_bw = []
            for i in range(N):
                c = np.zeros(N, dtype=int)
                c[i] = _kernel[i].shape[i] - _center[i][i] - 1
                c_bw.append(c)
        return k_bw, c_bw

    # ------------------------------------------------------------------ evaluation
    def _cast_warn(self, arr):
        if arr.dtype == pxrt.Width(self._dtype).torch:
            return arr
        if self._enable_warnings:
            warnings.warn("Computation may not be performed at the requested precision.", PrecisionWarning)
        import torch

        return _dev.cast(arr, torch.empty((1,), dtype=pxrt.Width(self._dtype).torch, device=arr.device))

    # ------------------------------------------------------------------ FFT path (large N-D kernels)
    # Non-separable constant-mode kernels with at least this many taps go through the FFT.  None: 1280 for 2-D
    # tap boxes the LDS-tiled direct kernel takes (2048^2 with 31 x 31 taps 0.30 ms direct, 0.40 ms FFT), 256
    # for other 2-D boxes (wider than 65 on an axis or more than 2048 taps: only the generic one-thread-per-output
    # kernel would run them, 2.1 ms at 15 x 15 on 2048^2) and for 3-D and more (9 x 9 x 9 on 256^3: 2.9 ms
    # direct, 1.8 ms FFT); set an int to override.
    FFT_MIN_TAPS = None
    TILE_MAX_EXTENT, TILE_MAX_TAPS = 65, 2048  # the tiled kernel's envelope (csrc/stencil.hip launch_nd_tile)

    @classmethod
    def _default_fft_min_taps(cls, K):
        tiled = max(K) <= cls.TILE_MAX_EXTENT and int(np.prod(K)) <= cls.TILE_MAX_TAPS
        return 1280 if (len(K) == 2 and tiled) else 256

    def _fft_min_taps(self, K):
        return self.FFT_MIN_TAPS if self.FFT_MIN_TAPS is not None else self._default_fft_min_taps(K)

    @staticmethod
    def _smooth(n):
        """Smallest 2^a 3^b 5^c 7^d >= n (lengths the mixed-radix FFT kernel runs in LDS)."""
        m = n
        while True:
            k = m
            for p in (2, 3, 5, 7):
                while k % p == 0:
                    k //= p
            if k == 1:
                return m
            m += 1

    def _fft_plan(self, x):
        """Linear correlation through an FFT of the zero-padded signal (no wrap-around: L >= n + K - 1):
        y = Crop_[0,n)( IFFT( FFT(Pad(x)) * FFT(k_circ) ) / prod(L) ) with k_circ[(c - j) mod L] = k[j];
        the adjoint multiplies by the conjugate spectrum.  Returns the cached plan or None."""
        cache = getattr(self, "_fft_cache", None)
        key = str(x.dtype)
        if cache is not None and key in cache:
            return cache[key]
        plan = None
        st = self._st_fw[0]
        K = st.kernel.shape
        min_taps = self._fft_min_taps(K)
        if (not self._separable and all(m == "constant" for m in self._mode) and int(np.prod(K)) >= min_taps):
            L = tuple(self._smooth(n + k - 1) for n, k in zip(self._arg_shape, K))
            lim = 4096 if x.dtype == pxrt.Width.SINGLE.torch else 2048
            if max(L) <= lim and len(L) <= 8:
                import torch

                k = np.asarray(st.kernel, dtype=np.float64)
                c = np.asarray(st.center, dtype=int)
                kc = np.zeros(L, dtype=np.float64)
                idx = np.indices(K).reshape(len(K), -1)
                tgt = tuple(((c[:, None] - idx) % np.array(L)[:, None]))
                np.add.at(kc, tgt, k.reshape(-1))
                kc /= float(np.prod(L))  # the unnormalised inverse FFT's 1/prod(L), folded into the spectrum
                npdt = np.float32 if x.dtype == torch.float32 else np.float64
                kd = torch.from_numpy(kc.reshape(-1).astype(npdt)).to(x.device)  # host-cast upload
                spec = _dev.fft(_dev.real_to_complex(kd), L, tuple(range(len(L))), 1, inverse=False)
                plan = dict(L=L, spec=spec)
        if cache is None:
            cache = self._fft_cache = {}
        cache[key] = plan
        return plan

    def _run_fft(self, x, S, plan, adjoint):
        L, n = plan["L"], self._arg_shape
        D = len(L)
        hi = [l - m for l, m in zip(L, n)]
        xp = _dev.pad(x, S, n, [0] * D, hi, ("constant",) * D).reshape(S, -1)
        z = _dev.fft(_dev.real_to_complex(xp), L, tuple(range(D)), S, inverse=False)
        z = _dev.complex_mul(z, plan["spec"], conj_b=adjoint, out=z)
        z = _dev.fft(z, L, tuple(range(D)), S, inverse=True, out=z)
        yp = _dev.complex_real_part(z)
        return _dev.trim(yp, S, L, [0] * D, hi, embed=False).reshape(S, -1)

    def _run(self, arr, specs, adjoint):
        x = _dev.require(self._cast_warn(arr))
        sh = x.shape[:-1]
        S = int(np.prod(sh)) if len(sh) else 1
        N = self.dim
        x = x.reshape(S, N)
        plan = self._fft_plan(x)
        if plan is not None:
            return self._run_fft(x, S, plan, adjoint).reshape(*sh, N)
        y = _dev.empty((S, N), x)
        if all(m == "constant" for m in self._mode):
            if self._separable:
                taps = [None if st.identity else st.axis_taps() for st in specs]
                _dev.stencil_sep(x, y, S, self._arg_shape, taps)
            else:
                offs, coefs = specs[0].device_taps(x)
                box = specs[0].tap_box()
                _dev.stencil_nd(x, y, S, self._arg_shape, offs, coefs, zero_partial=False,
                                off_lo=box[0] if box else None, off_hi=box[1] if box else None)
            return y.reshape(*sh, N)
        # general boundary modes: explicit padded array, reference chain semantics
        lo = [l for l, _ in self._pad_width]
        hi = [r for _, r in self._pad_width]
        if not adjoint:
            cur = _dev.pad(x, S, self._arg_shape, lo, hi, self._mode)
        else:
            cur = _dev.trim(x, S, self._pad_shape, lo, hi, embed=True)
        cur = cur.reshape(S, -1)
        for st in specs:
            if st.identity:
                continue
            nxt = _dev.empty(cur.shape, cur)
            if st.axis is not None:
                o, c = st.axis_taps()
                _dev.stencil_axis(cur, nxt, S, self._pad_shape, st.axis, o, c, zero_partial=True)
            else:
                offs, coefs = st.device_taps(cur)
                box = st.tap_box()
                _dev.stencil_nd(cur, nxt, S, self._pad_shape, offs, coefs, zero_partial=True,
                                off_lo=box[0] if box else None, off_hi=box[1] if box else None)
            cur = nxt
        if not adjoint:
            out = _dev.trim(cur, S, self._pad_shape, lo, hi, embed=False)
        else:
            out = _dev.pad_adjoint(cur, S, self._arg_shape, lo, hi, self._mode)
        return out.reshape(*sh, N)

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return self._run(arr, self._st_fw, adjoint=False)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        return self._run(arr, self._st_bw, adjoint=True)

    def estimate_lipschitz(self, **kwargs):
        if "__rule" in kwargs:
            kernels = [st.kernel for st in self._st_fw]
            kernel = functools.reduce(operator.mul, kernels, 1)
            L_st = np.linalg.norm(np.asarray(kernel).reshape(-1), ord=1)
            L_pad = 1.0
            for N, m, (l, r) in zip(self._arg_shape, self._mode, self._pad_width):
                if m in ("wrap", "symmetric"):
                    L_pad *= np.sqrt(1 + np.ceil((l + r) / N))
                elif m == "reflect":
                    L_pad *= np.sqrt(1 + np.ceil((l + r) / (N - 2)))
                elif m == "edge":
                    L_pad *= np.sqrt(1 + max(l, r))
            return float(L_st * L_pad)
        return super().estimate_lipschitz(**kwargs)

    @pxrt.enforce_precision()
    def trace(self, **kwargs):
        if all(m == "constant" for m in self._mode):
            tr = functools.reduce(operator.mul, [st.kernel[tuple(st.center)] for st in self._st_fw], 1)
            return float(tr * self.dim)
        return super().trace(**kwargs)

    # ------------------------------------------------------------------ introspection (stencil.py:689-789)
    @property
    def kernel(self):
        if len(self._st_fw) == 1:
            return self._st_fw[0].kernel
        return [st.kernel.reshape(-1) for st in self._st_fw]

    @property
    def center(self):
        if len(self._st_fw) == 1:
            return tuple(self._st_fw[0].center)
        return tuple(st.center[d] for d, st in enumerate(self._st_fw))

    @property
    def relative_indices(self):
        if len(self._st_fw) == 1:
            return [np.arange(s) - c for c, s in zip(self.center, self.kernel.shape)]
        return [np.arange(k.size) - c for c, k in zip(self.center, self.kernel)]

    @property
    def arg_shape(self):
        return self._arg_shape

    def visualize(self) -> str:
        kern = self._st_fw[0].kernel if len(self._st_fw) == 1 else functools.reduce(np.multiply.outer, self.kernel)
        k = np.array(kern, dtype=str)
        k[tuple(self.center)] = "(" + k[tuple(self.center)] + ")"
        return np.array2string(k, separator=" ").replace("'", "")


Correlate = Stencil


class Convolve(Stencil):
    """Convolution = Stencil with forward/backward stencils swapped (stencil.py:794-887)."""

    def __init__(self, arg_shape, kernel, center, mode="constant", enable_warnings: bool = True):
        super().__init__(arg_shape=arg_shape, kernel=kernel, center=center, mode=mode, enable_warnings=enable_warnings)
        self._st_fw, self._st_bw = self._st_bw, self._st_fw
