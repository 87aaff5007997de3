"""
Device-array kernels: thin Python entry points over the C-ABI (``include/pyxu_amd.h``).

Every function takes/returns torch-ROCm tensors resident on the current device, launches on
``torch.cuda.current_stream()`` and raises on any non-zero status.  Host arrays are rejected with
a TypeError: this package has no CPU compute path.
"""
import ctypes as ct
import os

import numpy as np

from pyxu_amd._lib import check, f64_array, i32_array, i64_array, int_array, lib

__all__ = []  # internal module

RED_SUMSQ, RED_DIFFSQ, RED_DOT, RED_ABS, RED_MAXABS, RED_SUM, RED_NEGCNT, RED_MIN, RED_MAX = range(9)
MODES = {"constant": 0, "wrap": 1, "reflect": 2, "symmetric": 3, "edge": 4}


def _torch():
    import torch

    return torch


def wait_event(ev, spin_s=1e-3):
    """Wait for a recorded HIP event: poll it for up to `spin_s` seconds, then yield between polls so that a
    long wait does not starve other threads.  A stop check waits for the device queue the host has run ahead
    by (stop_rate x the step time at most: ~0.25 ms at 20 PGD steps of 2048^2), and the step enqueued
    behind the check covers only one step time after the event: a blocking hipEventSynchronize, or a
    sleep(0) between polls, wakes the host up tens of microseconds late and leaves the device idle."""
    import time

    if ev.query():
        return
    t_end = time.perf_counter() + spin_s
    while not ev.query():
        if time.perf_counter() > t_end:
            time.sleep(0)


def dtcode(t) -> int:
    torch = _torch()
    if t.dtype == torch.float32:
        return 0
    if t.dtype == torch.float64:
        return 1
    raise TypeError(f"pyxu_amd: unsupported dtype {t.dtype} (float32/float64 only).")


def require(t, name="arr"):
    """Validate a device operand: CUDA (ROCm) tensor, float32/64, contiguous."""
    if _TIMER is not None:  # other device work is about to be enqueued: close the timing window
        _TIMER.interrupt()
    if not (type(t).__module__.startswith("torch") and hasattr(t, "is_cuda")):
        raise TypeError(
            f"pyxu_amd: `{name}` must be an MI355X device tensor (got {type(t).__name__}); "
            "move host data with pyxu_amd.util.to_device()."
        )
    if not t.is_cuda:
        raise TypeError(f"pyxu_amd: `{name}` lives on {t.device}; pyxu_amd computes on the MI355X only.")
    dtcode(t)
    return t if t.is_contiguous() else t.contiguous()


def ptr(t) -> int:
    return t.data_ptr()


def _raw_stream_fn():
    torch = _torch()
    get = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    dev = getattr(torch._C, "_cuda_getDevice", None)
    if get is None or dev is None:  # pragma: no cover - older torch
        return lambda: torch.cuda.current_stream().cuda_stream
    return lambda: get(dev())


_RAW_STREAM = None


def stream():
    """hipStream_t of torch's current stream on the current device (fast path: the raw-stream query,
    ~10x cheaper than torch.cuda.current_stream(), which matters at tens of us per solver step)."""
    global _RAW_STREAM
    if _RAW_STREAM is None:
        _RAW_STREAM = _raw_stream_fn()
    return ct.c_void_p(_RAW_STREAM())


_TSTREAM = (None, None)  # (raw hipStream_t, torch stream object) of the last record_event


def record_event(ev):
    """ev.record() on torch's current stream, without torch.cuda.current_stream()'s Python device lookup on
    every call (a few microseconds, paid once per solver step at stop_rate 1): the torch stream object is
    cached per raw stream."""
    global _TSTREAM
    torch = _torch()
    key = (_RAW_STREAM() if _RAW_STREAM is not None else None, torch._C._cuda_getDevice())
    if key[0] is None or key != _TSTREAM[0]:
        _TSTREAM = (key, torch.cuda.current_stream())
    ev.record(_TSTREAM[1])
    return ev


class LaunchTimer:
    """HIP-event windows around runs of back-to-back fused solver-step launches.

    Measurement hook for bench.py: while installed (``set_launch_timer``), the fused step kernels
    open a window (start event on the launch stream = torch's current stream, which the kernel runs
    on) and close it after ``window`` consecutive launches, or earlier when any other device work
    (a stop-criterion reduction / copy) is about to be enqueued (``interrupt``).  ``mean_ms()`` =
    total window time / launches inside windows = the average launch duration, measured live on
    the timed region's own launches, with one event pair per window rather than per launch.

    ``single=True``: ONE window over the whole timed region, opened right AFTER the first launch (so
    that the first launch's start-up latency on an idle device is not counted) and closed by
    ``close()``; interrupts are ignored, so the window also holds the stop checks' small kernels and
    any host-bound gap between launches (an upper bound on the kernel's own duration).  Two events in
    the region instead of two per interrupted window: the per-step windows cost ~2.4 us of host time
    per PGD step at 2048^2 (40.3 k vs 37.1 k image-it/s, profiles/r04p_timer_ab.txt).
    """

    def __init__(self, window=10, single=False):
        self.windows = []  # (ev0, ev1, launches)
        self.window = max(1, int(window))
        self.single = bool(single)
        self._open = None
        self._count = 0
        self._first = True
        # single mode: both events created here, outside the timed region (creating one costs host time)
        self._spare = [_torch().cuda.Event(enable_timing=True) for _ in range(2)] if self.single else []

    def _event(self):
        ev = self._spare.pop(0) if self._spare else _torch().cuda.Event(enable_timing=True)
        ev.record(_torch().cuda.current_stream())
        return ev

    def begin(self):
        if self.single:
            return True
        if self._open is None:
            self._open = self._event()
            self._count = 0
        return True

    def end(self, _tok=None):
        if self.single:
            if self._first:  # the window starts behind the first launch
                self._first = False
                self._open = self._event()
                self._count = 0
            else:
                self._count += 1
            return
        self._count += 1
        if self._count >= self.window:
            self.interrupt()

    def interrupt(self):
        if self.single:
            return
        self.close()

    def close(self):
        if self._open is not None and self._count > 0:
            self.windows.append((self._open, self._event(), self._count))
        self._open = None
        self._count = 0

    @property
    def launches(self):
        return sum(c for _, _, c in self.windows)

    def mean_ms(self):
        self.close()
        if not self.windows:
            return None
        self.windows[-1][1].synchronize()
        return sum(a.elapsed_time(b) for a, b, _ in self.windows) / self.launches


_TIMER = None


def set_launch_timer(timer):
    """Install (or remove, with None) the LaunchTimer of the fused solver-step kernels."""
    global _TIMER
    _TIMER = timer


_USE_COUNT = None


def storage_exclusive(t) -> bool:
    """True iff no other tensor shares `t`'s storage.  Solvers overwrite a buffer in place only when
    the Python reference count of the tensor object says nobody else holds it AND this holds: views
    such as ``img.reshape(-1)`` or ``batch[i]`` passed as x0 / z0 keep the storage's use count above
    that of a lone tensor.  The reference allocates fresh arrays every step, so anything a user can
    still reach must never be written."""
    global _USE_COUNT
    if _USE_COUNT is None:
        torch = _torch()
        _USE_COUNT = getattr(torch._C, "_storage_Use_Count", None) or (lambda _c: 1 << 30)
    # a lone tensor: its TensorImpl + the temporary storage wrapper created here
    return _USE_COUNT(t.untyped_storage()._cdata) <= 2


TUNE_NORMAL_KERNEL = 1  # PXA_TUNE_NORMAL_KERNEL: pxa_dense_normal A/B (0 row-split, 1 one workgroup per row, 2 row-split without the exchange)
TUNE_DENSE_KERNEL = 2  # PXA_TUNE_DENSE_KERNEL: 0 LDS-staged MFMA GEMM (B >= 32), 1 the register-streamed kernel
TUNE_DUAL_WGS = 4  # PXA_TUNE_DUAL_WGS: kernel C's target workgroup count (A/B; 0 = default)
TUNE_PGD_DIAG = 3  # PXA_TUNE_PGD_DIAG: bit 5 = s_memtime phase trace of the PGD tile kernel
TUNE_PGD_STAGGER = 6  # PXA_TUNE_PGD_STAGGER: (sel << 8) | n, delayed first-round workgroups (A/B probe)
TUNE_PDS_EVENTS = 5  # PXA_TUNE_PDS_EVENTS: per-kernel HIP events inside pxa_pds_step (pds_kernel_ms)
TUNE_PDS_MARCH = 7  # PXA_TUNE_PDS_MARCH: kernel D A/B (bit 0: two positions per thread)
TUNE_FFT_KERNEL = 8  # PXA_TUNE_FFT_KERNEL: 0 in-place register-staged FFT kernel, 1 the ping-pong Stockham kernel
TUNE_GRAD_KERNEL = 9  # PXA_TUNE_GRAD_KERNEL: 0 axis-0 march gradient kernels, 1 the row kernels (same bits)
TUNE_STENCIL_ND = 10  # PXA_TUNE_STENCIL_ND: 0 LDS-tiled N-D stencil where it applies, 1 the generic kernel (same sums)
TUNE_PGD_PIPE = 12  # PXA_TUNE_PGD_PIPE: 1 the pipelined PGD kernel (LDS-DMA window prefetch; same bits, slower)
TUNE_DUAL_ROWS = 11  # PXA_TUNE_DUAL_ROWS: kernel C rows per thread (0 / 1 one-row kernel, 2 or 4 row-blocked; same bits)


def tuning(key, value=-1):
    """Process-wide kernel-selection knob of the C-ABI (pxa_tuning): sets it when value >= 0 and
    returns the previous value.  For A/B measurements and variant-parity tests only."""
    r = int(lib.pxa_tuning(int(key), int(value)))
    if r < 0:
        check(r, "pxa_tuning")
    return r


def _tuning_from_env():
    """PXA_TUNE="key=value[,key=value...]" (keys: the PXA_TUNE_* numbers) sets knobs at import, so that A/B
    runs of bench.py / scripts need no code change."""
    spec = os.environ.get("PXA_TUNE", "").strip()
    for item in filter(None, (t.strip() for t in spec.split(","))):
        k, _, v = item.partition("=")
        try:
            tuning(int(k), int(v))
        except (ValueError, TypeError, RuntimeError) as e:  # a malformed item must not break the import
            import warnings

            warnings.warn(f"PXA_TUNE: ignoring {item!r} ({e})", RuntimeWarning, stacklevel=2)


def empty(shape, like):
    return _torch().empty(shape, dtype=like.dtype, device=like.device)


def empty_f64(shape, like):
    return _torch().empty(shape, dtype=_torch().float64, device=like.device)


def to_device_like(a, like):
    """Host numpy array -> device tensor of `like`'s dtype (an upload, no compute)."""
    return _torch().as_tensor(np.ascontiguousarray(a), device=like.device).to(like.dtype)


def empty_like(t):
    return _torch().empty_like(t, memory_format=_torch().contiguous_format)


def copy(x):
    x = require(x)
    return x.clone(memory_format=_torch().contiguous_format)


def scalar_dt(x):
    return np.float32 if dtcode(x) == 0 else np.float64


# ------------------------------------------------------------------ element-wise
def axpby(a, x, b=0.0, y=None, out=None):
    """out = a*x + b*y."""
    x = require(x, "x")
    if y is not None:
        y = require(y, "y")
        assert y.numel() == x.numel() and y.dtype == x.dtype
    out = empty_like(x) if out is None else out
    check(
        lib.pxa_axpby(dtcode(x), x.numel(), float(a), ptr(x), float(b), ptr(y) if y is not None else None, ptr(out), stream()),
        "pxa_axpby",
    )
    return out


def axpby_bcast(a, x, b, y, out=None):
    """out = a*x + b*y with y (M,) broadcast over x's leading dims (x: (..., M))."""
    x, y = require(x, "x"), require(y, "y")
    if y.numel() == x.numel():
        return axpby(a, x, b, y, out=out)
    out = empty_like(x) if out is None else out
    check(lib.pxa_axpby_bcast(dtcode(x), x.numel(), float(a), ptr(x), float(b), ptr(y), y.numel(), ptr(out), stream()), "pxa_axpby_bcast")
    return out


def axpy_rows(c, s, x, y, out=None):
    """out[r] = y[r] + s * c[r] * x[r] for x, y of shape (rows, n); c a (rows,) device vector."""
    x, y, c = require(x, "x"), require(y, "y"), require(c, "c")
    rows = c.numel()
    out = empty_like(y) if out is None else out
    check(lib.pxa_axpy_rows(dtcode(x), rows, x.numel() // max(rows, 1), ptr(c), float(s), ptr(x), ptr(y), ptr(out), stream()),
          "pxa_axpy_rows")
    return out


def row_ratio(num, den, like, out=None):
    """out[r] = num[r] / den[r] (float64 device vectors) cast to like's dtype, on the device."""
    num, den = require(num, "num"), require(den, "den")
    torch = _torch()
    assert num.dtype == torch.float64 and den.dtype == torch.float64 and num.numel() == den.numel()
    out = torch.empty((num.numel(),), dtype=like.dtype, device=like.device) if out is None else out
    check(lib.pxa_row_ratio(dtcode(like), num.numel(), ptr(num), ptr(den), ptr(out), stream()), "pxa_row_ratio")
    return out


def lincomb3(a, x, b, y, c, z, out=None):
    x, y, z = require(x), require(y), require(z)
    out = empty_like(x) if out is None else out
    check(lib.pxa_lincomb3(dtcode(x), x.numel(), float(a), ptr(x), float(b), ptr(y), float(c), ptr(z), ptr(out), stream()), "pxa_lincomb3")
    return out


def extrapolate(a, x, y, out=None):
    """(x - y) * a + x."""
    x, y = require(x), require(y)
    out = empty_like(x) if out is None else out
    check(lib.pxa_extrapolate(dtcode(x), x.numel(), float(a), ptr(x), ptr(y), ptr(out), stream()), "pxa_extrapolate")
    return out


def div(x, d, out=None):
    x = require(x)
    out = empty_like(x) if out is None else out
    check(lib.pxa_div(dtcode(x), x.numel(), ptr(x), float(d), ptr(out), stream()), "pxa_div")
    return out


def add_scalar(x, s, out=None):
    x = require(x)
    out = empty_like(x) if out is None else out
    check(lib.pxa_add_scalar(dtcode(x), x.numel(), ptr(x), float(s), ptr(out), stream()), "pxa_add_scalar")
    return out


def fill(out, v):
    out = require(out)
    check(lib.pxa_fill(dtcode(out), out.numel(), float(v), ptr(out), stream()), "pxa_fill")
    return out


def zeros(shape, like):
    return fill(empty(shape, like), 0.0)


def mul(x, y, out=None):
    x, y = require(x), require(y)
    out = empty_like(x) if out is None else out
    check(lib.pxa_mul(dtcode(x), x.numel(), ptr(x), ptr(y), ptr(out), stream()), "pxa_mul")
    return out


def clip(x, lo, hi=None, out=None):
    x = require(x)
    out = empty_like(x) if out is None else out
    check(lib.pxa_clip(dtcode(x), x.numel(), ptr(x), float(lo), float(hi or 0.0), int(hi is not None), ptr(out), stream()), "pxa_clip")
    return out


def prox_l1(x, tau, out=None):
    x = require(x)
    out = empty_like(x) if out is None else out
    check(lib.pxa_prox_l1(dtcode(x), x.numel(), ptr(x), float(tau), ptr(out), stream()), "pxa_prox_l1")
    return out


def admm_l1_update(x, z, u, cgrad, rho_m1, thr, tau):
    """ADMM outer update (h = lam L1, K = Id) + the next CG right-hand side in one launch
    (pxa_admm_l1_update): returns (u', z', b, r0, p0, x0), views of one (6, *x.shape) buffer."""
    x, z, u, cgrad = require(x), require(z), require(u), require(cgrad)
    n = x.numel()
    assert z.numel() == n and u.numel() == n and cgrad.numel() == n
    assert z.dtype == x.dtype and u.dtype == x.dtype and cgrad.dtype == x.dtype
    out = empty((6,) + tuple(x.shape), x)
    check(lib.pxa_admm_l1_update(dtcode(x), n, ptr(x), ptr(z), ptr(u), ptr(cgrad), float(rho_m1), float(thr),
                                 float(tau), ptr(out), stream()), "pxa_admm_l1_update")
    return tuple(out.unbind(0))


def fenchel_prox_l1(x, sigma, lam, out=None):
    x = require(x)
    out = empty_like(x) if out is None else out
    check(lib.pxa_fenchel_prox_l1(dtcode(x), x.numel(), ptr(x), float(sigma), float(lam), ptr(out), stream()), "pxa_fenchel_prox_l1")
    return out


def moreau_grad_l1(x, mu, scale, out=None):
    x = require(x)
    out = empty_like(x) if out is None else out
    check(lib.pxa_moreau_grad_l1(dtcode(x), x.numel(), ptr(x), float(mu), float(scale), ptr(out), stream()), "pxa_moreau_grad_l1")
    return out


def prox_l21(x, tau, outer, group, inner, out=None):
    x = require(x)
    out = empty_like(x) if out is None else out
    check(lib.pxa_prox_l21(dtcode(x), outer, group, inner, ptr(x), float(tau), ptr(out), stream()), "pxa_prox_l21")
    return out


def fenchel_prox_l21(x, sigma, lam, outer, group, inner, out=None):
    x = require(x)
    out = empty_like(x) if out is None else out
    check(
        lib.pxa_fenchel_prox_l21(dtcode(x), outer, group, inner, ptr(x), float(sigma), float(lam), ptr(out), stream()),
        "pxa_fenchel_prox_l21",
    )
    return out


def moreau_grad_l21(x, mu, scale, outer, group, inner, out=None):
    x = require(x)
    out = empty_like(x) if out is None else out
    check(
        lib.pxa_moreau_grad_l21(dtcode(x), outer, group, inner, ptr(x), float(mu), float(scale), ptr(out), stream()),
        "pxa_moreau_grad_l21",
    )
    return out


def group_norm(x, outer, group, inner):
    x = require(x)
    out = empty((outer * inner,), x)
    check(lib.pxa_group_norm(dtcode(x), outer, group, inner, ptr(x), ptr(out), stream()), "pxa_group_norm")
    return out


# ------------------------------------------------------------------ array primitives (csrc/array.hip)
UN_SQRT, UN_SIGN, UN_ABS, UN_NEG, UN_SQUARE, UN_RECIP, UN_POSINF = range(7)
BIN_FMAX, BIN_FMIN, BIN_ADD, BIN_SUB, BIN_MUL, BIN_DIV, BIN_MAXIMUM, BIN_MINIMUM, BIN_POW = range(9)


def copy2d(src, dst, rows, n, lds, ldd, src_off=0, dst_off=0, accumulate=0, col_stride=1):
    """dst[dst_off + r*ldd + i] = src[src_off + r*lds + i*col_stride] for r < rows, i < n (element
    offsets; col_stride 0 repeats one value per row); accumulate 1: dst += src; 2: dst = 0 + src (the
    first term of a Python sum)."""
    es = src.element_size()
    check(lib.pxa_copy2d(dtcode(src), int(rows), int(n), ptr(src) + int(src_off) * es, int(lds), int(col_stride),
                         ptr(dst) + int(dst_off) * es, int(ldd), int(accumulate), stream()), "pxa_copy2d")
    return dst


def take_cols(x, off, n):
    """x[..., off:off + n] as a contiguous device array (a view when x has no leading stack)."""
    x = require(x)
    d = x.shape[-1]
    if x.ndim == 1 or x.numel() == d:
        return x.reshape(-1)[off:off + n].reshape(*x.shape[:-1], n)
    rows = x.numel() // d
    out = empty((*x.shape[:-1], n), x)
    return copy2d(x, out, rows, n, d, n, src_off=off)


def concat_cols(parts, out=None):
    """numpy.concatenate(parts, axis=-1) for device arrays with equal leading shapes."""
    parts = [require(p) for p in parts]
    lead = parts[0].shape[:-1]
    total = sum(p.shape[-1] for p in parts)
    out = empty((*lead, total), parts[0]) if out is None else out
    rows = out.numel() // max(total, 1)
    off = 0
    for p in parts:
        copy2d(p, out, rows, p.shape[-1], p.shape[-1], total, dst_off=off)
        off += p.shape[-1]
    return out


def unary(op, x, out=None):
    x = require(x)
    out = empty_like(x) if out is None else out
    check(lib.pxa_unary(dtcode(x), int(op), x.numel(), ptr(x), ptr(out), stream()), "pxa_unary")
    return out


def binary(op, x, y, out=None, like=None):
    """out = op(x, y); x / y device arrays of one shape or Python scalars (broadcast)."""
    xa = None if np.isscalar(x) else require(x, "x")
    ya = None if np.isscalar(y) else require(y, "y")
    ref = xa if xa is not None else (ya if ya is not None else like)
    if xa is not None and ya is not None:
        assert xa.shape == ya.shape and xa.dtype == ya.dtype, "binary: shapes / dtypes differ"
    out = empty_like(ref) if out is None else out
    check(lib.pxa_binary(dtcode(ref), int(op), ref.numel(), ptr(xa) if xa is not None else None,
                         float(x) if xa is None else 0.0, ptr(ya) if ya is not None else None,
                         float(y) if ya is None else 0.0, ptr(out), stream()), "pxa_binary")
    return out


def where(cond, x, y, like=None):
    torch = _torch()
    cond = require_bool(cond)
    xa = None if np.isscalar(x) else require(x, "x")
    ya = None if np.isscalar(y) else require(y, "y")
    ref = xa if xa is not None else (ya if ya is not None else like)
    out = empty(cond.shape, ref)
    assert out.numel() == cond.numel()
    check(lib.pxa_where(dtcode(ref), out.numel(), cond.data_ptr(), ptr(xa) if xa is not None else None,
                        float(x) if xa is None else 0.0, ptr(ya) if ya is not None else None,
                        float(y) if ya is None else 0.0, ptr(out), stream()), "pxa_where")
    return out


def require_bool(c):
    torch = _torch()
    if not (hasattr(c, "is_cuda") and c.is_cuda and c.dtype == torch.bool):
        raise TypeError("pyxu_amd: condition must be a boolean device tensor")
    return c if c.is_contiguous() else c.contiguous()


def isnan(x):
    torch = _torch()
    x = require(x)
    out = torch.empty(x.shape, dtype=torch.bool, device=x.device)
    check(lib.pxa_isnan(dtcode(x), x.numel(), ptr(x), out.data_ptr(), stream()), "pxa_isnan")
    return out


def bool_reduce(c, mode):
    """any (mode 0) / all (mode 1) of a boolean device tensor -> 0-d boolean device tensor."""
    torch = _torch()
    c = require_bool(c)
    out = torch.empty((), dtype=torch.bool, device=c.device)
    check(lib.pxa_bool_reduce(c.numel(), int(mode), c.data_ptr(), out.data_ptr(), stream()), "pxa_bool_reduce")
    return out


def cast(x, dtype_like):
    """(dtype of dtype_like) copy of x (float32 <-> float64)."""
    x = require(x)
    out = _torch().empty(x.shape, dtype=dtype_like.dtype, device=x.device)
    check(lib.pxa_cast(dtcode(x), dtcode(out), x.numel(), ptr(x), ptr(out), stream()), "pxa_cast")
    return out


def set_diag(out, rows, ld, off, value):
    check(lib.pxa_set_diag(dtcode(out), int(rows), int(ld), int(off), float(value), ptr(out), stream()), "pxa_set_diag")
    return out


def dir_contract(w, wp, x, S, G, J, K, N, adjoint=False):
    """pxa_dir_contract: y = sum_j w[g, j] * x[j % K] (apply, (S, K, N) -> (S, G, N)) or its adjoint."""
    x, w = require(x, "x"), require(w, "w")
    y = empty((S, K if adjoint else G, N), x)
    check(lib.pxa_dir_contract(dtcode(x), int(S), int(G), int(J), int(K), int(N), ptr(w), int(wp), ptr(x), ptr(y),
                               int(bool(adjoint)), stream()), "pxa_dir_contract")
    return y


def transpose(x):
    """(rows, cols) -> contiguous (cols, rows)."""
    x = require(x)
    rows, cols = x.shape
    out = empty((cols, rows), x)
    check(lib.pxa_transpose(dtcode(x), rows, cols, ptr(x), ptr(out), stream()), "pxa_transpose")
    return out


# ------------------------------------------------------------------ reductions
def relerr_stats(x, x_prev, out, copy=True):
    """RelError statistics in one pass (pxa_relerr_stats): out[0] = sum (x - x_prev)^2 and
    out[1] = sum x_prev^2 per row (out: contiguous float64 (2, rows) buffer, device or pinned host);
    returns the copy of x the criterion keeps (or None with copy=False)."""
    torch = _torch()
    x = require(x)
    x_prev = require(x_prev)
    assert x_prev.shape == x.shape and x_prev.dtype == x.dtype
    n = x.shape[-1] if x.ndim > 0 else 1
    rows = x.numel() // max(n, 1) if x.numel() else 0
    assert out.dtype == torch.float64 and out.is_contiguous() and out.numel() == 2 * max(rows, 1)
    assert 0 < rows <= 65535, "relerr_stats: rows out of range (use row_reduce)"
    xc = empty_like(x) if copy else None
    wsz = int(lib.pxa_relerr_stats_workspace_bytes(rows, n))
    work = torch.empty((max(wsz // 8, 1),), dtype=torch.float64, device=x.device)
    check(lib.pxa_relerr_stats(dtcode(x), rows, n, ptr(x), ptr(x_prev), ptr(xc) if copy else None, out.data_ptr(),
                               ptr(work), stream()), "pxa_relerr_stats")
    return xc


def cg_update(x, r, p, ap, rr, rr_out, rr_host, work, have_pap=False):
    """pxa_cg_update: the CG iteration tail after A p on (rows, n) x / r / p / A p (in place), from this
    step's ||r||^2 `rr` (device float64 (rows,)); ||r'||^2 lands in rr_out (device) and in rr_host: a
    HostFlagBuffer(rows, rows, rows) (returns the publication's sequence number, which its wait() takes), a
    pinned host tensor, or None.  have_pap: `work` already holds the <p, A p> partials (pxa_cg_update_tail;
    dense_normal(..., pdot=work) wrote them with A p)."""
    rows, n = x.shape
    seq, vp_, fp_ = 0, None, None
    if isinstance(rr_host, HostFlagBuffer):
        seq, vp_, fp_ = rr_host.next_seq(), rr_host.vptr, rr_host.fptr
    elif rr_host is not None:
        vp_ = rr_host.data_ptr()
    fn = lib.pxa_cg_update_tail if have_pap else lib.pxa_cg_update
    check(fn(dtcode(x), rows, n, ptr(x), ptr(r), ptr(p), ptr(ap), rr.data_ptr(), rr_out.data_ptr(), vp_, fp_, seq,
             work.data_ptr(), stream()), "pxa_cg_update")
    return seq


def cg_update_xr(x, r, p, ap, rr, work):
    """pxa_cg_update_xr: x += alpha p, r -= alpha A p and the ||r'||^2 partials (work + rows * 64 doubles), with the
    <p, A p> partials already in `work` (dense_normal(..., pdot=work)); the p update is left to the next
    dense_normal_pfold."""
    rows, n = x.shape
    check(lib.pxa_cg_update_xr(dtcode(x), rows, n, ptr(x), ptr(r), ptr(p), ptr(ap), rr.data_ptr(), work.data_ptr(),
                               stream()), "pxa_cg_update_xr")


def dense_normal_pfold(A, r, p, p_new, rr, rr_out, fb, seq, s, d, work, pdot):
    """pxa_dense_normal_pdot_pfold: p_new = r + beta p (the CG's previous p update, beta from cg_update_xr's ||r'||^2
    partials at pdot + 64 doubles and `rr`), then Y = s A^T (A p_new) + d p_new and the <p_new, Y> partials into
    pdot; ||r'||^2 into rr_out (device) and HostFlagBuffer `fb` under publication `seq`.  Returns Y."""
    M, N = A.shape
    wsz = int(lib.pxa_dense_normal_workspace_bytes(dtcode(p), M, N, 1))
    if wsz == 0 or work is None or work.numel() < wsz:
        raise ValueError("pxa_dense_normal_pdot_pfold: unsupported operand or workspace")
    Y = empty(p.shape, p)
    check(lib.pxa_dense_normal_pdot_pfold(dtcode(p), M, N, ptr(A), ptr(r), ptr(p), ptr(p_new), rr.data_ptr(),
                                          pdot.data_ptr() + 64 * 8, rr_out.data_ptr(), fb.vptr, fb.fptr, int(seq),
                                          float(s), float(d), ptr(Y), ptr(work), pdot.data_ptr(), stream()),
          "pxa_dense_normal_pdot_pfold")
    return Y


def tile_partials_fold(parts, rows, per_row, out):
    """RelError statistics from the fused PGD step's per-tile partials (pxa_tile_partials_fold):
    out (contiguous float64 (2, rows), device or pinned host) = per-row sum (x_new - x)^2, sum x^2."""
    assert out.is_contiguous() and out.numel() == 2 * rows
    check(lib.pxa_tile_partials_fold(int(rows), int(per_row), parts.data_ptr(), out.data_ptr(), None, 0, stream()),
          "pxa_tile_partials_fold")
    return out


def tile_partials_publish(parts, rows, per_row, fb, seq):
    """pxa_tile_partials_fold of `parts` into HostFlagBuffer `fb` under an existing publication number `seq`."""
    check(lib.pxa_tile_partials_fold(int(rows), int(per_row), parts.data_ptr(), fb.vptr, fb.fptr, int(seq), stream()),
          "pxa_tile_partials_fold")


class FlagWaitError(RuntimeError):
    """A HostFlagBuffer publication never landed although its stream is idle."""


def wait_flags(flags, seq, spin_s, stream_idle):
    """Host side of HostFlagBuffer.wait: busy-poll `flags` (uint32 array in coherent host memory) for
    `spin_s` seconds, then poll with a yield, asking `stream_idle()` each round.  Once the stream reports idle
    every write of the kernels before it has landed, so flags that still differ from `seq` after one more
    look will never change: raise FlagWaitError (the wait used to spin forever there)."""
    import time

    if len(flags) == 2:  # (one row: two flags, compared as scalars -- ~20x cheaper than the array compare)
        if flags[0] == seq and flags[1] == seq:
            return
    elif (flags == seq).all():
        return
    t_end = time.perf_counter() + spin_s
    while not (flags == seq).all():
        if time.perf_counter() > t_end:
            if stream_idle() and not (flags == seq).all():
                raise FlagWaitError(
                    f"publication {seq} never landed (flags {np.unique(flags).tolist()[:4]}) and the stream is "
                    "idle: the publishing kernel did not run, or the sequence number was overwritten")
            time.sleep(0)


class HostFlagBuffer:
    """Coherent host memory (pxa_host_alloc) for statistics a kernel publishes to the host: `values`
    (float64 (nvals,)) and one completion flag per value group (`flags`, uint32 (nflags,)).  The device writes
    the values, then the flags (system-scope release); the host polls the flags -- no stream event between the
    statistics and the next kernel, and no event wake-up latency.  Used by the fused RelError fold (2 rows
    values, 2 rows flags: `stats` is the (2, rows) view) and by CG's ||r'||^2 (rows, rows)."""

    def __init__(self, rows, nvals=None, nflags=None):
        self.rows = int(rows)
        nv = 2 * self.rows if nvals is None else int(nvals)
        nf = nv if nflags is None else int(nflags)
        nb = 8 * nv + 4 * nf + 4
        p = ct.c_void_p()
        check(lib.pxa_host_alloc(nb, ct.byref(p)), "pxa_host_alloc")
        self._ptr = p.value
        raw = (ct.c_uint8 * nb).from_address(self._ptr)
        self.values = np.frombuffer(raw, dtype=np.float64, count=nv)
        self.flags = np.frombuffer(raw, dtype=np.uint32, count=nf, offset=8 * nv)
        self.flags[:] = 0
        self.vptr, self.fptr = self._ptr, self._ptr + 8 * nv
        self.seq = 0
        self._free = lib.pxa_host_free

    @property
    def stats(self):
        return self.values.reshape(2, self.rows)

    def landed(self, seq):
        """Whether every flag of publication `seq` is set (no wait)."""
        f = self.flags
        if len(f) == 2:
            return bool(f[0] == seq and f[1] == seq)
        return bool((f == seq).all())

    def next_seq(self):
        """A new publication number, for a kernel about to be launched on the CURRENT stream: that stream is
        remembered with it, so that wait() asks the publishing stream (not whichever stream is current by
        then) whether the publication can still land."""
        self.seq = (self.seq % 0xFFFFFFFE) + 1
        global _RAW_STREAM
        if _RAW_STREAM is None:
            _RAW_STREAM = _raw_stream_fn()
        streams = self.__dict__.setdefault("_streams", {})
        streams[self.seq] = int(_RAW_STREAM() or 0)  # the raw handle: ~10x cheaper than a torch stream object
        if len(streams) > 16:
            streams.pop(next(iter(streams)))
        return self.seq

    def fold(self, parts, per_row):
        """Enqueue pxa_tile_partials_fold into this buffer under a new sequence number; returns it."""
        seq = self.next_seq()
        check(lib.pxa_tile_partials_fold(self.rows, int(per_row), parts.data_ptr(), self.vptr, self.fptr, seq,
                                         stream()), "pxa_tile_partials_fold")
        return seq

    def wait(self, seq, spin_s=1e-3):
        """Poll the flags until every value of publication `seq` has landed (as wait_event).  Raises
        instead of spinning forever when the stream has drained without publishing `seq` (an earlier
        kernel faulted, the publishing kernel never ran, or `seq` was overwritten by a later publication);
        an asynchronous device error surfaces through the stream query."""
        raw = self.__dict__.get("_streams", {}).get(seq)

        def idle():  # only asked once the spin has expired: building the stream object here costs nothing
            torch = _torch()
            if raw is None:  # a sequence number this buffer did not hand out: the current stream is all we know
                return torch.cuda.current_stream().query()
            if raw == 0:
                return torch.cuda.default_stream().query()
            return torch.cuda.ExternalStream(raw).query()

        wait_flags(self.flags, seq, spin_s, idle)

    def __del__(self):
        if getattr(self, "_ptr", None):
            self._free(self._ptr)
            self._ptr = None


def row_reduce(op, x, y=None, out=None):
    """Per-row reduction over the last axis -> float64 device tensor of shape x.shape[:-1] (or (1,)).
    `out`: optional contiguous float64 device buffer of max(rows, 1) elements to write into."""
    torch = _torch()
    x = require(x)
    n = x.shape[-1] if x.ndim > 0 else 1
    rows = x.numel() // max(n, 1) if x.numel() else 0
    if y is not None:
        y = require(y)
        assert y.shape == x.shape
    if out is None:
        out = torch.empty((max(rows, 1),), dtype=torch.float64, device=x.device)
    else:
        assert out.dtype == torch.float64 and out.is_contiguous() and out.numel() == max(rows, 1)
    if rows == 0:
        return out.zero_()
    # rows beyond the grid-y limit are processed in slabs
    step = 65535
    for r0 in range(0, rows, step):
        r1 = min(rows, r0 + step)
        es = x.element_size()
        wsz = int(lib.pxa_row_reduce_workspace_bytes(r1 - r0, n))
        work = torch.empty((max(wsz // 8, 1),), dtype=torch.float64, device=x.device)
        check(
            lib.pxa_row_reduce(
                dtcode(x), op, r1 - r0, n, ptr(x) + r0 * n * es, (ptr(y) + r0 * n * es) if y is not None else None,
                out.data_ptr() + r0 * 8, ptr(work), stream(),
            ),
            "pxa_row_reduce",
        )
    return out.reshape(x.shape[:-1]) if x.ndim > 1 else out


def row_reduce_pow(p, x, y=None, out=None):
    """Per-row sum |x - y|^p (p > 0) or non-zero count (p == 0) -> float64 device (rows,) tensor."""
    torch = _torch()
    x = require(x)
    n = x.shape[-1] if x.ndim > 0 else 1
    rows = x.numel() // max(n, 1) if x.numel() else 0
    if y is not None:
        y = require(y)
        assert y.shape == x.shape
    if out is None:
        out = torch.empty((max(rows, 1),), dtype=torch.float64, device=x.device)
    if rows == 0:
        return out.zero_()
    step = 65535
    es = x.element_size()
    for r0 in range(0, rows, step):
        r1 = min(rows, r0 + step)
        wsz = int(lib.pxa_row_reduce_workspace_bytes(r1 - r0, n))
        work = torch.empty((max(wsz // 8, 1),), dtype=torch.float64, device=x.device)
        check(lib.pxa_row_reduce_pow(dtcode(x), r1 - r0, n, float(p), ptr(x) + r0 * n * es,
                                     (ptr(y) + r0 * n * es) if y is not None else None, out.data_ptr() + r0 * 8,
                                     ptr(work), stream()), "pxa_row_reduce_pow")
    return out


# ------------------------------------------------------------------ stencils
def stencil_axis(x, y, stack, shape, axis, offsets, coefs, zero_partial=False, xs=None, ys=None, beta=0.0, x_off=0, y_off=0):
    """One separable-axis pass (see pxa_stencil_axis).  `x_off`/`y_off`: element offsets into x/y."""
    N = int(np.prod(shape))
    es = x.element_size()
    check(
        lib.pxa_stencil_axis(
            dtcode(x), stack, len(shape), i64_array(shape), axis, len(offsets), i32_array(offsets), f64_array(coefs),
            int(zero_partial), ptr(x) + x_off * es, N if xs is None else xs, ptr(y) + y_off * es, N if ys is None else ys,
            float(beta), stream(),
        ),
        "pxa_stencil_axis",
    )
    return y


def stencil_sep(x, y, stack, shape, taps, beta=0.0, xs=None, ys=None, x_off=0, y_off=0):
    """Separable constant-mode filter; taps[d] = (offsets, coefs) or None (identity axis)."""
    torch = _torch()
    D = len(shape)
    MT = 64
    ntaps = [0 if t is None else len(t[0]) for t in taps]
    offs = [0] * (D * MT)
    cfs = [0.0] * (D * MT)
    for d, t in enumerate(taps):
        if t is not None:
            for q, (o, c) in enumerate(zip(*t)):
                offs[d * MT + q] = o
                cfs[d * MT + q] = c
    N = int(np.prod(shape))
    wsz = int(lib.pxa_stencil_sep_workspace_bytes(dtcode(x), stack, D, i64_array(shape), int_array(ntaps)))
    work = torch.empty((max(wsz, 1),), dtype=torch.uint8, device=x.device) if wsz else None
    es = x.element_size()
    check(
        lib.pxa_stencil_sep(
            dtcode(x), stack, D, i64_array(shape), int_array(ntaps), i32_array(offs), f64_array(cfs),
            ptr(x) + x_off * es, N if xs is None else xs, ptr(y) + y_off * es, N if ys is None else ys, float(beta),
            ptr(work) if work is not None else None, stream(),
        ),
        "pxa_stencil_sep",
    )
    return y


def stencil_nd(x, y, stack, shape, offsets_dev, coefs_dev, zero_partial=False, beta=0.0, xs=None, ys=None, x_off=0, y_off=0,
               off_lo=None, off_hi=None):
    """N-D stencil; with the tap offsets' per-axis range (off_lo / off_hi, host ints) pxa_stencil_nd_box, which
    runs the LDS-tiled kernel where it applies."""
    N = int(np.prod(shape))
    ntaps = coefs_dev.numel()
    es = x.element_size()
    if off_lo is not None and off_hi is not None:
        lo, hi = (np.ascontiguousarray(v, dtype=np.int32) for v in (off_lo, off_hi))
        check(
            lib.pxa_stencil_nd_box(
                dtcode(x), stack, len(shape), i64_array(shape), ntaps, ptr(offsets_dev), ptr(coefs_dev),
                lo.ctypes.data, hi.ctypes.data, int(zero_partial), ptr(x) + x_off * es, N if xs is None else xs,
                ptr(y) + y_off * es, N if ys is None else ys, float(beta), stream(),
            ),
            "pxa_stencil_nd_box",
        )
        return y
    check(
        lib.pxa_stencil_nd(
            dtcode(x), stack, len(shape), i64_array(shape), ntaps, ptr(offsets_dev), ptr(coefs_dev), int(zero_partial),
            ptr(x) + x_off * es, N if xs is None else xs, ptr(y) + y_off * es, N if ys is None else ys, float(beta), stream(),
        ),
        "pxa_stencil_nd",
    )
    return y


def pad(x, stack, shape, lo, hi, modes):
    pshape = [n + l + h for n, l, h in zip(shape, lo, hi)]
    y = empty((stack * int(np.prod(pshape)),), x)
    check(
        lib.pxa_pad(dtcode(x), stack, len(shape), i64_array(shape), i64_array(lo), i64_array(hi),
                    int_array([MODES[m] for m in modes]), ptr(x), ptr(y), stream()),
        "pxa_pad",
    )
    return y


def pad_adjoint(x, stack, shape, lo, hi, modes):
    y = empty((stack * int(np.prod(shape)),), x)
    work = empty((x.numel(),), x)
    check(
        lib.pxa_pad_adjoint(dtcode(x), stack, len(shape), i64_array(shape), i64_array(lo), i64_array(hi),
                            int_array([MODES[m] for m in modes]), ptr(x), ptr(y), ptr(work), stream()),
        "pxa_pad_adjoint",
    )
    return y


def trim(x, stack, big_shape, lo, hi, embed):
    core = [n - l - h for n, l, h in zip(big_shape, lo, hi)]
    n_out = int(np.prod(big_shape if embed else core))
    y = empty((stack * n_out,), x)
    check(
        lib.pxa_trim(dtcode(x), stack, len(big_shape), i64_array(big_shape), i64_array(lo), i64_array(hi), int(embed),
                     ptr(x), ptr(y), stream()),
        "pxa_trim",
    )
    return y


def gather_cols(x, idx, out=None):
    """out[r, j] = x[r, idx[j]] for x (rows, n) and device int64 idx (m,)."""
    x = require(x)
    n = x.shape[-1]
    rows = int(np.prod(x.shape[:-1]))
    m = idx.numel()
    out = empty((*x.shape[:-1], m), x) if out is None else out
    check(lib.pxa_gather_cols(dtcode(x), rows, n, ptr(x), m, ptr(idx), ptr(out), stream()), "pxa_gather_cols")
    return out


def scatter_cols(y, idx, n, out=None):
    """out (rows, n) = 0 then out[r, idx[j]] = y[r, j] (idx unique)."""
    y = require(y)
    m = y.shape[-1]
    rows = int(np.prod(y.shape[:-1]))
    out = empty((*y.shape[:-1], n), y) if out is None else out
    check(lib.pxa_scatter_cols(dtcode(y), rows, m, ptr(y), n, ptr(idx), ptr(out), stream()), "pxa_scatter_cols")
    return out


# ------------------------------------------------------------------ gradient
def gradient2(x, stack, shape, dirs, o0, c0, o1, c1, adjoint=False):
    D = len(dirs)
    N = int(np.prod(shape))
    out = empty((stack * (N if adjoint else D * N),), x)
    fn = lib.pxa_gradient2_adjoint if adjoint else lib.pxa_gradient2
    check(
        fn(dtcode(x), stack, len(shape), i64_array(shape), D, int_array(dirs), int_array(o0), f64_array(c0),
           int_array(o1), f64_array(c1), ptr(x), ptr(out), stream()),
        "pxa_gradient2",
    )
    return out


# ------------------------------------------------------------------ dense
def dense_matmat(A, X, trans):
    """trans=0: Y = X A^T (X: (B, N)); trans=1: Y = X A (X: (B, M))."""
    torch = _torch()
    M, N = A.shape
    B = X.shape[0]
    Y = empty((B, N if trans else M), X)
    wsz = int(lib.pxa_dense_workspace_bytes(dtcode(X), int(trans), M, N, B))
    work = torch.empty((max(wsz, 1),), dtype=torch.uint8, device=X.device) if wsz else None
    check(
        lib.pxa_dense_matmat(dtcode(X), int(trans), M, N, B, ptr(A), ptr(X), ptr(Y), ptr(work) if work is not None else None, stream()),
        "pxa_dense_matmat",
    )
    return Y


def dense_normal_supported(A, x):
    """True when pxa_dense_normal takes (A, x): one fp32 right-hand side, N % 4 == 0, N <= 65536."""
    M, N = A.shape
    B = x.numel() // max(N, 1)
    return (A.dtype == x.dtype and x.shape[-1] == N and B == 1 and A.is_contiguous() and x.is_contiguous()
            and int(lib.pxa_dense_normal_workspace_bytes(dtcode(x), M, N, 1)) > 0)


def dense_normal(A, x, s, d, work=None, pdot=None):
    """Y = s * A^T (A x) + d * x in one pass over A (pxa_dense_normal); `work`: a reusable uint8 device
    buffer of at least pxa_dense_normal_workspace_bytes bytes (allocated when None).  pdot: a float64 device
    buffer that receives the CG's <x, Y> partials in the same launches (pxa_dense_normal_pdot, for
    cg_update(..., have_pap=True) with pdot as its work)."""
    torch = _torch()
    M, N = A.shape
    wsz = int(lib.pxa_dense_normal_workspace_bytes(dtcode(x), M, N, 1))
    if wsz == 0:
        raise ValueError("pxa_dense_normal: unsupported operand (see dense_normal_supported)")
    if work is None or work.numel() < wsz:
        work = torch.empty((wsz,), dtype=torch.uint8, device=x.device)
    Y = empty(x.shape, x)
    if pdot is None:
        check(lib.pxa_dense_normal(dtcode(x), M, N, 1, ptr(A), ptr(x), float(s), float(d), ptr(Y), ptr(work), stream()),
              "pxa_dense_normal")
    else:
        assert pdot.dtype == torch.float64 and pdot.is_cuda
        check(lib.pxa_dense_normal_pdot(dtcode(x), M, N, ptr(A), ptr(x), float(s), float(d), ptr(Y), ptr(work),
                                        pdot.data_ptr(), stream()), "pxa_dense_normal_pdot")
    return Y


# ------------------------------------------------------------------ fused solver steps
def pgd_tv2d_args(stack, y_images, n0, n1, taps0, taps1, h0, h1, lam, mu, prox, prox_w):
    """Pre-built ctypes arguments of the iteration-invariant part of pxa_pgd_tv2d_step."""
    o0, k0 = taps0
    o1, k1 = taps1
    return (int(stack), int(y_images), int(n0), int(n1), len(o0), i32_array(o0), f64_array(k0), len(o1), i32_array(o1),
            f64_array(k1), float(h0), float(h1), float(lam), float(mu))


def pgd_tv2d_step(x, x_prev, hty, x_new, stack, y_images, n0, n1, taps0, taps1, h0, h1, lam, mu, a, tau, prox, prox_w, partials=None,
                  pre=None, x_ref=None):
    """One fused PGD iteration (pxa_pgd_tv2d_step).  `pre`: pgd_tv2d_args(...) cached by the caller.  With
    `partials`, the per-tile RelError statistics are taken against `x_ref` (None: against x)."""
    if pre is None:
        pre = pgd_tv2d_args(stack, y_images, n0, n1, taps0, taps1, h0, h1, lam, mu, prox, prox_w)
    ev = _TIMER.begin() if _TIMER is not None else None  # measurement hook (bench.py), normally None
    check(
        lib.pxa_pgd_tv2d_step(
            dtcode(x), *pre, float(a), float(tau), int(prox), float(prox_w),
            x.data_ptr(), x_prev.data_ptr(), hty.data_ptr(), x_new.data_ptr(), ptr(partials) if partials is not None else None,
            x_ref.data_ptr() if x_ref is not None else None, stream(),
        ),
        "pxa_pgd_tv2d_step",
    )
    if ev is not None:
        _TIMER.end(ev)
    return x_new


class PgdPlan:
    """pxa_pgd_tv2d_plan: the fused PGD step's iteration-invariant parameters, prepared once per solve, and the
    device counter of its last-workgroup RelError fold.  ``step`` is one iteration (pxa_pgd_tv2d_plan_step) with
    the few per-step arguments, so a PGD step costs one short ctypes call."""

    def __init__(self, like, stack, y_images, n0, n1, taps0, taps1, h0, h1, lam, mu, prox):
        o0, k0 = taps0
        o1, k1 = taps1
        h = ct.c_void_p()
        check(lib.pxa_pgd_tv2d_plan(dtcode(like), int(stack), int(y_images), int(n0), int(n1), len(o0), i32_array(o0),
                                    f64_array(k0), len(o1), i32_array(o1), f64_array(k1), float(h0), float(h1),
                                    float(lam), float(mu), int(prox), ct.byref(h)), "pxa_pgd_tv2d_plan")
        self._h = h.value
        self._fn = lib.pxa_pgd_tv2d_plan_step
        self._fn_fold = lib.pxa_pgd_tv2d_plan_step_fold
        self._free = lib.pxa_pgd_tv2d_plan_free

    def step(self, x, x_prev, hty, x_new, a, tau, prox_w, partials=None, x_ref=None, sink=None, seq=0,
             fold_launch=False):
        """One iteration; with `sink` (a HostFlagBuffer of (2, rows) values) its partials are also folded there
        under publication `seq`: by the launch's last workgroup, or with `fold_launch` by a fold launch enqueued
        behind it in the same C call (pxa_pgd_tv2d_plan_step_fold)."""
        ev = _TIMER.begin() if _TIMER is not None else None  # measurement hook (bench.py), normally None
        r = (self._fn_fold if fold_launch else self._fn)(self._h, float(a), float(tau), float(prox_w), x.data_ptr(), x_prev.data_ptr(), hty.data_ptr(),
                     x_new.data_ptr(), partials.data_ptr() if partials is not None else None,
                     x_ref.data_ptr() if x_ref is not None else None, sink.vptr if sink is not None else None,
                     sink.fptr if sink is not None else None, int(seq), stream())
        if r:
            check(r, "pxa_pgd_tv2d_plan_step")
        if ev is not None:
            _TIMER.end(ev)
        return x_new

    def step_wpub(self, x, x_prev, hty, x_new, a, tau, prox_w, partials, prev=None):
        """One iteration with window partials into `partials`; `prev` = (partials of the previous such launch,
        HostFlagBuffer, seq): folded and published by an extra workgroup of this launch
        (pxa_pgd_tv2d_plan_step_wpub)."""
        ev = _TIMER.begin() if _TIMER is not None else None
        pp, fb, seq = prev if prev is not None else (None, None, 0)
        r = lib.pxa_pgd_tv2d_plan_step_wpub(self._h, float(a), float(tau), float(prox_w), x.data_ptr(), x_prev.data_ptr(),
                                            hty.data_ptr(), x_new.data_ptr(), partials.data_ptr(),
                                            pp.data_ptr() if pp is not None else None, fb.vptr if fb is not None else None,
                                            fb.fptr if fb is not None else None, int(seq), stream())
        if r:
            check(r, "pxa_pgd_tv2d_plan_step_wpub")
        if ev is not None:
            _TIMER.end(ev)
        return x_new

    def step_window(self, x, x_prev, hty, x_new, a, tau, prox_w, partials, sink, seq):
        """One iteration whose partials are the RelError statistics of the (x, x_prev) pair it reads -- the stop
        check before it -- folded into `sink` under publication `seq` by a fold launch behind it
        (pxa_pgd_tv2d_plan_step_wfold)."""
        ev = _TIMER.begin() if _TIMER is not None else None
        r = lib.pxa_pgd_tv2d_plan_step_wfold(self._h, float(a), float(tau), float(prox_w), x.data_ptr(), x_prev.data_ptr(),
                                             hty.data_ptr(), x_new.data_ptr(), partials.data_ptr(), sink.vptr, sink.fptr,
                                             int(seq), stream())
        if r:
            check(r, "pxa_pgd_tv2d_plan_step_wfold")
        if ev is not None:
            _TIMER.end(ev)
        return x_new

    def __del__(self):
        if getattr(self, "_h", None):
            self._free(self._h)
            self._h = None


_PDS_W = 17  # per-axis tap slots of pxa_pds_step (2 * 8 + 1)


def pds_args(stack, y_images, n0, n1, n2, D, taps, c0, c1, tau, sigma, rho, lam, prox, prox_w, h_kind):
    """Pre-built ctypes arguments of pxa_pds_step (everything but the arrays)."""
    offs, cfs = [], []
    for o, c in taps:
        offs += list(o) + [0] * (_PDS_W - len(o))
        cfs += list(c) + [0.0] * (_PDS_W - len(c))
    return (i64_array([stack, y_images, n0, n1, n2, D]), i32_array([len(t[0]) for t in taps]), i32_array(offs),
            f64_array(cfs), f64_array(list(c0) + list(c1)), f64_array([tau, sigma, rho, lam, prox_w]), int(prox),
            int(h_kind))


def pds_step(algo, pre, x, u, z, hty, x_out, u_out, z_out, work_q, work_w, nseg=0):
    """One fused PD3O (algo 0) / Condat-Vu (algo 1) iteration (pxa_pds_step); `pre` from pds_args."""
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    ev = _TIMER.begin() if _TIMER is not None else None
    check(lib.pxa_pds_step(dtcode(z), int(algo), *pre, p(x), p(u), p(z), p(hty), p(x_out), p(u_out), p(z_out),
                           p(work_q), p(work_w), int(nseg), stream()), "pxa_pds_step")
    if ev is not None:
        _TIMER.end(ev)


def pds_step_la(algo, pre, primed, x, u, z, hty, x_out, u_out, z_out, work_q, work_kt, work_w, nseg=0):
    """One look-ahead PD3O / Condat-Vu iteration (pxa_pds_step_la): kernel B + kernel D (dual update fused
    with the next iteration's axis-0 march); `primed` = the previous call left x / work_q / work_kt."""
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    ev = _TIMER.begin() if _TIMER is not None else None
    check(lib.pxa_pds_step_la(dtcode(z), int(algo), *pre, int(bool(primed)), p(x), p(u), p(z), p(hty), p(x_out),
                              p(u_out), p(z_out), p(work_q), p(work_kt), p(work_w), int(nseg), stream()),
          "pxa_pds_step_la")
    if ev is not None:
        _TIMER.end(ev)


def tv_dual_update(w, z, geom, c0, c1, sigma, lam, rho, h_kind, relax=0, out=None):
    """z_out = relax(fenchel_prox_{sigma h}(z + sigma Grad w)), h = lam L1 (h_kind 0) / lam L21 (1):
    the PDS dual update alone (pxa_tv_dual_update).  geom = (stack, n0, n1, n2, D); relax 0 PD3O, 1 CV."""
    w = require(w, "w")
    z = require(z, "z")
    if w.dtype != z.dtype:
        raise TypeError("pyxu_amd: w and z must share a dtype")
    stack, n0, n1, n2, D = (int(v) for v in geom)
    if w.numel() != stack * n0 * n1 * n2 or z.numel() != D * w.numel():
        raise ValueError(f"pyxu_amd: tv_dual_update geometry {tuple(geom)} does not match w {tuple(w.shape)}, "
                         f"z {tuple(z.shape)}")
    out = empty_like(z) if out is None else require(out, "out")
    check(lib.pxa_tv_dual_update(dtcode(z), int(relax), i64_array([stack, n0, n1, n2, D]),
                                 f64_array(list(c0) + list(c1)), float(sigma), float(lam), float(rho), int(h_kind),
                                 ptr(w), ptr(z), ptr(out), stream()), "pxa_tv_dual_update")
    return out


def pds_kernel_ms(reset=True):
    """(steps, [ms A, ms B, ms C] summed) of the pxa_pds_step calls recorded under TUNE_PDS_EVENTS."""
    buf = (ct.c_double * 3)()
    n = int(lib.pxa_pds_kernel_ms(ct.cast(buf, ct.c_void_p), int(bool(reset))))
    if n < 0:
        check(n, "pxa_pds_kernel_ms")
    return n, [buf[0], buf[1], buf[2]]


# ------------------------------------------------------------------ FFT
def fft(z, shape, axes, stack, inverse, out=None):
    """Unnormalised DFT over `axes` of `stack` complex arrays of `shape`, interleaved (re, im) real
    tensors (pxa_fft).  inverse=False: exp(-2 pi i ..) (fftn, norm="backward"); True: exp(+..)
    (ifftn, norm="forward")."""
    torch = _torch()
    z = require(z, "z")
    out = empty_like(z) if out is None else out
    sh, ax = i64_array(shape), int_array(axes)
    wsz = int(lib.pxa_fft_workspace_bytes(dtcode(z), len(shape), sh, len(axes), ax, int(stack)))
    if wsz == (1 << 64) - 1:  # (size_t)-1: arguments outside the envelope
        check(-3, "pxa_fft_workspace_bytes")  # PXA_ERR_UNSUPPORTED
    work = torch.empty((wsz,), dtype=torch.uint8, device=z.device) if wsz > 0 else None
    check(lib.pxa_fft_ex(dtcode(z), len(shape), sh, len(axes), ax, int(stack), int(bool(inverse)), ptr(z), ptr(out),
                         ptr(work) if work is not None else None, stream()), "pxa_fft_ex")
    return out


def real_to_complex(x):
    x = require(x, "x")
    z = empty((*x.shape[:-1], 2 * x.shape[-1]), x)
    check(lib.pxa_real_to_complex(dtcode(x), x.numel(), ptr(x), ptr(z), stream()), "pxa_real_to_complex")
    return z


def complex_real_part(z):
    z = require(z, "z")
    x = empty((*z.shape[:-1], z.shape[-1] // 2), z)
    check(lib.pxa_complex_real_part(dtcode(z), x.numel(), ptr(z), ptr(x), stream()), "pxa_complex_real_part")
    return x


def complex_mul(a, b, conj_b=False, out=None):
    """out = a * b (b broadcast over a's leading stack) for interleaved complex tensors."""
    a, b = require(a, "a"), require(b, "b")
    out = empty_like(a) if out is None else out
    check(lib.pxa_complex_mul(dtcode(a), a.numel() // 2, b.numel() // 2, ptr(a), ptr(b), int(bool(conj_b)), ptr(out),
                              stream()), "pxa_complex_mul")
    return out


_tuning_from_env()
