"""
ctypes binding of ``libpyxu_amd.so`` — the C-ABI declared in ``include/pyxu_amd.h``.

The library is the ONLY compute path of this package.  If it is missing or fails to load, every
compute call raises :py:class:`BackendUnavailable`; there is no CPU fallback.
"""
import ctypes as ct
import os
import threading

__all__ = ["lib", "check", "BackendUnavailable", "LIB_PATH", "EXPORTS"]

# PXA_LIB_PATH: the probe build of scripts/ (csrc/Makefile `probe`); the product loads the in-tree library
LIB_PATH = os.environ.get("PXA_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpyxu_amd.so")

i32, i64, f64, vp, sz = ct.c_int, ct.c_int64, ct.c_double, ct.c_void_p, ct.c_size_t
P_i64 = ct.POINTER(ct.c_int64)
P_i32 = ct.POINTER(ct.c_int32)
P_int = ct.POINTER(ct.c_int)
P_f64 = ct.POINTER(ct.c_double)

# name -> (restype, argtypes); must list every function of include/pyxu_amd.h
EXPORTS = {
    "pxa_version": (ct.c_char_p, []),
    "pxa_error_string": (ct.c_char_p, [i32]),
    "pxa_abi_version": (i32, []),
    "pxa_tuning": (i32, [i32, i32]),
    "pxa_axpby": (i32, [i32, i64, f64, vp, f64, vp, vp, vp]),
    "pxa_axpby_bcast": (i32, [i32, i64, f64, vp, f64, vp, i64, vp, vp]),
    "pxa_axpy_rows": (i32, [i32, i64, i64, vp, f64, vp, vp, vp, vp]),
    "pxa_row_ratio": (i32, [i32, i64, vp, vp, vp, vp]),
    "pxa_lincomb3": (i32, [i32, i64, f64, vp, f64, vp, f64, vp, vp, vp]),
    "pxa_extrapolate": (i32, [i32, i64, f64, vp, vp, vp, vp]),
    "pxa_div": (i32, [i32, i64, vp, f64, vp, vp]),
    "pxa_add_scalar": (i32, [i32, i64, vp, f64, vp, vp]),
    "pxa_fill": (i32, [i32, i64, f64, vp, vp]),
    "pxa_mul": (i32, [i32, i64, vp, vp, vp, vp]),
    "pxa_clip": (i32, [i32, i64, vp, f64, f64, i32, vp, vp]),
    "pxa_prox_l1": (i32, [i32, i64, vp, f64, vp, vp]),
    "pxa_admm_l1_update": (i32, [i32, i64, vp, vp, vp, vp, f64, f64, f64, vp, vp]),
    "pxa_prox_l21": (i32, [i32, i64, i64, i64, vp, f64, vp, vp]),
    "pxa_fenchel_prox_l1": (i32, [i32, i64, vp, f64, f64, vp, vp]),
    "pxa_fenchel_prox_l21": (i32, [i32, i64, i64, i64, vp, f64, f64, vp, vp]),
    "pxa_moreau_grad_l1": (i32, [i32, i64, vp, f64, f64, vp, vp]),
    "pxa_moreau_grad_l21": (i32, [i32, i64, i64, i64, vp, f64, f64, vp, vp]),
    "pxa_group_norm": (i32, [i32, i64, i64, i64, vp, vp, vp]),
    "pxa_row_reduce_workspace_bytes": (sz, [i64, i64]),
    "pxa_row_reduce": (i32, [i32, i32, i64, i64, vp, vp, vp, vp, vp]),
    "pxa_row_reduce_pow": (i32, [i32, i64, i64, f64, vp, vp, vp, vp, vp]),
    "pxa_relerr_stats_workspace_bytes": (sz, [i64, i64]),
    "pxa_relerr_stats": (i32, [i32, i64, i64, vp, vp, vp, vp, vp, vp]),
    "pxa_tile_partials_fold": (i32, [i64, i64, vp, vp, vp, ct.c_uint32, vp]),
    "pxa_host_alloc": (i32, [sz, ct.POINTER(vp)]),
    "pxa_host_free": (i32, [vp]),
    "pxa_cg_update_workspace_bytes": (sz, [i64]),
    "pxa_cg_update": (i32, [i32, i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, ct.c_uint32, vp, vp]),
    "pxa_cg_update_tail": (i32, [i32, i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, ct.c_uint32, vp, vp]),
    "pxa_cg_update_xr": (i32, [i32, i64, i64, vp, vp, vp, vp, vp, vp, vp]),
    "pxa_stencil_axis": (i32, [i32, i64, i32, P_i64, i32, i32, P_i32, P_f64, i32, vp, i64, vp, i64, f64, vp]),
    "pxa_stencil_sep_workspace_bytes": (sz, [i32, i64, i32, P_i64, P_int]),
    "pxa_stencil_sep": (i32, [i32, i64, i32, P_i64, P_int, P_i32, P_f64, vp, i64, vp, i64, f64, vp, vp]),
    "pxa_stencil_nd": (i32, [i32, i64, i32, P_i64, i32, vp, vp, i32, vp, i64, vp, i64, f64, vp]),
    "pxa_stencil_nd_box": (i32, [i32, i64, i32, P_i64, i32, vp, vp, vp, vp, i32, vp, i64, vp, i64, f64, vp]),
    "pxa_pad": (i32, [i32, i64, i32, P_i64, P_i64, P_i64, P_int, vp, vp, vp]),
    "pxa_pad_adjoint": (i32, [i32, i64, i32, P_i64, P_i64, P_i64, P_int, vp, vp, vp, vp]),
    "pxa_trim": (i32, [i32, i64, i32, P_i64, P_i64, P_i64, i32, vp, vp, vp]),
    "pxa_gather_cols": (i32, [i32, i64, i64, vp, i64, vp, vp, vp]),
    "pxa_scatter_cols": (i32, [i32, i64, i64, vp, i64, vp, vp, vp]),
    "pxa_gradient2": (i32, [i32, i64, i32, P_i64, i32, P_int, P_int, P_f64, P_int, P_f64, vp, vp, vp]),
    "pxa_gradient2_adjoint": (i32, [i32, i64, i32, P_i64, i32, P_int, P_int, P_f64, P_int, P_f64, vp, vp, vp]),
    "pxa_dense_workspace_bytes": (sz, [i32, i32, i64, i64, i64]),
    "pxa_dense_matmat": (i32, [i32, i32, i64, i64, i64, vp, vp, vp, vp, vp]),
    "pxa_dense_normal_workspace_bytes": (sz, [i32, i64, i64, i64]),
    "pxa_dense_normal": (i32, [i32, i64, i64, i64, vp, vp, f64, f64, vp, vp, vp]),
    "pxa_dense_normal_pdot": (i32, [i32, i64, i64, vp, vp, f64, f64, vp, vp, vp, vp]),
    "pxa_dense_normal_pdot_pfold": (i32, [i32, i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, ct.c_uint32, f64, f64, vp, vp,
                                          vp, vp]),
    "pxa_copy2d": (i32, [i32, i64, i64, vp, i64, i64, vp, i64, i32, vp]),
    "pxa_unary": (i32, [i32, i32, i64, vp, vp, vp]),
    "pxa_binary": (i32, [i32, i32, i64, vp, f64, vp, f64, vp, vp]),
    "pxa_where": (i32, [i32, i64, vp, vp, f64, vp, f64, vp, vp]),
    "pxa_cast": (i32, [i32, i32, i64, vp, vp, vp]),
    "pxa_isnan": (i32, [i32, i64, vp, vp, vp]),
    "pxa_bool_reduce": (i32, [i64, i32, vp, vp, vp]),
    "pxa_set_diag": (i32, [i32, i64, i64, i64, f64, vp, vp]),
    "pxa_transpose": (i32, [i32, i64, i64, vp, vp, vp]),
    "pxa_dir_contract": (i32, [i32, i64, i64, i64, i64, i64, vp, i64, vp, vp, i32, vp]),
    "pxa_pgd_tv2d_partials_count": (i32, [i64, i64, i64]),
    "pxa_pgd_tv2d_last_kernel": (i32, []),
    "pxa_pgd_tile_trace": (i32, [vp, i32]),
    "pxa_pgd_tv2d_plan": (i32, [i32, i64, i64, i64, i64, i32, P_i32, P_f64, i32, P_i32, P_f64, f64, f64, f64, f64, i32,
                                ct.POINTER(vp)]),
    "pxa_pgd_tv2d_plan_step": (i32, [vp, f64, f64, f64, vp, vp, vp, vp, vp, vp, vp, vp, ct.c_uint32, vp]),
    "pxa_pgd_tv2d_plan_step_fold": (i32, [vp, f64, f64, f64, vp, vp, vp, vp, vp, vp, vp, vp, ct.c_uint32, vp]),
    "pxa_pgd_tv2d_plan_step_wfold": (i32, [vp, f64, f64, f64, vp, vp, vp, vp, vp, vp, vp, ct.c_uint32, vp]),
    "pxa_pgd_tv2d_plan_step_wpub": (i32, [vp, f64, f64, f64, vp, vp, vp, vp, vp, vp, vp, vp, ct.c_uint32, vp]),
    "pxa_pgd_tv2d_plan_free": (i32, [vp]),
    "pxa_pgd_tv2d_step": (
        i32,
        [i32, i64, i64, i64, i64, i32, P_i32, P_f64, i32, P_i32, P_f64, f64, f64, f64, f64, f64, f64, i32, f64,
         vp, vp, vp, vp, vp, vp, vp],
    ),
    "pxa_fft": (i32, [i32, i32, P_i64, i32, P_int, i64, i32, vp, vp, vp]),
    "pxa_fft_workspace_bytes": (sz, [i32, i32, P_i64, i32, P_int, i64]),
    "pxa_fft_ex": (i32, [i32, i32, P_i64, i32, P_int, i64, i32, vp, vp, vp, vp]),
    "pxa_complex_mul": (i32, [i32, i64, i64, vp, vp, i32, vp, vp]),
    "pxa_real_to_complex": (i32, [i32, i64, vp, vp, vp]),
    "pxa_complex_real_part": (i32, [i32, i64, vp, vp, vp]),
    "pxa_pds_kernel_ms": (i32, [vp, i32]),
    "pxa_pds_step": (
        i32,
        [i32, i32, P_i64, P_i32, P_i32, P_f64, P_f64, P_f64, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp],
    ),
    "pxa_tv_dual_update": (i32, [i32, i32, P_i64, P_f64, f64, f64, f64, i32, vp, vp, vp, vp]),
    "pxa_pds_step_la": (
        i32,
        [i32, i32, P_i64, P_i32, P_i32, P_f64, P_f64, P_f64, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
         i32, vp],
    ),
}


class BackendUnavailable(RuntimeError):
    """The HIP C-ABI library could not be loaded (no silent fallback exists)."""


class _Lib:
    def __init__(self):
        self._handle = None
        self._err = None
        self._lock = threading.Lock()

    def _load(self):
        with self._lock:
            if self._handle is not None or self._err is not None:
                return
            try:
                h = ct.CDLL(LIB_PATH, mode=ct.RTLD_GLOBAL)
                fns = {}
                for name, (res, args) in EXPORTS.items():
                    fn = getattr(h, name)
                    fn.restype = res
                    fn.argtypes = args
                    fns[name] = fn
                self._handle = h
                self.__dict__.update(fns)  # later lookups bypass __getattr__ (no lock on the hot path)
            except OSError as e:  # missing / unloadable .so
                self._err = e

    @property
    def loaded(self) -> bool:
        self._load()
        return self._handle is not None

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        self._load()
        if self._handle is None:
            raise BackendUnavailable(
                f"pyxu_amd: HIP library not available at {LIB_PATH} ({self._err}). "
                "Build it with `python -c 'import __graft_entry__ as g; g.build()'` (or `make -C pyxu_amd/csrc`)."
            )
        return getattr(self._handle, name)


lib = _Lib()


def check(code: int, where: str = ""):
    """Raise RuntimeError for a non-zero status returned by the C-ABI."""
    if code != 0:
        msg = lib.pxa_error_string(int(code)).decode()
        raise RuntimeError(f"{where}: {msg} (code {code})" if where else f"{msg} (code {code})")


def i64_array(vals):
    vals = [int(v) for v in vals]
    return (ct.c_int64 * max(1, len(vals)))(*vals)


def i32_array(vals):
    vals = [int(v) for v in vals]
    return (ct.c_int32 * max(1, len(vals)))(*vals)


def int_array(vals):
    vals = [int(v) for v in vals]
    return (ct.c_int * max(1, len(vals)))(*vals)


def f64_array(vals):
    vals = [float(v) for v in vals]
    return (ct.c_double * max(1, len(vals)))(*vals)
