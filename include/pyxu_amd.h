/*
 * pyxu_amd — C-ABI of the MI355X (gfx950) proximal-splitting backend.
 *
 * This is the drop-in boundary for Pyxu's proximal-splitting hot path.
 * Every entry point is a plain `extern "C"` function over raw device pointers and sizes:
 *   - returns 0 on success, a HIP error code (>0) or a PXA_ERR_* code (<0) on failure
 *     (pxa_error_string() gives a message); no exception crosses the ABI;
 *   - the caller owns every buffer (device pointers, e.g. torch-ROCm `data_ptr()`); scratch space is
 *     passed in explicitly.  The compute entry points never allocate device memory and never
 *     synchronise, so they are graph-capturable, including the first call on a new FFT length (its
 *     twiddle table lives in static device memory of the library and is filled by a kernel enqueued on
 *     the caller's stream: tests/test_gpu_fft.py::test_fft_graph_capture_cold_length).  The exceptions,
 *     all outside the compute calls or behind measurement knobs:
 *       * pxa_pgd_tv2d_plan() allocates the plan's 4-byte device counter (released by
 *         pxa_pgd_tv2d_plan_free()); call it before a capture, then capture pxa_pgd_tv2d_plan_step();
 *       * pxa_host_alloc() / pxa_host_free() allocate / release coherent host memory (their purpose);
 *       * pxa_tuning(PXA_TUNE_PDS_MARCH, bit 2), the opt-in coupled kernel-D variant of A/B runs,
 *         allocates its progress counters on first use;
 *       * pxa_pds_kernel_ms() and pxa_pgd_tile_trace() (measurement hooks) wait for recorded events /
 *         copy a device symbol to the host;
 *   - `stream` is a hipStream_t (NULL = legacy default stream); launches are asynchronous;
 *   - functions are re-entrant (safe from Pyxu's solver worker thread, reference
 *     src/pyxu/abc/solver.py:710-718);
 *   - arrays are C-contiguous, laid out exactly as the reference's NDArrays: a leading stack of
 *     independent problems followed by the row-major flattening of `arg_shape`
 *     (reference src/pyxu/operator/linop/stencil/stencil.py:441-461).
 *
 * dtype codes: PXA_F32 (float) and PXA_F64 (double), mirroring pyxu.runtime.Width
 * (reference src/pyxu/runtime/_runtime.py:25-45).
 *
 * Reference interfaces replaced are cited per function (paths under /root/reference/src/pyxu).
 */
#ifndef PYXU_AMD_H
#define PYXU_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PXA_F32 0
#define PXA_F64 1

#define PXA_OK 0
#define PXA_ERR_ARG (-1)         /* invalid argument (shape, count, null pointer, ...) */
#define PXA_ERR_DTYPE (-2)       /* unsupported dtype code */
#define PXA_ERR_UNSUPPORTED (-3) /* valid request outside this build's supported envelope */

#define PXA_MAX_DIM 4    /* spatial rank supported by stencil / gradient kernels */
#define PXA_MAX_TAPS 64  /* taps per separable-axis pass (kernel-argument resident) */

/* Boundary modes of Pad (operator/linop/pad.py:145-160). */
#define PXA_MODE_CONSTANT 0
#define PXA_MODE_WRAP 1
#define PXA_MODE_REFLECT 2
#define PXA_MODE_SYMMETRIC 3
#define PXA_MODE_EDGE 4

/* Kernel-selection knobs (pxa_tuning). */
#define PXA_TUNE_PGD_KERNEL 0 /* fused PGD step (pxa_pgd_tv2d_step / _plan_step): 0 / 1 the tile kernel (default); v >= 2 the
                                * strip kernel with strips of v tiles (a workgroup walks a column strip, keeping the shared
                                * window rows in LDS and prefetching each next tile's new rows; 16-B aligned rows only, else
                                * the tile kernel).  Same bits; measured slower (A/B and tests only). */
#define PXA_TUNE_NORMAL_KERNEL 1 /* A/B of pxa_dense_normal: 0 row-split kernel (each row in four column parts,
                                    one workgroup each, part-dots exchanged), 1 one workgroup per row (results
                                    equal up to summation order), 2 the row-split kernel computing every part-dot
                                    in every member instead of exchanging (the same bits as 0) */
#define PXA_TUNE_DENSE_KERNEL 2 /* A/B of the fp32 MFMA dense path (pxa_dense_matmat, B >= 32): 0 the LDS-staged
                                   kernel, 1 the register-streamed kernel of rounds 1-3 (same results up to
                                   summation order) */
#define PXA_TUNE_DUAL_WGS 4 /* A/B of the PDS dual-update kernel C: workgroups it aims for when it splits the
                               axis-0 march into segments (0: 2048) */
#define PXA_TUNE_PGD_DIAG 3 /* fused PGD tile kernel, PROBE BUILD ONLY (make -C pyxu_amd/csrc probe; the production
                              library ignores it): bit 5 s_memtime phase trace (pxa_pgd_tile_trace); timing probes
                              with WRONG results: bit 6 skips passes A / B, bit 7 the window loads, bit 8 loads x only,
                              bit 9 the H^T y loads, bit 10 the x_new stores (scripts/pgd_modes_probe.py diag) */
#define PXA_TUNE_PGD_STAGGER 6 /* fused PGD tile kernel A/B probe, PROBE BUILD ONLY: v = (sel << 8) | n delays the
                                  workgroups picked by `sel` in the first dispatch round by n x 1024 cycles */
#define PXA_TUNE_PDS_EVENTS 5 /* measurement hook: > 0 makes pxa_pds_step record HIP events around each
                                 of its kernels (pxa_pds_kernel_ms) */
#define PXA_TUNE_PDS_MARCH 7 /* A/B of pxa_pds_step_la's kernel D: bit 0 lets a thread own two positions
                                (default one); bit 1 a persistent grid of the resident capacity (default one
                                workgroup per unit); bit 2 a soft progress coupling of row-neighbour workgroups
                                (fp32, radius 6: each waits, boundedly, while a started neighbour lags more than
                                2 + (value >> 3) planes); bit 8 the march without its plane prefetch (the default
                                issues every load of plane q + 1 before plane q is computed), bit 9 two planes
                                ahead; same bits */
#define PXA_TUNE_FFT_KERNEL 8 /* A/B of the in-LDS FFT (pxa_fft, lines that fit one workgroup): 0 in-place register-staged
                                 stages on padded lines with a twiddle table, 1 the ping-pong Stockham kernel of rounds
                                 1-3 (results equal up to rounding); bits 256 / 512 force 512- / 1024-thread
                                 workgroups of the in-place kernel, bit 1024 turns off its buffer-load fast path
                                 (same bits) */
#define PXA_TUNE_GRAD_KERNEL 9 /* A/B of pxa_gradient2 / pxa_gradient2_adjoint: 0 the axis-0 march (each input plane
                                  loaded once, XCD-banded in-plane blocks), 1 the row kernel of rounds 1-3 (same
                                  bits) */
#define PXA_TUNE_STENCIL_ND 10 /* A/B of the stencil kernels: bit 0 makes pxa_stencil_nd_box use the generic
                                   one-thread-per-output kernel instead of the LDS-tiled one, bit 1 makes the
                                   separable-axis passes (pxa_stencil_axis / _sep) use the scalar kernel instead of
                                   the vector / LDS-tiled ones, bit 2 turns off the LDS-tiled off-last-axis pass
                                   (same sums either way) */
#define PXA_TUNE_DUAL_ROWS 11 /* A/B of the PDS dual-update kernel C (pxa_tv_dual_update, the three-launch step): rows of w
                                * per thread, 0 the one-row kernel (the next plane's loads issued one plane early), 1 the
                                * one-row kernel without that prefetch, 2 or 4 the row-blocked kernel (a thread's row + 1
                                * neighbours are its own rows), 8 the plane-block kernel (3-D fp32 16-B vectors: an 8 x 128
                                * block of each plane staged in LDS with its halo row / column; 9: the same with z loaded one plane ahead).  Same
                                * bits. */
#define PXA_TUNE_PGD_PIPE 12 /* A/B of the fused PGD step: 1 the pipelined kernel (two resident workgroups per CU, each
                               * walking its XCD's tiles, the next tile's x / x_prev window fetched by LDS-DMA into a
                               * staging area during the current tile; fp32, 16-B aligned rows, R <= 7).  Same bits;
                               * measured slower (profiles/r06n_pgd_pipe_ab.txt). */
#define PXA_TUNE_COUNT 13

/* Row reductions (pxa_row_reduce). */
#define PXA_RED_SUMSQ 0  /* sum x^2            : SquaredL2Norm.apply, norm(ord=2)^2   (norm.py:91-94) */
#define PXA_RED_DIFFSQ 1 /* sum (x-y)^2        : RelError numerator (opt/stop.py:365-371) */
#define PXA_RED_DOT 2    /* sum x*y            : CG alpha denominator (opt/solver/cg.py:130) */
#define PXA_RED_ABS 3    /* sum |x|            : L1Norm.apply (norm.py:42-45) */
#define PXA_RED_MAXABS 4 /* max |x|            : LInfinityNorm / norm(ord=inf) */
#define PXA_RED_SUM 5    /* sum x              : Sum / QuadraticFunc.apply (operator.py:1255-1262) */
#define PXA_RED_NEGCNT 6 /* count(x < 0)       : PositiveOrthant.apply (func/indicator.py:198-202) */
#define PXA_RED_MIN 7    /* min x (NaN-propagating, numpy.min) : Memorize.info (opt/stop.py:181-196) */
#define PXA_RED_MAX 8    /* max x (NaN-propagating, numpy.max) : Memorize.info */

/* ---------------------------------------------------------------------------------------------
 * Library information
 * ------------------------------------------------------------------------------------------- */
const char* pxa_version(void);
const char* pxa_error_string(int code);
/* Number of exported compute entry points (for the loader's self-check). */
int pxa_abi_version(void);

/* Process-wide kernel-selection knob `key` (PXA_TUNE_*): sets it to `value` when value >= 0 and
 * returns the previous value (PXA_ERR_ARG for an unknown key).  Defaults (0) pick the fastest
 * kernel; the other values exist for A/B measurements and the parity tests between variants. */
int pxa_tuning(int key, int value);

/* ---------------------------------------------------------------------------------------------
 * Element-wise kernels: the arithmetic glue of the operator algebra
 * (abc/arithmetic.py ScaleRule :167-218, ArgShiftRule :580-652, AddRule :843-943) and the solver
 * updates (opt/solver/pgd.py:173-191, opt/solver/pds.py:429-442, :747-761, :1631-1638).
 * `out` may alias any input.
 * ------------------------------------------------------------------------------------------- */

/* out = a*x + b*y      (y may be NULL: out = a*x). */
int pxa_axpby(int dtype, int64_t n, double a, const void* x, double b, const void* y, void* out, void* stream);

/* out[i] = a*x[i] + b*y[i % ny]: y broadcast over the leading stack dims (ArgShiftRule.apply/prox/grad,
 * arithmetic.py:580-652; AddRule range broadcasting :843-849). */
int pxa_axpby_bcast(int dtype, int64_t n, double a, const void* x, double b, const void* y, int64_t ny, void* out,
                    void* stream);
/* out[r, i] = y[r, i] + s * c[r] * x[r, i] over a (rows, n) stack, c a device vector of `rows` scalars
 * (CG.m_step on stacked right-hand sides, opt/solver/cg.py:125-153: per-row alpha / beta). */
int pxa_axpy_rows(int dtype, int64_t rows, int64_t n, const void* c, double s, const void* x, const void* y, void* out,
                  void* stream);
/* out[r] = (dtype)(num[r] / den[r]) for float64 device vectors num, den of `rows` entries: the CG step
 * coefficients alpha / beta (opt/solver/cg.py:125-153) formed on the device, so the step needs no host
 * round trip for <p, A p>. */
int pxa_row_ratio(int dtype, int64_t rows, const double* num, const double* den, void* out, void* stream);

/* out = a*x + b*y + c*z. */
int pxa_lincomb3(int dtype, int64_t n, double a, const void* x, double b, const void* y, double c, const void* z,
                 void* out, void* stream);

 /* out = (x - y) * a + x   (PGD momentum step y_k, opt/solver/pgd.py:179-181). */
int pxa_extrapolate(int dtype, int64_t n, double a, const void* x, const void* y, void* out, void* stream);

/* out = x / d          (SquaredL2Norm.prox: y /= 2*tau+1, norm.py:100-104; moreau grad x /= mu). */
int pxa_div(int dtype, int64_t n, const void* x, double d, void* out, void* stream);

/* out = x + s           with s a broadcast scalar (ArgShiftRule with scalar shift, arithmetic.py:580-584). */
int pxa_add_scalar(int dtype, int64_t n, const void* x, double s, void* out, void* stream);

/* out[i] = v. */
int pxa_fill(int dtype, int64_t n, double v, void* out, void* stream);

/* out = x * y (element-wise product; QuadraticFunc.apply, operator.py:1255). */
int pxa_mul(int dtype, int64_t n, const void* x, const void* y, void* out, void* stream);

/* out = clip(x, lo, hi); has_hi=0 means no upper bound.  PositiveOrthant.prox (func/indicator.py:204-206). */
int pxa_clip(int dtype, int64_t n, const void* x, double lo, double hi, int has_hi, void* out, void* stream);

/* L1Norm.prox (operator/func/norm.py:47-52): out = fmax(0, |x| - tau) * sign(x). */
int pxa_prox_l1(int dtype, int64_t n, const void* x, double tau, void* out, void* stream);

/* ADMM outer update for h = lam ||.||_1 and K = Id (opt/solver/pds.py:1606-1620) fused with the next
 * x-update's right-hand side (QuadraticFunc.prox, operator.py:1257-1291), element-wise in one pass with the
 * rounding of the separate map calls:  zt = z + x - u;  u' = prox_l1(x + zt, thr);
 * z' = zt + (rho-1) x - (rho-1) u';  b = (u' - z') / tau - cgrad.  `out` holds 6 x n elements:
 * u', z', b, b, b, 0 (the CG's b, r0, p0 and x0 = 0).  Replaces seven pxa_lincomb3 / pxa_axpby /
 * pxa_prox_l1 / pxa_div launches and the CG set-up's fill and two copies. */
int pxa_admm_l1_update(int dtype, int64_t n, const void* x, const void* z, const void* u, const void* cgrad,
                       double rho_m1, double thr, double tau, void* out, void* stream);

/* L21Norm.prox (norm.py:352-364) with x viewed as (outer, group, inner) and the l2 norm taken over
 * `group` at each (outer, inner):  out = x * (1 - tau / fmax(||x||_2, tau)). */
int pxa_prox_l21(int dtype, int64_t outer, int64_t group, int64_t inner, const void* x, double tau, void* out,
                 void* stream);

/* ProxFunc.fenchel_prox of lam*L1Norm (operator.py:905-944 Moreau form, arithmetic.py:182-183):
 *   out = x - sigma * prox_{lam*|.|_1 / sigma}(x / sigma). */
int pxa_fenchel_prox_l1(int dtype, int64_t n, const void* x, double sigma, double lam, void* out, void* stream);

/* ProxFunc.fenchel_prox of lam*L21Norm, same (outer, group, inner) view as pxa_prox_l21. */
int pxa_fenchel_prox_l21(int dtype, int64_t outer, int64_t group, int64_t inner, const void* x, double sigma,
                         double lam, void* out, void* stream);

/* Gradient of scale * moreau_envelope(mu) of L1 / L21 (operator.py:1053-1058, arithmetic.py:209-213):
 *   out = scale * (x - prox_{mu f}(x)) / mu. */
int pxa_moreau_grad_l1(int dtype, int64_t n, const void* x, double mu, double scale, void* out, void* stream);
int pxa_moreau_grad_l21(int dtype, int64_t outer, int64_t group, int64_t inner, const void* x, double mu,
                        double scale, void* out, void* stream);

/* Per-(outer, inner) l2 norm over `group` (L21Norm.apply inner part, norm.py:338-350), written to
 * `out` (outer*inner elements, dtype). */
int pxa_group_norm(int dtype, int64_t outer, int64_t group, int64_t inner, const void* x, void* out, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Row reductions (opt/stop.py RelError/AbsError :353-382, :250-266; math/linalg.py norm :14-22;
 * opt/solver/cg.py:125-153).  x (and y) are (rows, n); out is a DEVICE array of `rows` doubles.
 * Accumulation is in double, in a fixed order (deterministic run to run).
 * `work` must hold pxa_row_reduce_workspace_bytes(rows, n) bytes of device memory.
 * ------------------------------------------------------------------------------------------- */
size_t pxa_row_reduce_workspace_bytes(int64_t rows, int64_t n);
int pxa_row_reduce(int dtype, int op, int64_t rows, int64_t n, const void* x, const void* y, double* out, void* work,
                   void* stream);

/* General Ln statistic of AbsError / RelError with any norm >= 0 (opt/stop.py:222-297, 300-396:
 * xp.linalg.norm(ord=p)): out[r] = sum |x - y|^p over row r (p > 0; y may be NULL), or the count of
 * non-zero entries of x - y (p == 0, NumPy's ord=0).  Same workspace as pxa_row_reduce. */
int pxa_row_reduce_pow(int dtype, int64_t rows, int64_t n, double p, const void* x, const void* y, double* out,
                       void* work, void* stream);

/* CG iteration tail after A p (opt/solver/cg.py:125-153), for `rows` stacked problems of n entries, in
 * three launches: alpha = (T)(rr / <p, A p>), x += alpha p, r -= alpha A p, rr' = ||r||^2,
 * beta = (T)(rr' / rr), p = r + beta p.  rr: this step's ||r||^2 per row (device double); rr_out (device,
 * != rr) and rr_host (pinned / device-mapped host memory, may be NULL) receive rr'; with `flags` (rows words
 * of pxa_host_alloc memory, rr_host then in that memory too) flag[row] is set to `seq` once rr_host[row] is
 * visible to the host, so the stop check polls it instead of waiting for a stream event.  All sums in double
 * with a fixed partition and order.  `work`: pxa_cg_update_workspace_bytes(rows) bytes. */
size_t pxa_cg_update_workspace_bytes(int64_t rows);
int pxa_cg_update(int dtype, int64_t rows, int64_t n, void* x, void* r, void* p, const void* ap, const double* rr,
                  double* rr_out, double* rr_host, uint32_t* flags, uint32_t seq, void* work, void* stream);

/* pxa_cg_update without its first launch: work[0 .. rows * 64) already holds the <p, A p> partials, written
 * together with A p by pxa_dense_normal_pdot (same partition and bits as pxa_cg_update's own). */
int pxa_cg_update_tail(int dtype, int64_t rows, int64_t n, void* x, void* r, void* p, const void* ap, const double* rr,
                       double* rr_out, double* rr_host, uint32_t* flags, uint32_t seq, void* work, void* stream);

/* The CG tail's first half alone (pxa_cg_update_tail without the p update): x += alpha p, r -= alpha A p, and the
 * ||r'||^2 partials at work + rows * 64 doubles, for a following pxa_dense_normal_pdot_pfold that forms p' = r' +
 * beta p inside its operator pass (cg.py:125-153; same bits as pxa_cg_update_tail + pxa_dense_normal_pdot). */
int pxa_cg_update_xr(int dtype, int64_t rows, int64_t n, void* x, void* r, const void* p, const void* ap, const double* rr,
                     void* work, void* stream);

/* RelError statistics from the fused PGD step's per-tile partials (pxa_pgd_tv2d_step[_y] with
 * `partials`): out[0 * rows + r] = sum (x_new - x)^2 and out[1 * rows + r] = sum x^2 over the per_row
 * consecutive tiles of stack row r, fixed summation order.  At stop_rate 1 the criterion's stored x_prev
 * IS the step's x, so this replaces the separate pass over x and x_prev (stop.py:353-382); at stop_rate > 1
 * the step's partials were taken against the previous check's iterate (x_ref).  `out` may be device or
 * pinned (device-mapped) host memory.  With `flags` != NULL (2 * rows words of pxa_host_alloc memory, like
 * `out`), statistic q's flag is set to `seq` once out[q] is visible to the host (system-scope release): a
 * stop check then polls the flags instead of waiting for a stream event. */
int pxa_tile_partials_fold(int64_t rows, int64_t per_row, const double* partials, double* out, uint32_t* flags,
                           uint32_t seq, void* stream);
/* Host memory the device reads and writes coherently during a kernel (hipHostMalloc, coherent + mapped):
 * the stop checks' statistics and completion flags.  The same pointer is valid on the device. */
int pxa_host_alloc(size_t bytes, void** ptr);
int pxa_host_free(void* ptr);
/* RelError.stop in one pass (opt/stop.py:353-382, norm=2): out[0:rows] = sum (x - x_prev)^2 and
 * out[rows:2 rows] = sum x_prev^2 per row (same bits as pxa_row_reduce DIFFSQ / SUMSQ), and, when
 * x_copy is not NULL, x_copy = x (the `x.copy()` the criterion keeps, stop.py:381).  `out` may be
 * device memory or device-mapped pinned host memory (RelError.stop_async reads it after an event).
 * `work` must hold pxa_relerr_stats_workspace_bytes(rows, n) bytes of device memory. */
size_t pxa_relerr_stats_workspace_bytes(int64_t rows, int64_t n);
int pxa_relerr_stats(int dtype, int64_t rows, int64_t n, const void* x, const void* x_prev, void* x_copy, double* out,
                     void* work, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Stencils (operator/linop/stencil/stencil.py:356-627, _stencil.py:232-476; pad.py; select.py).
 *
 * All stencil entry points act on `stack` independent arrays of spatial shape `shape[0..ndim)`;
 * array s starts at x + s*x_stack_stride (elements) and y + s*y_stack_stride.
 * Output: y = corr(x) + beta*y  (beta = 0 overwrites; beta = 1 accumulates, as vstack adjoints do,
 * blocks.py:838-860).
 * Taps are given in the reference's code-generation order (itertools.product over the kernel,
 * _stencil.py:284-305) after its constant folding: taps with isclose(k, 0) removed, taps with
 * isclose(k, 1) replaced by exactly 1.
 *
 * zero_partial = 0 : zero-padding semantics, out[i] = sum_q k_q x[i + off_q] with x = 0 outside;
 *                    this is Trim o S o Pad for mode="constant" (stencil.py:441-450) in one pass.
 * zero_partial = 1 : numba @stencil semantics on an already-padded array: out[i] = 0 wherever one
 *                    offset leaves the array (_stencil.py:238-244, :337-383).
 * ------------------------------------------------------------------------------------------- */

/* One separable-axis pass: taps along `axis` only; offsets[q] = q - center (relative index). */
int pxa_stencil_axis(int dtype, int64_t stack, int ndim, const int64_t* shape, int axis, int ntaps,
                     const int32_t* offsets, const double* coefs, int zero_partial, const void* x,
                     int64_t x_stack_stride, void* y, int64_t y_stack_stride, double beta, void* stream);

/* Fused separable filter over every axis with a non-trivial kernel (axis order 0..ndim-1, as
 * Stencil._stencil_chain applies them).  Per axis a: ntaps[a] taps at offsets/coefs
 * [a*PXA_MAX_TAPS ..).  ntaps[a] == 0 marks an identity axis.  Constant mode (zero_partial=0) only.
 * `work` must hold pxa_stencil_sep_workspace_bytes(...) bytes (intermediate field) or be NULL when
 * at most one axis is non-trivial. */
size_t pxa_stencil_sep_workspace_bytes(int dtype, int64_t stack, int ndim, const int64_t* shape,
                                       const int* ntaps);
int pxa_stencil_sep(int dtype, int64_t stack, int ndim, const int64_t* shape, const int* ntaps,
                    const int32_t* offsets, const double* coefs, const void* x, int64_t x_stack_stride, void* y,
                    int64_t y_stack_stride, double beta, void* work, void* stream);

/* Non-separable N-D stencil.  Taps live in DEVICE memory: offsets_dev (ntaps x ndim int32, relative
 * offsets) and coefs_dev (ntaps, dtype). */
int pxa_stencil_nd(int dtype, int64_t stack, int ndim, const int64_t* shape, int ntaps, const int32_t* offsets_dev,
                   const void* coefs_dev, int zero_partial, const void* x, int64_t x_stack_stride, void* y,
                   int64_t y_stack_stride, double beta, void* stream);

/* pxa_stencil_nd with the tap offsets' range per axis given on the host (off_lo[a] <= every offset along axis a
 * <= off_hi[a]): 2-D / 3-D stencils whose reach fits run LDS-tiled (the input box staged once per 16 x 64 output
 * tile, four outputs per thread), same sums as pxa_stencil_nd (taps in list order, one fma each); others fall
 * back to it.  Replaces the same reference call as pxa_stencil_nd (stencil.py:441-461, _stencil.py codegen). */
int pxa_stencil_nd_box(int dtype, int64_t stack, int ndim, const int64_t* shape, int ntaps, const int32_t* offsets_dev,
                       const void* coefs_dev, const int32_t* off_lo, const int32_t* off_hi, int zero_partial,
                       const void* x, int64_t x_stack_stride, void* y, int64_t y_stack_stride, double beta,
                       void* stream);

/* Pad.apply (pad.py:235-306): y (stack, shape + lo + hi) from x (stack, shape); modes per axis. */
int pxa_pad(int dtype, int64_t stack, int ndim, const int64_t* shape, const int64_t* pad_lo, const int64_t* pad_hi,
            const int* modes, const void* x, void* y, void* stream);

/* Pad.adjoint (pad.py:307-372): y (stack, shape) from x (stack, padded shape).  `work` holds one
 * padded-size scratch field (stack * prod(shape + lo + hi) elements). */
int pxa_pad_adjoint(int dtype, int64_t stack, int ndim, const int64_t* shape, const int64_t* pad_lo,
                    const int64_t* pad_hi, const int* modes, const void* x, void* y, void* work, void* stream);

/* Trim.apply / SubSample (select.py:120-142, :205-251) when embed=0: y = x[lo : n - hi] per axis.
 * Trim.adjoint (select.py:144-167) when embed=1: y (padded) = 0 except the core, which receives x. */
int pxa_trim(int dtype, int64_t stack, int ndim, const int64_t* shape, const int64_t* lo, const int64_t* hi,
             int embed, const void* x, void* y, void* stream);

/* SubSample.apply (select.py:119-141) for any index specifier: y (rows, m) = x[:, idx] with x
 * (rows, n) and idx_dev (m,) int64 flat positions in [0, n) (the host ravels numpy's indexing). */
int pxa_gather_cols(int dtype, int64_t rows, int64_t n, const void* x, int64_t m, const int64_t* idx_dev, void* y,
                    void* stream);

/* SubSample.adjoint (select.py:143-167): out (rows, n) = 0, then out[:, idx] = y (rows, m).  idx
 * entries must be unique (the host keeps numpy's last-write-wins entry of a repeated position). */
int pxa_scatter_cols(int dtype, int64_t rows, int64_t m, const void* y, int64_t n, const int64_t* idx_dev, void* out,
                     void* stream);

/* ---------------------------------------------------------------------------------------------
 * Gradient (operator/linop/diff.py Gradient :1113-1265 = vstack of 2-tap finite-difference
 * Stencils, blocks.py:660-679, :838-860) in ONE pass over x (apply) or z (adjoint),
 * constant (zero) boundary.  Direction d (0 <= d < ndir) differentiates spatial axis dirs[d] with
 * taps (off0[d], coef0[d]) and (off1[d], coef1[d]) in code-generation order.
 * apply  : g (stack, ndir, N) direction-major, g[s,d,i] = c0 x[i+o0 e] + c1 x[i+o1 e]
 * adjoint: x (stack, N), x[s,i] = sum_d ( c1' z_d[i-o1 e] + c0' z_d[i-o0 e] )   (flipped order)
 * ------------------------------------------------------------------------------------------- */
int pxa_gradient2(int dtype, int64_t stack, int ndim, const int64_t* shape, int ndir, const int* dirs,
                  const int* off0, const double* coef0, const int* off1, const double* coef1, const void* x, void* g,
                  void* stream);
int pxa_gradient2_adjoint(int dtype, int64_t stack, int ndim, const int64_t* shape, int ndir, const int* dirs,
                          const int* off0, const double* coef0, const int* off1, const double* coef1, const void* z,
                          void* x, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Dense LinOp (operator/linop/base.py _ExplicitLinOp._matmat :407-419, apply/adjoint :421-427):
 *   trans = 0 : Y (B x M) = X (B x N) A^T      (A.dot(x) per stacked row)
 *   trans = 1 : Y (B x N) = X (B x M) A        (A^T.dot(z) per stacked row)
 * A is (M x N) row-major.  `work` must hold pxa_dense_workspace_bytes(...) bytes.
 * fp32 with B >= 2 stacked right-hand sides runs on the matrix cores (v_mfma_f32_32x32x2_f32, A
 * streamed once, split-K partials summed in a fixed order); smaller B and fp64 use the GEMV kernels.
 * ------------------------------------------------------------------------------------------- */
size_t pxa_dense_workspace_bytes(int dtype, int trans, int64_t M, int64_t N, int64_t B);
int pxa_dense_matmat(int dtype, int trans, int64_t M, int64_t N, int64_t B, const void* A, const void* X, void* Y,
                     void* work, void* stream);

/* Normal operator of a dense LinOp in ONE pass over A: Y = s * A^T (A X) + d * X, one right-hand side
 * (B = 1), fp32, N % 4 == 0, N <= 65536.  Replaces the apply of the CG operator Q + I / tau that
 * QuadraticFunc.prox builds for ADMM's x-update (abc/operator.py:1273-1291 QuadraticFunc.prox,
 * opt/solver/pds.py:1645-1653, Q = K^T c K from abc/arithmetic.py ChainRule._quad_spec), i.e. the
 * K.apply -> K.adjoint -> AddRule chain of opt/solver/cg.py:130 (`Ap = self._A.apply(p)`).
 * Each row is split in four column parts, one per workgroup of a group; the part-dots are exchanged
 * inside the launch (a member that does not answer in time is replaced by computing its part here, with
 * the same bits), t = ((d0 + d1) + d2) + d3 in every member.  Workgroup partials of A^T (A X) (fixed
 * partition) are summed in a fixed order: deterministic.  The workspace also holds the exchange words.
 * pxa_dense_normal_workspace_bytes() returns 0 for unsupported cases, where pxa_dense_normal returns
 * PXA_ERR_UNSUPPORTED (the caller then composes pxa_dense_matmat calls). */
size_t pxa_dense_normal_workspace_bytes(int dtype, int64_t M, int64_t N, int64_t B);
int pxa_dense_normal(int dtype, int64_t M, int64_t N, int64_t B, const void* A, const void* X, double s, double d,
                     void* Y, void* work, void* stream);

/* pxa_dense_normal (B = 1) that also writes the <X, Y> partials of the CG iterating on this operator into
 * pdot (pxa_cg_update's partition: min(64, ceil(N / 256)) doubles), folded into the partial-sum reduction
 * launch (one launch instead of two reductions and the CG's dot); then pxa_cg_update_tail with pdot as the
 * head of its workspace.  Same bits as pxa_dense_normal followed by pxa_cg_update. */
int pxa_dense_normal_pdot(int dtype, int64_t M, int64_t N, const void* A, const void* X, double s, double d, void* Y,
                          void* work, double* pdot, void* stream);

/* pxa_dense_normal_pdot with the CG's previous p update folded into the pass (one row, fp32, the split-row kernel):
 * p' = r' + beta p with beta = ||r'||^2 / ||r||^2, ||r'||^2 folded from pxa_cg_update_xr's partials `part_rr`; p' is
 * written to P_new (!= P) and used as the operand; ||r'||^2 goes to rr_out (device) and, with rr_host / flags, to
 * coherent host memory with publication `seq`, as pxa_cg_update does.  Same bits as pxa_cg_update(_tail) followed
 * by pxa_dense_normal_pdot on p'.  PXA_ERR_UNSUPPORTED under PXA_TUNE_NORMAL_KERNEL = 1. */
int pxa_dense_normal_pdot_pfold(int dtype, int64_t M, int64_t N, const void* A, const void* R, const void* P, void* P_new,
                                const double* rr, const double* part_rr, double* rr_out, double* rr_host, uint32_t* flags,
                                uint32_t seq, double s, double d, void* Y, void* work, double* pdot, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Array primitives: the data movement of the operator algebra and the NumPy-named functions of the
 * backend's array module (SURVEY.md §8(b) `xp` list), so that no array arithmetic of the product path
 * runs outside this library.
 * ------------------------------------------------------------------------------------------- */

/* dst[r*ldd + i] = src[r*lds + i] (accumulate 0), dst + src (1), or 0 + src (2: the first term of
 * a Python sum(), which maps -0.0 to +0.0 exactly as the reference's row sums), r < rows, i < n.
 * Block operators (operator/blocks.py:660-679, 838-860: slicing arr[..., off:off+dim], the row sums
 * of hstack.apply / vstack.adjoint, concatenate), lds = 0 broadcasts one row (CG x0 broadcast,
 * opt/solver/cg.py:96-110), diagonal extraction (lds = n + 1).  src_col_stride is 1, or 0 to repeat
 * src[r*lds] along the row (Sum.adjoint, operator/linop/reduce.py). */
int pxa_copy2d(int dtype, int64_t rows, int64_t n, const void* src, int64_t lds, int64_t src_col_stride, void* dst,
               int64_t ldd, int accumulate, void* stream);

/* out = f(x): op 0 sqrt, 1 sign (numpy.sign), 2 fabs, 3 negative, 4 square, 5 reciprocal,
 * 6 (x > 0 ? +inf : 0) (indicator value from a violation count, func/indicator.py:198-202). */
#define PXA_UN_SQRT 0
#define PXA_UN_SIGN 1
#define PXA_UN_ABS 2
#define PXA_UN_NEG 3
#define PXA_UN_SQUARE 4
#define PXA_UN_RECIP 5
#define PXA_UN_POSINF 6
int pxa_unary(int dtype, int op, int64_t n, const void* x, void* out, void* stream);

/* out = f(x, y) with x / y arrays of n elements or NULL for the broadcast scalars xs / ys:
 * op 0 fmax, 1 fmin (NaN-ignoring, numpy.fmax/fmin), 2 add, 3 subtract, 4 multiply, 5 divide,
 * 6 maximum, 7 minimum (NaN-propagating), 8 power. */
#define PXA_BIN_FMAX 0
#define PXA_BIN_FMIN 1
#define PXA_BIN_ADD 2
#define PXA_BIN_SUB 3
#define PXA_BIN_MUL 4
#define PXA_BIN_DIV 5
#define PXA_BIN_MAXIMUM 6
#define PXA_BIN_MINIMUM 7
#define PXA_BIN_POW 8
int pxa_binary(int dtype, int op, int64_t n, const void* x, double xs, const void* y, double ys, void* out,
               void* stream);

/* numpy.where(cond, x, y): cond is n bytes (bool), x / y arrays or NULL for scalars xs / ys. */
int pxa_where(int dtype, int64_t n, const void* cond, const void* x, double xs, const void* y, double ys, void* out,
              void* stream);

/* out[i] = isnan(x[i]) as bytes; pxa_bool_reduce: out[0] = any (mode 0) / all (mode 1) of n bytes. */
int pxa_isnan(int dtype, int64_t n, const void* x, void* out, void* stream);
int pxa_bool_reduce(int64_t n, int mode, const void* x, void* out, void* stream);

/* out = (dtype_out) x: float64 statistics to the array dtype and back. */
int pxa_cast(int dtype_in, int dtype_out, int64_t n, const void* x, void* out, void* stream);

/* out[r*ld + off + r] = value, r < rows (identity columns of LinOp.asarray, operator.py:1593-1628). */
int pxa_set_diag(int dtype, int64_t rows, int64_t ld, int64_t off, double value, void* out, void* stream);

/* dst (cols x rows) = src (rows x cols)^T (LinOp.asarray / TransposeRule.asarray, arithmetic.py:1496). */
int pxa_transpose(int dtype, int64_t rows, int64_t cols, const void* src, void* dst, void* stream);

/* Directional contraction of a stacked derivative output: Sum o DiagonalOp o {Gradient, Hessian} of
 * DirectionalDerivative / DirectionalGradient / DirectionalLaplacian / DirectionalHessian
 * (operator/linop/diff.py:1938-2759).  x and y hold S stacked problems of N pixels:
 *   adjoint = 0: y[s][g][p] = sum_{j<J} w[g][j][p] * x[s][j % K][p]              x: (S, K, N) -> y: (S, G, N)
 *   adjoint = 1: y[s][k][p] = sum_{g<G} sum_{j<J, j%K==k} w[g][j][p] * x[s][g][p]  x: (S, G, N) -> y: (S, K, N)
 * w: (G, J, N) when wp = 1, or (G, J) applied at every pixel when wp = 0; J a multiple of K.  Products are
 * rounded, then added in (j, g) order (the reference's DiagonalOp then numpy.sum). */
int pxa_dir_contract(int dtype, int64_t S, int64_t G, int64_t J, int64_t K, int64_t N, const void* w, int64_t wp,
                     const void* x, void* y, int adjoint, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Fused solver steps (the whole m_step of a recognised problem in one launch).
 *
 * PGD on  F(x) = 1/2||H x - y||^2 + lam * env_mu(L21 o Grad)(x),  G = PositiveOrthant | l1w*L1 | 0
 * (opt/solver/pgd.py:173-191 with the arithmetic of AddRule/ChainRule/ScaleRule/ArgShiftRule):
 *   yk   = x + a (x - x_prev)
 *   grad = (H^T H) yk - H^T y + Grad^T( lam * (v - prox_{mu L21}(v)) / mu ),  v = Grad yk
 *   x_new = prox_{tau G}( yk - tau * grad )
 * H is a separable zero-boundary (mode="constant") correlation over 2 spatial axes (taps0 on axis
 * 0, taps1 on axis 1, offsets/coefs in code-generation order); Grad the forward-difference
 * Gradient (diff.py default scheme) with spacing h0, h1.  H^T H is applied as the exact banded
 * normal operator (interior: autocorrelation of the taps; boundary rows: the truncated sums), which
 * equals the reference's H^T (H yk - y) up to fp rounding; `hty` = H^T y is iteration-invariant and
 * computed once by the caller (e.g. pxa_stencil_sep with the flipped taps).  `stack` independent
 * images, each (n0, n1), contiguous; image s uses data image (s % y_images) of hty (1 = one y shared
 * by a stack of initial points, stack = batch-as-axis images with their own data).  x_new must not
 * alias x or x_prev.  If `partials` is not NULL, each (tile, wavefront) slot writes (sum (x_new-x)^2,
 * sum x^2) for RelError into partials[2*slot..] (double); with x_ref != NULL the statistics are taken against
 * x_ref instead of x, i.e. (sum (x_new-x_ref)^2, sum x_ref^2): RelError at stop_rate > 1 compares with the
 * iterate of the previous check (opt/stop.py:353-382) — pxa_pgd_tv2d_partials_count() gives the
 * number of slots (tiles x 4; the slots of one image are contiguous).  prox codes: 0 none, 1 positive
 * orthant, 2 l1 with weight prox_w.  pxa_pgd_tv2d_last_kernel() is the kernel the calling thread launched
 * last: 1 the tile kernel, 2 the strip kernel (PXA_TUNE_PGD_KERNEL), 3 the pipelined kernel (PXA_TUNE_PGD_PIPE), 0 none
 * yet.
 * ------------------------------------------------------------------------------------------- */
int pxa_pgd_tv2d_partials_count(int64_t stack, int64_t n0, int64_t n1);
/* Prepared form of pxa_pgd_tv2d_step for a solver's iterations (replaces the same call per PGD.m_step,
 * opt/solver/pgd.py:173-191, and the RelError fold of its stop checks, opt/stop.py:353-382):
 * pxa_pgd_tv2d_plan() folds the taps and builds the iteration-invariant parameters once (arguments as
 * pxa_pgd_tv2d_step's, prox_w excluded) into an opaque handle; pxa_pgd_tv2d_plan_step() runs one iteration
 * with the per-step a, tau, prox_w and arrays (as pxa_pgd_tv2d_step).  With rel_values != NULL (then partials
 * and rel_flags too) the workgroup that finishes last also folds the partials into rel_values[(2, rows)],
 * rows = stack / y_images, exactly as pxa_tile_partials_fold does (same bits), and sets rel_flags[q] = seq
 * (2 * rows words; pxa_host_alloc memory) after its value, system-wide: a stop check then needs no fold
 * launch.  A plan holds a device counter: launches of one plan must not run concurrently (one stream).
 * pxa_pgd_tv2d_plan_free() releases it. */
int pxa_pgd_tv2d_plan(int dtype, int64_t stack, int64_t y_images, int64_t n0, int64_t n1, int nt0, const int32_t* off0,
                      const double* coef0, int nt1, const int32_t* off1, const double* coef1, double h0, double h1,
                      double lam, double mu, int prox, void** plan);
int pxa_pgd_tv2d_plan_step(void* plan, double a, double tau, double prox_w, const void* x, const void* x_prev,
                           const void* hty, void* x_new, double* partials, const void* x_ref, double* rel_values,
                           uint32_t* rel_flags, uint32_t seq, void* stream);
/* As pxa_pgd_tv2d_plan_step with rel_values / rel_flags required, the fold done by a pxa_tile_partials_fold
 * launch enqueued right behind the step (same bits as the in-kernel fold, flags seen ~3 us after the step
 * instead of the last workgroup's late write-back): the stop_rate-1 path, one C call per iteration. */
int pxa_pgd_tv2d_plan_step_fold(void* plan, double a, double tau, double prox_w, const void* x, const void* x_prev,
                                const void* hty, void* x_new, double* partials, const void* x_ref, double* rel_values,
                                uint32_t* rel_flags, uint32_t seq, void* stream);
/* pxa_pgd_tv2d_plan_step with the RelError statistics of the PREVIOUS iterate pair (the stop check that precedes
 * this launch at stop_rate 1, opt/stop.py:353-382): the launch's partials are (sum (x - x_prev)^2, sum x_prev^2) per
 * (tile, wave), taken from the window loads it makes anyway (no load of x beyond them), and a fold launch behind it
 * publishes them as pxa_tile_partials_fold does into rel_values / rel_flags (seq).  Used by the solver's lagged
 * stop checks (pyxu_amd/abc/solver.py), which resolve a check after the next step has run. */
int pxa_pgd_tv2d_plan_step_wfold(void* plan, double a, double tau, double prox_w, const void* x, const void* x_prev,
                                 const void* hty, void* x_new, double* partials, double* rel_values, uint32_t* rel_flags,
                                 uint32_t seq, void* stream);
/* pxa_pgd_tv2d_plan_step with window partials (as pxa_pgd_tv2d_plan_step_wfold: the statistics of the (x, x_prev)
 * pair it reads, into `partials`), and with prev_partials != NULL one extra workgroup that folds prev_partials -- the
 * partials of the previous such launch, complete by now -- exactly as pxa_tile_partials_fold does (same bits) into
 * rel_values[(2, rows)] and then sets rel_flags[q] = seq: a stop check's statistics are published by the launch
 * after the one that computed them, with no fold launch of their own (the solver's lagged stop checks resolve a
 * check two launches later).  partials and prev_partials must differ (two buffers, alternately). */
int pxa_pgd_tv2d_plan_step_wpub(void* plan, double a, double tau, double prox_w, const void* x, const void* x_prev,
                                const void* hty, void* x_new, double* partials, const double* prev_partials,
                                double* rel_values, uint32_t* rel_flags, uint32_t seq, void* stream);
int pxa_pgd_tv2d_plan_free(void* plan);
int pxa_pgd_tv2d_last_kernel(void);
/* Diagnostics: s_memtime stamps of the tile kernel's last launch under PXA_TUNE_PGD_DIAG bit 5
 * (workgroups 0, 1, grid/2, grid-1; waves 0..3; 8 phase points; n <= 128 words). */
int pxa_pgd_tile_trace(uint64_t* host_out, int n);
int pxa_pgd_tv2d_step(int dtype, int64_t stack, int64_t y_images, int64_t n0, int64_t n1, int nt0, const int32_t* off0,
                      const double* coef0, int nt1, const int32_t* off1, const double* coef1, double h0, double h1,
                      double lam, double mu, double a, double tau, int prox, double prox_w, const void* x,
                      const void* x_prev, const void* hty, void* x_new, double* partials, const void* x_ref,
                      void* stream);


/* ---------------------------------------------------------------------------------------------
 * FFT LinOp (operator/linop/fft/fft.py:257-379).  `stack` arrays of complex values (interleaved
 * re/im, i.e. the reference's view_as_real layout, (stack, *shape, 2)), transformed over the
 * `naxes` distinct `axes` of `shape`:
 *   inverse = 0: apply   = fftn(x, axes, norm="backward")  (exp(-2 pi i jk/n), unnormalised)
 *   inverse = 1: adjoint = ifftn(x, axes, norm="forward")  (exp(+2 pi i jk/n), unnormalised)
 * `out` may alias `in`.  Lengths whose prime factors are in {2, 3, 5, 7} run a mixed-radix Stockham
 * FFT in LDS (n <= 10240 in fp32, 5120 in fp64); other lengths up to 2048 an exact DFT in LDS.  Every
 * other length (like the reference's scipy.fft) needs a workspace: longer smooth lengths run a
 * four-step split n = n1 n2, the rest Bluestein's chirp-z on a 2^k-point FFT.  pxa_fft (no workspace)
 * returns PXA_ERR_UNSUPPORTED for those; pxa_fft_ex takes `work` of pxa_fft_workspace_bytes(...)
 * bytes (0: none needed; (size_t)-1: unsupported arguments).
 * ------------------------------------------------------------------------------------------- */
int pxa_fft(int dtype, int ndim, const int64_t* shape, int naxes, const int* axes, int64_t stack, int inverse,
            const void* in, void* out, void* stream);
size_t pxa_fft_workspace_bytes(int dtype, int ndim, const int64_t* shape, int naxes, const int* axes, int64_t stack);
int pxa_fft_ex(int dtype, int ndim, const int64_t* shape, int naxes, const int* axes, int64_t stack, int inverse,
               const void* in, void* out, void* work, void* stream);
/* out[i] = a[i] * b[i % nb] over n complex elements (b conjugated if conj_b): the spectrum product of
 * the FFT path of large zero-boundary stencils (Stencil.apply/adjoint, stencil.py:441-461). */
int pxa_complex_mul(int dtype, int64_t n, int64_t nb, const void* a, const void* b, int conj_b, void* out,
                    void* stream);
/* z[i] = x[i] + 0j (FFT(real=True).apply input, fft.py:320-330); n complex elements. */
int pxa_real_to_complex(int dtype, int64_t n, const void* x, void* z, void* stream);
/* x[i] = Re z[i] (FFT(real=True).adjoint output, fft.py:370-379); n complex elements. */
int pxa_complex_real_part(int dtype, int64_t n, const void* z, void* x, void* stream);

/* Measurement hook: with pxa_tuning(PXA_TUNE_PDS_EVENTS, 1), pxa_pds_step / pxa_pds_step_la record HIP
 * events around their kernels (at most 64 steps).  This call waits for the last of them and writes into
 * ms_abc[3] the summed durations of kernels A (axis-0 march; the look-ahead step's priming march, 0 when
 * primed), B (in-plane G + update) and C (dual update; kernel D in the look-ahead step) over the
 * recorded steps, then (reset != 0) forgets them.  Returns the number of steps (>= 0) or an error. */
int pxa_pds_kernel_ms(double* ms_abc, int reset);
/* ---------------------------------------------------------------------------------------------
 * Fused primal-dual splitting iteration (replaces PD3O.m_step, opt/solver/pds.py:747-761, algo 0, and
 * CondatVu.m_step, pds.py:429-442, algo 1) for f = 1/2 ||S . - y||^2, K = Gradient over the D trailing
 * axes (forward differences, zero boundary), h = lam L1 (h_kind 0, anisotropic TV) or lam L21 over
 * the D directions (h_kind 1, isotropic TV), g given by `prox` (0 none, 1 positive orthant, 2 l1 with
 * weight prox_w).  Three launches: axis-0 march, in-plane tile, dual update (pds3d.hip).
 *   geom  = {stack, y_images, n0, n1, n2, D}: `stack` volumes of (n0, n1, n2) (n0 = 1, D = 2 for
 *           images); z is (stack, D, n0, n1, n2) direction-major, direction d on axis d + 3 - D.
 *   ntaps[3], offs[3][17], coefs[3][17]: the separable taps of S per axis (code-generation order;
 *           axis 0 = {[0], [1.0]} when it is not blurred).
 *   diff  = {c0[3], c1[3]}: forward-difference taps per AXIS, (K x)[i] = c0 x[i] + c1 x[i + e_a]
 *           (-1/h, 1/h); entries of non-differentiated axes are ignored.
 *   scal  = {tau, sigma, rho, lam, prox_w}.
 *   PD3O : reads u, z; writes x_out = prox_g(u - tau K^T z), u_out, z_out.  x is ignored.
 *   CV   : reads x, z; writes x_out, z_out (x_out must not alias x).  u / u_out are ignored.
 *   hty = S^T y (y_images volumes; volume s uses s % y_images), computed once by the caller.
 *   work_q: stack*n0*n1*n2 scratch (unused when axis 0 is not blurred), work_w: same size, required.
 *   u_out may alias u and z_out may alias z.  nseg: axis-0 segments of the march (<= 0: 1).
 * ------------------------------------------------------------------------------------------- */
int pxa_pds_step(int dtype, int algo, const int64_t* geom, const int32_t* ntaps, const int32_t* offs,
                 const double* coefs, const double* diff, const double* scal, int prox, int h_kind, const void* x,
                 const void* u, const void* z, const void* hty, void* x_out, void* u_out, void* z_out, void* work_q,
                 void* work_w, int nseg, void* stream);

/* The dual update of the PDS step on its own (kernel C of pxa_pds_step; SURVEY.md §8(d) "Gradient +
 * prox", K4): z_out = relax(fenchel_prox_{sigma h}(z + sigma K w)) with K = Gradient over the D trailing
 * axes (forward differences, zero boundary: diff.py:1113-1265), h = lam L1 (h_kind 0) or lam L21 over the
 * D directions (h_kind 1); fenchel_prox (abc/operator.py:905-944) evaluated as the projection onto the
 * dual-norm ball of radius lam that its Moreau form equals.  relax 0: PD3O's
 * (1 - rho) z + rho z_t (opt/solver/pds.py:760), 1: Condat-Vu's rho z_t + (1 - rho) z (pds.py:441).
 *   geom = {stack, n0, n1, n2, D}: w is (stack, n0, n1, n2); z and z_out are (stack, D, n0, n1, n2)
 *          direction-major, direction d on axis d + 3 - D (D = 2 requires n0 = 1: images).
 *   diff = {c0[3], c1[3]} as in pxa_pds_step.  z_out may alias z, not w. */
int pxa_tv_dual_update(int dtype, int relax, const int64_t* geom, const double* diff, double sigma, double lam,
                       double rho, int h_kind, const void* w, const void* z, void* z_out, void* stream);

/* Look-ahead form of pxa_pds_step (same problem class and arguments, pds_march.hpp): two launches per
 * iteration, kernel B and kernel D = the dual update of this iteration fused with the axis-0 march of
 * the next one, which is therefore already done when the next call starts (primed = 1).  A call with
 * primed = 0 first runs that march for the current state (one extra launch).
 *   PD3O : x is the current iterate x = prox_g(u - tau K^T z) (written here when primed = 0, else as the
 *          previous call's x_out left it); reads u, z; writes u_out, z_out and x_out = the NEXT iterate
 *          (the x the next call receives).  x_out != x.
 *   CV   : reads x, z; writes x_out, z_out (x_out != x).  u / u_out are ignored.
 *   work_kt (CV): K^T z of the current z (written when primed = 0), rewritten with K^T z_out.
 *   work_q: G0 of the current march variable (same priming rule), rewritten for the next iteration.
 *   z_out must not alias z.  u_out may alias u.  Returns as pxa_pds_step.
 * The caller keeps (x, work_q, work_kt) of one call for the next one; any change of the state in
 * between (a restart, a user-supplied z) requires primed = 0. */
int pxa_pds_step_la(int dtype, int algo, const int64_t* geom, const int32_t* ntaps, const int32_t* offs,
                    const double* coefs, const double* diff, const double* scal, int prox, int h_kind, int primed,
                    void* x, const void* u, const void* z, const void* hty, void* x_out, void* u_out, void* z_out,
                    void* work_q, void* work_kt, void* work_w, int nseg, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PYXU_AMD_H */
