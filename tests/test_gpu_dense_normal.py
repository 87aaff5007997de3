"""
GPU tests of the one-pass normal operator (pxa_dense_normal) and of its use inside CG / ADMM:
  * the kernel against a float64 NumPy restatement of s * A^T (A x) + d * x (north_star fp32 tolerance
    1e-5 norm-wise), for every register/LDS split of the row (N = 256 .. 65536, full and ragged last
    vector blocks, M smaller and larger than the 256-workgroup partition), and bit-identical run to run;
  * the row-split kernel (part-dots exchanged between four workgroups) against its no-exchange path bit for
    bit, and against the one-workgroup-per-row kernel;
  * the operator-tree matcher on the operator ADMM builds (reference abc/operator.py:1273-1291,
    abc/arithmetic.py:1255-1264), and on trees it must reject;
  * ADMM / CG trajectories through the fused operator against the unfused operator and the oracle.
"""
import numpy as np
import pytest

import oracle as orc
from conftest import rel_err

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs an MI355X", allow_module_level=True)

import pyxu_amd.abc as pxa  # noqa: E402
import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402
from pyxu_amd.opt.solver._normal import normal_form  # noqa: E402
from pyxu_amd.util import to_device, to_NUMPY  # noqa: E402


def _ref(A, x, s, d):
    A64, x64 = A.astype(np.float64), x.astype(np.float64)
    return s * (A64.T @ (A64 @ x64)) + d * x64


@pytest.mark.parametrize("M,N", [(7, 256), (300, 4096), (1000, 8192), (513, 12288), (64, 40000), (260, 65536),
                                 (2048, 65536)])
def test_dense_normal_vs_fp64(M, N):
    rng = np.random.default_rng(M + N)
    A = (rng.standard_normal((M, N)) / np.sqrt(M)).astype(np.float32)
    x = rng.standard_normal(N).astype(np.float32)
    Ad, xd = to_device(A), to_device(x)
    assert _dev.dense_normal_supported(Ad, xd)
    y1 = _dev.dense_normal(Ad, xd, 0.7, 1.3)
    y2 = _dev.dense_normal(Ad, xd, 0.7, 1.3)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)  # fixed partition and summation order
    assert rel_err(to_NUMPY(y1), _ref(A, x, 0.7, 1.3)) <= 1e-5


@pytest.mark.parametrize("M,N", [(1, 4), (3, 16), (8, 1000), (100, 4100), (257, 65532), (771, 65536), (2048, 65536),
                                 (8192, 65536)])
def test_dense_normal_kernels_agree(M, N):
    """The row-split kernel (PXA_TUNE_NORMAL_KERNEL 0: four workgroups per row, part-dots exchanged) against
    the same kernel computing every part-dot itself (2: the path a workgroup takes when a member is late) BIT
    FOR BIT, and both against the one-workgroup-per-row kernel (1) and float64 within the fp32 tolerance: group
    counts below 8 (solo), ragged parts (N4 not a multiple of 4 x 1024), row counts that leave padding rows."""
    rng = np.random.default_rng(M * 7 + N)
    A = (rng.standard_normal((M, N)) / np.sqrt(M)).astype(np.float32)
    x = rng.standard_normal(N).astype(np.float32)
    Ad, xd = to_device(A), to_device(x)
    out = {}
    old = _dev.tuning(_dev.TUNE_NORMAL_KERNEL, 0)
    try:
        for mode in (0, 2, 1, 0):
            _dev.tuning(_dev.TUNE_NORMAL_KERNEL, mode)
            y = _dev.dense_normal(Ad, xd, 0.7, 1.3)
            torch.cuda.synchronize()
            if mode in out:
                assert torch.equal(out[mode], y)  # run to run
            out[mode] = y
    finally:
        _dev.tuning(_dev.TUNE_NORMAL_KERNEL, old)
    assert torch.equal(out[0], out[2])
    ref = _ref(A, x, 0.7, 1.3)
    assert rel_err(to_NUMPY(out[0]), ref) <= 1e-5
    assert rel_err(to_NUMPY(out[1]), ref) <= 1e-5


def test_dense_normal_refuses_unsupported():
    A = to_device(np.ones((8, 10), np.float32))  # N % 4 != 0
    x = to_device(np.ones(10, np.float32))
    assert not _dev.dense_normal_supported(A, x)
    A64 = to_device(np.ones((8, 16), np.float64))
    assert not _dev.dense_normal_supported(A64, to_device(np.ones(16, np.float64)))
    A2 = to_device(np.ones((8, 16), np.float32))
    assert not _dev.dense_normal_supported(A2, to_device(np.ones((2, 16), np.float32)))  # stacked rhs


def _admm_cg_operator(K, M, tau, w=0.5):
    f = w * pxo.SquaredL2Norm(dim=M).asloss(to_device(np.zeros(M, np.float32))) * K
    Q, _, _ = f._quad_spec()
    return Q + pxo.HomothetyOp(cst=1 / tau, dim=Q.dim)


@pytest.mark.parametrize("w,tau", [(0.5, 1.0), (0.5, 0.25), (2.0, 3.0)])
def test_normal_form_of_admm_operator(w, tau):
    rng = np.random.default_rng(1)
    M, N = 24, 64
    with pxrt.Precision(pxrt.Width.SINGLE):
        K = pxa.LinOp.from_array(to_device(rng.standard_normal((M, N)).astype(np.float32)))
        A = _admm_cg_operator(K, M, tau, w)
        nf = normal_form(A)
        assert nf is not None
        mat, s, d = nf
        assert mat is K._mat
        assert np.isclose(s, 2 * w) and np.isclose(d, 1 / tau)
        p = to_device(rng.standard_normal(N).astype(np.float32))
        assert rel_err(to_NUMPY(_dev.dense_normal(mat, p, s, d)), to_NUMPY(A.apply(p))) <= 1e-5


def test_normal_form_rejects_other_operators():
    rng = np.random.default_rng(2)
    with pxrt.Precision(pxrt.Width.SINGLE):
        K = pxa.LinOp.from_array(to_device(rng.standard_normal((12, 16)).astype(np.float32)))
        K2 = pxa.LinOp.from_array(to_device(rng.standard_normal((12, 16)).astype(np.float32)))
        assert normal_form(K) is None  # not a normal operator
        assert normal_form(K.T * K2) is None  # two different matrices
        assert normal_form(K.T * K + K2.T * K2) is None
        G = pxo.Gradient(arg_shape=(4, 4))
        assert normal_form(G.T * G) is None  # not a dense matrix
        nf = normal_form(K.T * K)
        assert nf is not None and nf[1] == 1.0 and nf[2] == 0.0


@pytest.mark.parametrize("M,N", [(48, 160), (256, 2048)])
def test_admm_fused_normal_matches_generic_and_oracle(M, N):
    """ADMM C4-style: f = 1/2||K . - y||^2, h = lam L1, x-update = QuadraticFunc.prox -> CG.  The fused
    operator (one pass over K) gives the trajectory of the rule-by-rule operator within fp32 rounding,
    and both follow the fp64 oracle (oracle.admm_dense_l1 restating pds.py:1631-1660 + cg.py:125-153)."""
    rng = np.random.default_rng(M)
    A = (rng.standard_normal((M, N)) / np.sqrt(M)).astype(np.float32)
    xs = np.zeros(N, np.float32)
    xs[rng.choice(N, 8, replace=False)] = rng.standard_normal(8).astype(np.float32)
    y = (A @ xs + 0.01 * rng.standard_normal(M)).astype(np.float32)
    lam, tau, iters = 0.05, 1.0, 6
    out = {}
    import pyxu_amd.opt.solver.cg as cgm

    for fused in (True, False):
        saved = cgm.normal_form_ex
        if not fused:
            cgm.normal_form_ex = lambda op: None
        try:
            with pxrt.Precision(pxrt.Width.SINGLE):
                K = pxa.LinOp.from_array(to_device(A))
                f = 0.5 * pxo.SquaredL2Norm(dim=M).asloss(to_device(y)) * K
                h = lam * pxo.L1Norm(dim=N)
                s = pxs.ADMM(f=f, h=h, show_progress=False)
                s.fit(x0=to_device(np.zeros(N, np.float32)), tau=tau, stop_crit=pxst.MaxIter(iters))
                out[fused] = to_NUMPY(s.solution())
        finally:
            cgm.normal_form_ex = saved
    assert rel_err(out[True], out[False]) <= 1e-5
    xr, ur, _, _ = orc.admm_dense_l1(A.astype(np.float64), y.astype(np.float64), lam, np.zeros(N), tau, iters)
    assert rel_err(out[True], xr) <= 1e-4  # solution() = x (primal), fp32 vs the fp64 oracle


def test_cg_published_residual_stat_gives_same_stop_decisions():
    """The inline CG (QuadraticFunc.prox) hands its ||r||^2 to AbsError: same iterations and iterate as
    a CG whose stop criterion recomputes the norm itself."""
    rng = np.random.default_rng(3)
    M, N = 64, 256
    A = (rng.standard_normal((M, N)) / np.sqrt(M)).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    with pxrt.Precision(pxrt.Width.SINGLE):
        K = pxa.LinOp.from_array(to_device(A))
        Aop = K.T * K + pxo.HomothetyOp(cst=1.0, dim=N)
        res = {}
        for internal in (True, False):
            s = pxs.CG(A=Aop, show_progress=False, _internal=internal)
            crit = s.default_stop_crit() | pxst.MaxIter(2 * N)
            if internal:
                s._solve_inline(b=to_device(b), stop_crit=crit)
            else:
                s.fit(b=to_device(b), stop_crit=crit)
            res[internal] = (s._astate["idx"], to_NUMPY(s.solution()))
    assert res[True][0] == res[False][0]
    assert np.array_equal(res[True][1], res[False][1])


@pytest.mark.parametrize("M,N,mode", [(1024, 8192, 0), (256, 65536, 0), (300, 1000, 0), (64, 40000, 0),
                                      (512, 8192, 1), (2048, 65536, 1)])
def test_fused_cg_dot_same_bits(M, N, mode):
    """CG on the dense normal operator with <p, A p> folded into the operator's reduction launch
    (pxa_dense_normal_pdot + pxa_cg_update_tail) against the separate cg_dot launch: the same iterates and
    iteration count, bit for bit.  Shapes: the fused kernel with 2 partial slices (N % 256 chunks), chunks
    that are not float4 multiples or beyond the LDS stage (N = 1000, 40000: the fallback dot launch), and the
    one-workgroup-per-row kernel (mode 1: 8 slices, the fallback)."""
    import pyxu_amd.opt.solver.cg as cgm

    rng = np.random.default_rng(M + N)
    A = (rng.standard_normal((M, N)) / np.sqrt(M)).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    res = {}
    old = _dev.tuning(_dev.TUNE_NORMAL_KERNEL, mode)
    try:
        for fused in (True, False):
            cgm._FUSED_DOT = fused
            with pxrt.Precision(pxrt.Width.SINGLE):
                K = pxa.LinOp.from_array(to_device(A))
                q = pxa.QuadraticFunc(shape=(1, N), Q=K.T * K)
                x = q.prox(to_device(b), 0.5)  # CG on K^T K + 2 I, the sub-solver ADMM runs
                slvr = q._prox_cg(np.float32(0.5))[0]
                assert slvr._apply.fused
                res[fused] = (slvr._astate["idx"], to_NUMPY(x))
    finally:
        cgm._FUSED_DOT = True
        _dev.tuning(_dev.TUNE_NORMAL_KERNEL, old)
    assert res[True][0] == res[False][0] and res[True][0] >= 5
    assert np.array_equal(res[True][1].view(np.uint32), res[False][1].view(np.uint32))


@pytest.mark.parametrize("M,N,mode", [(1024, 8192, 0), (256, 65536, 0), (64, 40000, 0), (512, 8192, 2)])
def test_cg_p_fold_same_bits(M, N, mode):
    """The CG's p' = r' + beta p formed inside the next operator pass (pxa_cg_update_xr, then
    pxa_dense_normal_pdot_pfold, which also publishes ||r'||^2) against pxa_cg_update's own p launch: the same
    solution, residual, direction and iteration count, bit for bit; the fold path is taken (mode 2: every member
    forms the other parts' operand itself, from r' and p)."""
    import pyxu_amd.opt.solver.cg as cgm

    rng = np.random.default_rng(M + 3 * N)
    A = (rng.standard_normal((M, N)) / np.sqrt(M)).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    res, calls = {}, [0]
    orig = _dev.dense_normal_pfold

    def counted(*a, **k):
        calls[0] += 1
        return orig(*a, **k)

    old = _dev.tuning(_dev.TUNE_NORMAL_KERNEL, mode)
    _dev.dense_normal_pfold = counted
    try:
        for fold in (True, False):
            cgm._FOLD_P = fold
            with pxrt.Precision(pxrt.Width.SINGLE):
                K = pxa.LinOp.from_array(to_device(A))
                q = pxa.QuadraticFunc(shape=(1, N), Q=K.T * K)
                x = q.prox(to_device(b), 0.5)
                slvr = q._prox_cg(np.float32(0.5))[0]
                m = slvr._mstate
                res[fold] = (slvr._astate["idx"], to_NUMPY(x), to_NUMPY(m["residual"]), to_NUMPY(m["conjugate_dir"]))
            if fold:
                assert calls[0] >= 3, calls
    finally:
        cgm._FOLD_P = True
        _dev.dense_normal_pfold = orig
        _dev.tuning(_dev.TUNE_NORMAL_KERNEL, old)
    assert res[True][0] == res[False][0] and res[True][0] >= 5
    for a_, b_ in zip(res[True][1:], res[False][1:]):
        assert np.array_equal(a_.view(np.uint32), b_.view(np.uint32))
