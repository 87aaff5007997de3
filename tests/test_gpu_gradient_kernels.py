"""pxa_gradient2 / pxa_gradient2_adjoint: the axis-0 march kernels (PXA_TUNE_GRAD_KERNEL 0, default) against
the row kernels of rounds 1-3 (1) -- the same expressions per element, so the same bits -- and both against a
NumPy restatement of the reference's Trim o S o Pad finite differences (diff.py:157-261 via the oracle's
gradient) on 1-D to 4-D shapes, stacks, vector and scalar rows, and forward / backward / central taps."""
import numpy as np
import pytest
import torch

from pyxu_amd import _dev

pytestmark = pytest.mark.gpu


def np_dir(x, axis, o0, c0, o1, c1):
    """c0 x[i + o0 e_axis] + c1 x[i + o1 e_axis], zero outside (constant mode)"""
    def shifted(o):
        out = np.zeros_like(x)
        n = x.shape[axis]
        src = [slice(None)] * x.ndim
        dst = [slice(None)] * x.ndim
        if o >= 0:
            src[axis], dst[axis] = slice(o, n), slice(0, n - o)
        else:
            src[axis], dst[axis] = slice(0, n + o), slice(-o, n)
        out[tuple(dst)] = x[tuple(src)]
        return out
    return c0 * shifted(o0) + c1 * shifted(o1)


SCHEMES = {"forward": (0, -1.0, 1, 1.0), "backward": (-1, -1.0, 0, 1.0), "central": (-1, -0.5, 1, 0.5)}


@pytest.mark.parametrize("shape,stack", [((4096,), 1), ((64, 128), 2), ((2048, 2047), 1), ((33, 40, 64), 1),
                                         ((16, 8, 12, 32), 1), ((128, 256, 256), 1)])
@pytest.mark.parametrize("scheme", ["forward", "backward", "central"])
@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_gradient_march_matches_rows(shape, stack, scheme, dt):
    o0, c0, o1, c1 = SCHEMES[scheme]
    D = len(shape)
    dirs = list(range(D))
    rng = np.random.default_rng(sum(shape) + stack)
    x = rng.standard_normal((stack, *shape))
    xt = torch.tensor(x.reshape(-1), dtype=dt, device="cuda")
    args = (stack, list(shape), dirs, [o0] * D, [c0] * D, [o1] * D, [c1] * D)
    res = {}
    old = _dev.tuning(_dev.TUNE_GRAD_KERNEL, 0)
    try:
        for mode in (0, 1):
            _dev.tuning(_dev.TUNE_GRAD_KERNEL, mode)
            g = _dev.gradient2(xt, *args)
            a = _dev.gradient2(g, *args, adjoint=True)
            res[mode] = (g.cpu().numpy(), a.cpu().numpy())
    finally:
        _dev.tuning(_dev.TUNE_GRAD_KERNEL, old)
    assert np.array_equal(res[0][0], res[1][0]) and np.array_equal(res[0][1], res[1][1])
    ref = np.stack([np.stack([np_dir(x[s], d, o0, c0, o1, c1) for d in dirs]) for s in range(stack)])
    tol = 1e-6 if dt == torch.float32 else 1e-13
    g0 = res[0][0].reshape(ref.shape)
    assert np.max(np.abs(g0 - ref)) <= tol * max(1.0, np.max(np.abs(ref)))
    # adjoint: <G x, G x> == <x, G^T G x>
    gx = g0.reshape(-1).astype(np.float64)
    lhs = float(gx @ gx)
    rhs = float(x.reshape(-1) @ res[0][1].astype(np.float64))
    assert abs(lhs - rhs) <= (1e-5 if dt == torch.float32 else 1e-12) * abs(lhs)


def test_gradient_march_subset_directions():
    """directions (2, 0) of a 3-D volume (axis 0 not first, the last axis first) and a single middle axis"""
    rng = np.random.default_rng(5)
    x = rng.standard_normal((24, 16, 40))
    xt = torch.tensor(x.reshape(-1), dtype=torch.float32, device="cuda")
    for dirs in ([2, 0], [1]):
        D = len(dirs)
        args = (1, [24, 16, 40], dirs, [0] * D, [-1.0] * D, [1] * D, [1.0] * D)
        out = {}
        for mode in (0, 1):
            old = _dev.tuning(_dev.TUNE_GRAD_KERNEL, mode)
            try:
                g = _dev.gradient2(xt, *args)
                out[mode] = (g.cpu().numpy(), _dev.gradient2(g, *args, adjoint=True).cpu().numpy())
            finally:
                _dev.tuning(_dev.TUNE_GRAD_KERNEL, old)
        assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
        ref = np.stack([np_dir(x, d, 0, -1.0, 1, 1.0) for d in dirs]).reshape(-1)
        assert np.max(np.abs(out[0][0] - ref)) <= 1e-6
