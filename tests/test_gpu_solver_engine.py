"""
Solver-engine paths on the device (abc/solver.py, opt/stop.py): device-side Memorize (MIN / MAX
reductions + asynchronous D2H), asynchronous mid-run checkpoints, ASYNC-mode stats.  The PGD
iterates themselves are pinned by test_gpu_parity.py; here the engine bookkeeping is checked
against values recomputed from the same device state.
"""
import time

import numpy as np
import pytest

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
from pyxu_amd.util import to_device, to_NUMPY  # noqa: E402


def _problem(sh=(48, 40), stack=1):
    rng = np.random.default_rng(7)
    N = int(np.prod(sh))
    y = rng.standard_normal(N)
    with pxrt.Precision(pxrt.Width.DOUBLE):
        H = pxo.Gaussian(arg_shape=sh, sigma=1.0)
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(to_device(y)) * H
        f.diff_lipschitz = 1.0
        g = 0.05 * pxo.L1Norm(dim=N)
    x0 = rng.uniform(0, 1, (stack, N) if stack > 1 else N)
    return f, g, x0


@pytest.mark.parametrize("stack", [1, 3])
def test_track_objective_and_async_checkpoints(tmp_path, stack):
    f, g, x0 = _problem(stack=stack)
    with pxrt.Precision(pxrt.Width.DOUBLE):
        s = pxs.PGD(f=f, g=g, show_progress=False, folder=tmp_path / "w", stop_rate=2, writeback_rate=4)
        s.fit(x0=to_device(x0), stop_crit=pxst.MaxIter(6), track_objective=True)
        d = np.load(s.datafile)
        assert np.array_equal(d["x"], to_NUMPY(s.solution()))
        h = d["history"]
        assert list(h["iteration"]) == list(range(0, 13, 2))
        # the final record's Memorize value is the objective of the final state, min / max over the stack
        obj = to_NUMPY(s.objective_func()).reshape(-1)
        if stack == 1:
            assert np.isclose(h["Memorize[objective_func]"][-1], obj[0], rtol=1e-12)
        else:
            assert np.isclose(h["Memorize[objective_func]_min"][-1], obj.min(), rtol=1e-12)
            assert np.isclose(h["Memorize[objective_func]_max"][-1], obj.max(), rtol=1e-12)
        assert not (s.workdir / "data.npz.tmp").exists()


def test_min_max_reductions_match_numpy_with_nan():
    rng = np.random.default_rng(1)
    for dt in (np.float32, np.float64):
        x = rng.standard_normal((5, 1000)).astype(dt)
        x[3, 17] = np.nan
        X = to_device(x)
        mn = to_NUMPY(_dev.row_reduce(_dev.RED_MIN, X))
        mx = to_NUMPY(_dev.row_reduce(_dev.RED_MAX, X))
        assert np.array_equal(mn, x.min(axis=1).astype(np.float64), equal_nan=True)
        assert np.array_equal(mx, x.max(axis=1).astype(np.float64), equal_nan=True)


def test_async_mode_stats_consistent(tmp_path):
    """ASYNC fit: stats() polled while the worker runs never loses / duplicates / reorders a record."""
    f, g, x0 = _problem(sh=(96, 96))
    with pxrt.Precision(pxrt.Width.DOUBLE):
        s = pxs.PGD(f=f, g=g, show_progress=False, folder=tmp_path / "a", stop_rate=1)
        s.fit(x0=to_device(x0), stop_crit=pxst.MaxIter(300), mode=pxa.Mode.ASYNC)
        seen = []
        while s.busy():
            _, h = s.stats()
            if h is not None:
                seen.append(list(h["iteration"]))
            time.sleep(0.002)
        s.stop()
        _, h = s.stats()
    its = list(h["iteration"])
    assert its == list(range(len(its)))
    for snap in seen:
        assert snap == its[: len(snap)]


def _pgd_problem(sh=(64, 96), lam=0.02, mu=0.02):
    rng = np.random.default_rng(4)
    N = int(np.prod(sh))
    y = rng.standard_normal(N).astype(np.float32)
    H = pxo.Gaussian(arg_shape=sh, sigma=1.5)
    G = pxo.Gradient(arg_shape=sh)
    f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(to_device(y)) * H + lam * pxo.L21Norm(arg_shape=(2, *sh)).moreau_envelope(mu) * G
    f.diff_lipschitz = 1 + 8 * lam / mu
    return f, pxo.PositiveOrthant(dim=N), N


@pytest.mark.parametrize("stop_rate", [1, 3])
@pytest.mark.parametrize("mode", ["BLOCK", "MANUAL"])
def test_speculative_stop_checks_match_synchronous(stop_rate, mode, monkeypatch):
    """Speculative stop checks (the next fused PGD step runs while the host reads the RelError
    statistics, and is undone when the criterion fires) end with the same iterate, iteration count,
    momentum and history as the synchronous checks of the reference order (solver.py:588-652)."""
    res = {}
    for spec in (True, False):
        if not spec:  # the synchronous reference order: neither speculative nor lagged checks
            monkeypatch.setattr(pxs.PGD, "_spec_supported", lambda self: False)
            monkeypatch.setattr(pxs.PGD, "_lag_supported", lambda self: False)
        else:  # the speculative path itself (at stop_rate 1 the lagged engine would take over)
            monkeypatch.setattr(pxs.PGD, "_lag_supported", lambda self: False)
        with pxrt.Precision(pxrt.Width.SINGLE):
            f, g, N = _pgd_problem()
            s = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=stop_rate)
            crit = pxst.RelError(eps=2e-3) | pxst.MaxIter(400)
            x0 = to_device(np.zeros(N, np.float32))
            if mode == "BLOCK":
                s.fit(x0=x0, stop_crit=crit)
            else:
                s.fit(x0=x0, stop_crit=crit, mode=pxa.Mode.MANUAL)
                for _ in s.steps():
                    pass
            data, hist = s.stats()
            res[spec] = (to_NUMPY(data["x"]), s._astate["idx"], next(s._mstate["a"]),
                         {k: np.asarray(hist[k]) for k in hist.dtype.names})
        monkeypatch.undo()
    xs, idx_s, a_s, h_s = res[True]
    xn, idx_n, a_n, h_n = res[False]
    assert 20 < idx_n < 400 * stop_rate  # the relative-error criterion fired (MaxIter counts checks)
    assert idx_s == idx_n and a_s == a_n
    assert np.array_equal(xs, xn)
    assert set(h_s) == set(h_n)
    for k in h_n:
        if k == "duration":
            continue
        np.testing.assert_array_equal(h_s[k], h_n[k], err_msg=k)


def test_async_log_lags_by_at_most_one_batch(tmp_path):
    """ASYNC fit of the fused PGD with speculative checks at stop_rate 1: solver.log, read while the worker
    runs, trails the iteration count by at most two record batches (Solver._RECORD_LAG lines written
    unflushed), and holds every record's line once the solver stopped."""
    lag = pxa.Solver._RECORD_LAG
    with pxrt.Precision(pxrt.Width.SINGLE):
        f, g, N = _pgd_problem()
        s = pxs.PGD(f=f, g=g, show_progress=False, folder=tmp_path / "l", stop_rate=1)
        s.fit(x0=to_device(np.zeros(N, np.float32)), stop_crit=pxst.MaxIter(3000), mode=pxa.Mode.ASYNC)
        assert s._plan is not None and s._spec_supported()
        worst = 0
        while s.busy():
            before = s._astate["idx"]
            lines = s.logfile.read_text().count("] Iteration ")
            worst = max(worst, before - lines)
            time.sleep(0.005)
        s.stop()
        _, h = s.stats()
    assert worst <= 2 * lag + 4, worst
    assert s.logfile.read_text().count("] Iteration ") == len(h["iteration"])
