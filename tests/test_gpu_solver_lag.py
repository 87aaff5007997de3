"""
Lagged stop checks (abc/solver.py _lag_loop; VERDICT r05 Next #2): at stop_rate 1 the fused PGD solver keeps up to
_LAG RelError checks unresolved while the device runs ahead, and ends in the state of the check that fired.  Against
the synchronous reference order (solver.py:588-663, stop.py:353-382) on the same problem: the same stop iteration,
the same iterate bit for bit, the same history records (MaxIter counts checks), the same steps() items, also when
steps() is consumed in pieces, and the same log lines.  With the default window statistics (the next step's
(x, x_prev) loads: the same sums in another order) the RelError values agree to 1e-12 relative instead of bit for
bit; with the epilogue statistics they are bit-identical.
"""
import re

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
from pyxu_amd.util import to_device, to_NUMPY  # noqa: E402


def _problem(sh=(96, 128), stack=1):
    rng = np.random.default_rng(3)
    N = int(np.prod(sh))
    lam, mu = 0.02, 0.01
    y = rng.standard_normal(stack * N).astype(np.float32)
    if stack == 1:
        H = pxo.Gaussian(arg_shape=sh, sigma=1.5)
        G = pxo.Gradient(arg_shape=sh)
        l21 = pxo.L21Norm(arg_shape=(2, *sh))
    else:
        H = pxo.Gaussian(arg_shape=(stack, *sh), sigma=(0, 1.5, 1.5))
        G = pxo.Gradient(arg_shape=(stack, *sh), directions=(1, 2))
        l21 = pxo.L21Norm(arg_shape=(2, stack, *sh))
    f = 0.5 * pxo.SquaredL2Norm(dim=stack * N).asloss(to_device(y)) * H + lam * l21.moreau_envelope(mu) * G
    f.diff_lipschitz = 1 + 8 * lam / mu
    return f, pxo.PositiveOrthant(dim=stack * N), stack * N


def _run(lagged, crit_fn, mode, monkeypatch, tmp_path, tag, depth=8, inkernel=False, pieces=None, stack=1, window=True,
         pub=True):
    monkeypatch.setattr(pxa.Solver, "_LAG", depth if lagged else 0)
    monkeypatch.setattr(pxa.Solver, "_LAG_INKERNEL", inkernel)
    monkeypatch.setattr(pxa.Solver, "_LAG_WINDOW", window)
    monkeypatch.setattr(pxs.PGD, "_LAG_PUB", pub)
    if not lagged:  # the synchronous reference order itself (no speculative checks either)
        monkeypatch.setattr(pxs.PGD, "_spec_supported", lambda self: False)
    monkeypatch.setattr(pxa.Solver, "_LAG_INKERNEL", inkernel)
    with pxrt.Precision(pxrt.Width.SINGLE):
        f, g, N = _problem(stack=stack)
        s = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=1, folder=tmp_path / tag)
        x0 = to_device(np.zeros(N, np.float32))
        items, stats_eq = [], True
        if mode == "BLOCK":
            s.fit(x0=x0, stop_crit=crit_fn())
        else:
            s.fit(x0=x0, stop_crit=crit_fn(), mode=pxa.Mode.MANUAL)
            for n in (pieces or [None]):
                for it in s.steps(n):
                    items.append(to_NUMPY(it["x"]))
                    stats_eq &= bool(torch.equal(s.stats()[0]["x"], it["x"]))  # stats() between items: that item
        data, hist = s.stats()
        log = (tmp_path / tag / "solver.log").read_text()
        log = re.sub(r"\[[0-9: .-]+\]", "[t]", log)  # time stamps differ
        return dict(x=to_NUMPY(data["x"]), idx=s._astate["idx"], a=next(s._mstate["a"]), items=items, stats_eq=stats_eq,
                    hist={k: np.asarray(hist[k]) for k in hist.dtype.names}, log=log)


def _same(a, b, exact_rel=True, items=True):
    """Same run.  exact_rel=False (window statistics: the RelError sums of the same terms in another order): the
    RelError history values within 1e-12 relative, the log lines identical once their numbers are rounded to 9
    significant digits; everything else bit for bit."""
    assert a["idx"] == b["idx"] and a["a"] == b["a"]
    assert np.array_equal(a["x"], b["x"])
    assert set(a["hist"]) == set(b["hist"])
    for k in b["hist"]:
        if k.startswith("RelError") and not exact_rel:
            np.testing.assert_allclose(a["hist"][k], b["hist"][k], rtol=1e-12, atol=0, err_msg=k)
        else:
            np.testing.assert_array_equal(a["hist"][k], b["hist"][k], err_msg=k)
    if exact_rel:
        assert a["log"] == b["log"]
    else:
        rnd = lambda t: re.sub(r"[0-9]+\.[0-9]+(e[-+][0-9]+)?", lambda m: f"{float(m.group(0)):.9g}", t)  # noqa: E731
        assert rnd(a["log"]) == rnd(b["log"])
    if items:
        assert len(a["items"]) == len(b["items"])
        for u, v in zip(a["items"], b["items"]):
            assert np.array_equal(u, v)


@pytest.mark.parametrize("mode", ["BLOCK", "MANUAL"])
@pytest.mark.parametrize("stats", ["window", "window_fold_launch", "epilogue_fold_launch", "epilogue_inkernel_fold"])
def test_lagged_checks_match_synchronous_relerr_stop(mode, stats, monkeypatch, tmp_path):
    """RelError fires mid-run (~ iteration 60 of a MaxIter(500) budget).  Statistics from the next step's window
    (default), or from the step's epilogue folded by a fold launch / the step's last workgroup (bit-identical
    history)."""
    crit = lambda: pxst.MaxIter(500) | pxst.RelError(eps=3e-3)  # noqa: E731
    a = _run(True, crit, mode, monkeypatch, tmp_path, "lag", inkernel=stats == "epilogue_inkernel_fold",
             window=stats.startswith("window"), pub=stats == "window")
    b = _run(False, crit, mode, monkeypatch, tmp_path, "sync")
    monkeypatch.undo()
    assert 20 < b["idx"] < 500
    _same(a, b, exact_rel=not stats.startswith("window"))
    assert a["stats_eq"]


@pytest.mark.parametrize("depth", [1, 3, 16])
def test_lagged_checks_maxiter_stop_and_depths(depth, monkeypatch, tmp_path):
    """MaxIter fires first (every pending check resolved in order before it), at several lag depths; a stack of
    3 images (rows of the RelError statistics)."""
    crit = lambda: pxst.RelError(eps=1e-9) | pxst.MaxIter(37)  # noqa: E731
    a = _run(True, crit, "MANUAL", monkeypatch, tmp_path, "lag", depth=depth, stack=3)
    b = _run(False, crit, "MANUAL", monkeypatch, tmp_path, "sync", stack=3)
    assert b["idx"] == 37 and b["hist"]["N_iter"][-1] == 38
    _same(a, b, exact_rel=False)


def test_lagged_steps_consumed_in_pieces(monkeypatch, tmp_path):
    """steps(n) closed while checks are in flight returns to the state of its last item (the launches after it
    dropped); the next steps() continues exactly as the synchronous path."""
    crit = lambda: pxst.MaxIter(500) | pxst.RelError(eps=3e-3)  # noqa: E731
    a = _run(True, crit, "MANUAL", monkeypatch, tmp_path, "lag", pieces=[5, 1, 17, None])
    b = _run(False, crit, "MANUAL", monkeypatch, tmp_path, "sync")
    _same(a, b, exact_rel=False)
