"""CPU-only tests: C-ABI symbol table, operator algebra / Lipschitz bookkeeping, step-size rules,
tap generation, fused-plan recognition, solver bookkeeping.  No compute calls (no GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle as orc
from conftest import ROOT, golden_names, load_golden

import pyxu_amd
import pyxu_amd.abc as pxa
import pyxu_amd.operator as pxo
import pyxu_amd.opt.solver as pxs
import pyxu_amd.opt.stop as pxst
import pyxu_amd.runtime as pxrt
from pyxu_amd._lib import EXPORTS, LIB_PATH


def _header_functions():
    txt = open(os.path.join(ROOT, "include", "pyxu_amd.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pxa_\w+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    assert os.path.exists(LIB_PATH), "run __graft_entry__.build() first"
    lib = ctypes.CDLL(LIB_PATH)
    names = _header_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), n
    # the Python binding covers the whole header, and nothing else
    assert set(names) == set(EXPORTS), set(names) ^ set(EXPORTS)
    assert lib.pxa_abi_version() == 1


def test_error_strings():
    lib = pyxu_amd.lib
    assert lib.pxa_error_string(0) == b"success"
    assert b"invalid argument" in lib.pxa_error_string(-1)


def test_argument_validation_without_gpu():
    # invalid arguments are rejected on the host before any launch
    lib = pyxu_amd.lib
    assert lib.pxa_axpby(7, 10, 1.0, None, 0.0, None, None, None) == -2  # bad dtype
    assert lib.pxa_row_reduce(0, 99, 1, 4, 1, None, 1, 1, None) == -1  # bad op
    assert lib.pxa_pgd_tv2d_step(0, 1, 1, 8, 8, 0, None, None, 0, None, None, 1, 1, 0, 1, 0, 1, 0, 0, 1, 2, 3, 4, None, None, None) == -1


@pytest.mark.parametrize("name", golden_names("gaussian_"))
def test_gaussian_taps_match_reference(name):
    g = load_golden(name)
    with pxrt.Precision(pxrt.Width.SINGLE if g["x"].dtype == np.float32 else pxrt.Width.DOUBLE):
        op = pxo.Gaussian(arg_shape=tuple(g["arg_shape"]), sigma=float(g["sigma"]))
    np.testing.assert_array_equal(op.kernel[0], g["taps"])
    from scipy.ndimage._filters import _gaussian_kernel1d

    from pyxu_amd.operator.linop.filter import gaussian_kernel1d

    for order in (0, 1, 2):
        np.testing.assert_allclose(gaussian_kernel1d(1.7, order, 6), _gaussian_kernel1d(1.7, order, 6), rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("name", golden_names("stencil_"))
def test_stencil_lipschitz_and_pad(name):
    g = load_golden(name)
    dt = g["x"].dtype
    ks = [g[f"kernel{i}"] for i in range(int(g["n_kernels"]))]
    kern = ks if bool(g["separable"]) else ks[0]
    mode = str(g["mode"]) if g["mode"].ndim == 0 else tuple(str(s) for s in g["mode"])
    with pxrt.Precision(pxrt.Width.SINGLE if dt == np.float32 else pxrt.Width.DOUBLE):
        op = pxo.Stencil(arg_shape=tuple(g["arg_shape"]), kernel=kern, center=tuple(g["center"]), mode=mode)
        assert np.isclose(float(op.lipschitz), float(g["lipschitz"]), rtol=1e-6)
        assert op.shape == (int(np.prod(g["arg_shape"])),) * 2


@pytest.mark.parametrize("name", golden_names("gradient_"))
def test_gradient_lipschitz(name):
    g = load_golden(name)
    with pxrt.Precision(pxrt.Width.SINGLE if g["x"].dtype == np.float32 else pxrt.Width.DOUBLE):
        op = pxo.Gradient(arg_shape=tuple(g["arg_shape"]), directions=tuple(g["directions"]), mode=str(g["mode"]),
                          scheme=str(g["scheme"]), accuracy=int(g["accuracy"]), sampling=float(g["sampling"]))
    assert np.isclose(float(op.lipschitz), float(g["lipschitz"]), rtol=1e-6)
    assert op.shape == (len(g["directions"]) * int(np.prod(g["arg_shape"])), int(np.prod(g["arg_shape"])))
    # default forward scheme (and backward) run through the one-pass fused kernel
    if str(g["mode"]) == "constant" and (str(g["scheme"]) != "central"):
        assert op._fused is not None


def test_fd_taps_match_oracle():
    from pyxu_amd.operator.linop.diff import fd_coefficients

    for scheme in ("forward", "backward", "central"):
        for acc in (1, 2, 3):
            for dt in (np.float32, np.float64):
                a = fd_coefficients(1, scheme, acc, 0.5, dt)
                b = orc.fd_taps(1, scheme, acc, 0.5, dt)
                assert a[0] == b[0] and a[2] == b[2]
                np.testing.assert_array_equal(a[1], b[1])


def test_operator_algebra_types():
    torch = pytest.importorskip("torch")
    sh = (16, 20)
    N = 320
    with pxrt.Precision(pxrt.Width.SINGLE):
        H = pxo.Gaussian(arg_shape=sh, sigma=2.0)
        G = pxo.Gradient(arg_shape=sh)
        y = torch.zeros(N)  # host tensor: construction only
        data = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(y) * H
        assert isinstance(data, pxa.QuadraticFunc)
        assert np.isinf(data.diff_lipschitz)  # reference semantics: unknown until set
        tv = 0.01 * pxo.L21Norm(arg_shape=(2, *sh)).moreau_envelope(0.01) * G
        assert isinstance(tv, pxa.DiffFunc) and np.isclose(tv.diff_lipschitz, 0.01 / 0.01 * 8, rtol=1e-6)
        f = data + tv
        assert isinstance(f, pxa.DiffFunc) and not isinstance(f, pxa.ProxFunc)
        assert isinstance(G.T, pxa.LinOp) and G.T.shape == (N, 2 * N)
        assert isinstance(2 * pxo.L1Norm(dim=N), pxa.ProxFunc)
        assert isinstance(-pxo.L1Norm(dim=N), pxa.Func) and not isinstance(-pxo.L1Norm(dim=N), pxa.ProxFunc)
        assert isinstance(H.gram(), pxa.SelfAdjointOp)


def test_fused_plan_recognition():
    torch = pytest.importorskip("torch")
    from pyxu_amd.opt.solver._fused import match_pgd_deblur

    sh = (64, 48)
    N = int(np.prod(sh))
    with pxrt.Precision(pxrt.Width.SINGLE):
        y = torch.zeros(N)
        x0 = torch.zeros(N)
        H = pxo.Gaussian(arg_shape=sh, sigma=2.0)
        data = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(y) * H
        tv = 0.01 * pxo.L21Norm(arg_shape=(2, *sh)).moreau_envelope(0.02) * pxo.Gradient(arg_shape=sh)
        p = match_pgd_deblur(data + tv, pxo.PositiveOrthant(dim=N), x0)
        assert p is not None and p["prox"] == 1 and np.isclose(p["lam"], 0.01) and np.isclose(p["mu"], 0.02)
        assert p["n0"] == 64 and p["n1"] == 48 and len(p["taps0"][0]) == 13
        p = match_pgd_deblur(data, 0.3 * pxo.L1Norm(dim=N), x0)
        assert p is not None and p["prox"] == 2 and np.isclose(p["prox_scale"], 0.3) and p["lam"] == 0.0
        # not recognised -> generic path
        assert match_pgd_deblur(data, pxo.L21Norm(arg_shape=(2, 32, 48)), x0) is None
        Hs = pxo.Gaussian(arg_shape=sh, sigma=2.0, mode="symmetric")
        assert match_pgd_deblur(0.5 * pxo.SquaredL2Norm(dim=N).asloss(y) * Hs, None, x0) is None
        # batch-as-axis
        B = 3
        Hb = pxo.Gaussian(arg_shape=(B, *sh), sigma=(0, 2.0, 2.0))
        Gb = pxo.Gradient(arg_shape=(B, *sh), directions=(1, 2))
        fb = 0.5 * pxo.SquaredL2Norm(dim=B * N).asloss(torch.zeros(B * N)) * Hb + 0.01 * pxo.L21Norm(arg_shape=(2, B, *sh)).moreau_envelope(0.01) * Gb
        pb = match_pgd_deblur(fb, pxo.PositiveOrthant(dim=B * N), torch.zeros(B * N))
        assert pb is not None and pb["B"] == B


@pytest.mark.parametrize("name", golden_names("pds_"))
def test_pds_step_sizes_match_reference(name):
    g = load_golden(name)
    dt = g["x0"].dtype
    sh = tuple(g["arg_shape"])
    N = int(np.prod(sh))
    torch = pytest.importorskip("torch")
    with pxrt.Precision(pxrt.Width.SINGLE if dt == np.float32 else pxrt.Width.DOUBLE):
        H = pxo.Gaussian(arg_shape=sh, sigma=2.0)
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(torch.zeros(N)) * H
        f.diff_lipschitz = float(g["diff_lipschitz"])
        K = pxo.Gradient(arg_shape=sh)
        assert np.isclose(float(K.lipschitz), float(g["K_lipschitz"]), rtol=1e-7)
        h = 0.01 * pxo.L1Norm(dim=len(sh) * N)
        for key, klass in (("pd3o", pxs.PD3O), ("cv", pxs.CondatVu)):
            s = klass(f=f, h=h, K=K, show_progress=False)
            s._tuning_strategy = 1
            tau, sigma, delta = s._set_step_sizes(None, None, s._set_gamma(1))
            assert tau == g[f"{key}_tau"] and sigma == g[f"{key}_sigma"], key
            assert s._set_momentum_term(None, delta) == g[f"{key}_rho"]


def test_stop_criteria_host_logic():
    m = pxst.MaxIter(3)
    assert [m.stop({}) for _ in range(4)] == [False, False, False, True]
    m.clear()
    assert m.info() == {"N_iter": 0}
    c = pxst.MaxIter(1) | pxst.ManualStop()
    assert c.stop({}) is False and c.stop({}) is True
    with pytest.raises(ValueError):
        pxst.MaxIter(0)
    with pytest.raises(ValueError):
        pxst.RelError(eps=-1)
    with pytest.raises(ValueError):
        pxs.PGD(f=None, g=None)
    with pytest.raises(ValueError):
        pxs.PGD(f=pxo.L1Norm(3), stop_rate=0)


def test_precision_runtime():
    assert pxrt.getPrecision() == pxrt.Width.DOUBLE
    with pxrt.Precision(pxrt.Width.SINGLE):
        assert pxrt.coerce(1.5).dtype == np.float32
        with pxrt.EnforcePrecision(False):
            assert pxrt.coerce(1.5) == 1.5
    assert pxrt.coerce(np.arange(3)).dtype == np.float64
    with pytest.raises(TypeError):
        pxrt.coerce(np.ones(2, dtype=complex))


def test_host_arrays_are_rejected_loudly():
    torch = pytest.importorskip("torch")
    op = pxo.L1Norm(dim=4)
    with pytest.raises(TypeError):
        op.prox(np.ones(4), 0.1)
    with pytest.raises(TypeError):
        op.prox(torch.ones(4, dtype=torch.float64), 0.1)  # CPU tensor: no CPU compute path


# ----------------------------------------------------------------------------- bench harness (no GPU)
def test_bench_auto_stop_rate():
    import bench

    assert bench.auto_stop_rate(20) == 20
    assert bench.auto_stop_rate(200) == 50
    assert bench.auto_stop_rate(60) == 30
    assert bench.auto_stop_rate(97) == 1
    assert bench.auto_stop_rate(7) == 7


def test_bench_launcher_rank_envs_and_argv(tmp_path):
    """`bench.py --gpus N` self-launch: N children, each with its RANK / LOCAL_RANK / WORLD_SIZE and a
    127.0.0.1 rendezvous, started with the parent's argv (no GPU is touched by the parent)."""
    import sys

    import bench

    envs = bench.rank_envs(3, 29555, base={"PATH": "/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert all(e["WORLD_SIZE"] == "3" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555" for e in envs)
    # run the real launcher on a stand-in script that records its env and argv
    script = tmp_path / "child.py"
    script.write_text(
        "import os, sys, json\n"
        f"open(os.path.join({str(tmp_path)!r}, 'r' + os.environ['RANK'] + '.json'), 'w').write(json.dumps("
        "{'argv': sys.argv[1:], 'world': os.environ['WORLD_SIZE'], 'local': os.environ['LOCAL_RANK'], "
        "'addr': os.environ['MASTER_ADDR']}))\n")
    rc = bench.launch(["--gpus", "2", "--steps", "20"], 2, script=str(script))
    assert rc == 0
    import json

    for r in range(2):
        rec = json.loads((tmp_path / f"r{r}.json").read_text())
        assert rec == {"argv": ["--gpus", "2", "--steps", "20"], "world": "2", "local": str(r), "addr": "127.0.0.1"}
    # a failing rank makes the launcher fail (and stops the others)
    bad = tmp_path / "bad.py"
    bad.write_text("import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(3)\ntime.sleep(30)\n")
    assert bench.launch([], 2, script=str(bad)) == 3


def test_threaded_cpu_baseline_is_the_oracle():
    """bench.py's all-core CPU baseline (oracle/parallel.py) computes the single-thread oracle's PGD
    iterates bit for bit."""
    from oracle.parallel import pgd_tv_threaded

    sh = (97, 130)
    rng = np.random.default_rng(0)
    y = rng.standard_normal(sh[0] * sh[1]).astype(np.float32)
    taps, c = orc.gaussian_taps(2.0, 3.0, np.float32)
    blur = dict(arg_shape=sh, kernel=[taps, taps], center=[c, c])
    lam = mu = 0.01
    tau = np.float32(1 / np.float32(1 + 8 * lam / mu))
    x0 = rng.uniform(0, 1, sh[0] * sh[1]).astype(np.float32)
    grad = lambda v: orc.deblur_tv_grad(v, blur, y, lam, mu, dict(arg_shape=sh))
    ref, _ = orc.pgd(x0, grad, lambda z, t: orc.positive_orthant_prox(z), tau, 4)
    for th in (1, 4, 9):
        out, _ = pgd_tv_threaded(x0, blur, y, lam, mu, orc.positive_orthant_prox, tau, 4, th)
        assert np.array_equal(out, ref)


def test_block_operator_property_inference():
    """blocks.py:_COOBlock._infer_op / op(): the classes and Lipschitz bounds the reference infers
    (tests/golden/blocks_*.npz record them from the reference; checked here without a GPU)."""
    from conftest import load_golden

    g = load_golden("blocks_f32")
    with pxrt.Precision(pxrt.Width.SINGLE):
        V = pxo.vstack([pxo.Gradient(arg_shape=(6, 5)), pxo.IdentityOp(dim=30)])
        assert type(V).__name__ == str(g["gradid_cls"]) and V.shape == tuple(g["gradid_shape"])
        assert np.isclose(float(V.lipschitz), float(g["gradid_lip"]), rtol=1e-6)
        F = pxo.hstack([pxo.L1Norm(dim=5), pxo.SquaredL2Norm(dim=7)])
        assert type(F).__name__ == str(g["func_l1l2_cls"])
        Q = pxo.hstack([pxo.SquaredL2Norm(dim=5), 2.0 * pxo.SquaredL2Norm(dim=7)])
        assert type(Q).__name__ == str(g["func_q_cls"])
        assert np.isclose(float(Q.diff_lipschitz), float(g["func_q_dl"]), rtol=1e-6)
        B = pxo.block_diag([pxo.IdentityOp(dim=3), pxo.Gradient(arg_shape=(4,))])
        assert B.shape == (7, 7) and isinstance(B, pxa.SquareOp)
        assert np.isclose(float(B.lipschitz), 2.0)  # block-diagonal: max of the blocks' constants
        assert pxo.vstack([pxo.IdentityOp(dim=4)]).shape == (4, 4)  # a single block is returned as is
        with pytest.raises(AssertionError):
            pxo.vstack([pxo.IdentityOp(dim=4), pxo.IdentityOp(dim=5)])


def test_no_torch_arithmetic_in_the_product_path():
    """Every array operation of pyxu_amd goes through libpyxu_amd.so: torch is the device-array
    container only (north_star).  Allowed: allocation / views / host<->device copies, and the host
    staging of the gloo (CPU) collectives, marked on their lines."""
    import pathlib
    import re

    bad = re.compile(r"torch\.(cat|stack|linalg|matmul|mm|bmm|sqrt|exp|log|abs|sum|mean|where|clamp|maximum|minimum)\(|"
                     r"\.sqrt_\(|\.diagonal\(|broadcast_tensors|\.to\(\s*(torch\.)?(float|double)|\.sum\(\)\.cpu")
    hits = []
    for p in pathlib.Path(ROOT, "pyxu_amd").rglob("*.py"):
        for i, line in enumerate(p.read_text().splitlines(), 1):
            code = line.split("#")[0]
            if bad.search(code) and "gloo" not in line and "host" not in line:
                hits.append(f"{p.relative_to(ROOT)}:{i}: {line.strip()}")
    assert not hits, "\n".join(hits)


def test_filter_and_alias_construction_matches_reference_classes():
    """Host-only: the filters' and alias solvers' classes / shapes equal the reference's (goldens
    filters_*.npz, aliases_*.npz); the numerics are in tests/test_gpu_filters.py."""
    import pyxu_amd.operator as pxo
    import pyxu_amd.opt.solver as pxs
    import pyxu_amd.runtime as pxrt
    from conftest import load_golden

    g = load_golden("filters_f64")
    for tag in ("2d", "3d"):
        sh = tuple(int(v) for v in g[f"shape_{tag}"])
        with pxrt.Precision(pxrt.Width.DOUBLE):
            ops = {
                "dog": pxo.DoG(arg_shape=sh, low_sigma=1.0),
                "laplace": pxo.Laplace(arg_shape=sh),
                "sobel0": pxo.Sobel(arg_shape=sh, axis=0),
                "sobel": pxo.Sobel(arg_shape=sh),
                "prewitt1": pxo.Prewitt(arg_shape=sh, axis=1, mode="edge"),
                "scharr01": pxo.Scharr(arg_shape=sh, axis=(0, 1)),
                "st": pxo.StructureTensor(arg_shape=sh),
                "st_nos": pxo.StructureTensor(arg_shape=sh, smooth_sigma=0, mode="reflect"),
            }
        for k, op in ops.items():
            assert type(op).__name__ == str(g[f"{tag}_{k}_cls"]), (tag, k)
            assert op.shape == tuple(g[f"{tag}_{k}_shape"]), (tag, k)
    a = load_golden("aliases_f64")
    N = int(np.prod(a["arg_shape"]))
    l1 = pxo.L1Norm(dim=N)
    assert type(pxs.PP(g=l1, show_progress=False)).__name__ == str(a["pp_cls"])
    assert type(pxs.DR(g=l1, h=l1, show_progress=False)).__name__ == str(a["dr_cls"])
    assert type(pxs.FB(f=pxo.SquaredL2Norm(dim=N), g=l1, show_progress=False)).__name__ == str(a["fb_cls"])


def test_pad_subsample_shapes_and_lipschitz_match_reference():
    """Host-only: Pad / SubSample / Trim shapes and Pad's Lipschitz rule vs padselect goldens, and
    the SubSample index resolution (numpy semantics) vs a NumPy evaluation of the same selector."""
    import pyxu_amd.operator as pxo
    from conftest import load_golden

    g = load_golden("padselect_f64")
    pads = {"w2": ((5, 6), ((2, 1), (0, 3)), "wrap"), "r2": ((5, 6), (2, 3), "reflect"),
            "e2": ((5, 6), ((3, 0), (1, 4)), "edge"),
            "mix": ((5, 6, 4), ((1, 2), (3, 3), (0, 2)), ("edge", "wrap", "reflect"))}
    for k, (sh, pw, mode) in pads.items():
        op = pxo.Pad(arg_shape=sh, pad_width=pw, mode=mode)
        assert op.shape == tuple(g[f"pad_{k}_shape"]) and np.isclose(op.lipschitz, float(g[f"pad_{k}_lip"]))
    sels = {"rep": ((8, 6), ([2, 5, 2, 7],)), "pairs": ((6, 7), ([0, 2, 5], [1, 1, 6])),
            "neg": ((9, 8), (slice(None, None, -2), slice(2, 7))),
            "mask": ((3, 5, 4), (0, np.r_[True, False, False, True, False]))}
    for k, (sh, idx) in sels.items():
        op = pxo.SubSample(sh, *idx)
        assert op.shape == tuple(g[f"sel_{k}_shape"]), k
        x = g[f"sel_{k}_x"][0]
        assert np.array_equal(x[op._pos_host], g[f"sel_{k}_y"][0]), k  # resolved positions reproduce apply
        z = g[f"sel_{k}_z"][0]
        up = np.zeros(op.dim)
        up[op._pos_host[op._keep_host]] = z[op._keep_host]
        assert np.array_equal(up, g[f"sel_{k}_adj"][0]), k  # last-write-wins adjoint
    with pytest.raises(AssertionError):
        pxo.Pad(arg_shape=(4,), pad_width=4, mode="reflect")


class _ToySolver:
    """Host-only solver over numpy state: x_{k+1} = x_k / 2 (exercises the engine, not the math)."""

    @staticmethod
    def make(**kw):
        import pyxu_amd.abc as pxa

        class Toy(pxa.Solver):
            def m_init(self, x0, fail_at=None):
                self._mstate["x"] = np.asarray(x0, dtype=np.float64)
                self._mstate["k"] = 0
                self._fail_at = fail_at

            def m_step(self):
                self._mstate["k"] += 1
                if self._fail_at is not None and self._mstate["k"] == self._fail_at:
                    raise RuntimeError("boom")
                self._mstate["x"] = self._mstate["x"] / 2

            def default_stop_crit(self):
                import pyxu_amd.opt.stop as pxst

                return pxst.MaxIter(5)

            def objective_func(self):
                return np.r_[float(np.sum(self._mstate["x"]))]

            def solution(self):
                return self._mstate["x"]

        return Toy(log_var="x", show_progress=False, **kw)


def test_writeback_checkpoints_and_history_semantics(tmp_path):
    """stop_rate / writeback_rate / verbosity bookkeeping of abc/solver.py (reference solver.py:588-663):
    asynchronous mid-run checkpoints land in order and the final data.npz holds the final state;
    history has one record per stop check; track_objective adds Memorize columns."""
    import pyxu_amd.opt.stop as pxst

    s = _ToySolver.make(folder=tmp_path / "a", stop_rate=2, writeback_rate=4)
    s.fit(x0=np.ones(3) * 64, stop_crit=pxst.MaxIter(9), track_objective=True)
    d = np.load(s.datafile)
    # MaxIter counts stop checks (reference stop.py MaxIter): the 10th check, at idx 18, stops
    assert np.array_equal(d["x"], np.ones(3) * 64 / 2**18)
    h = d["history"]
    assert list(h["iteration"]) == list(range(0, 19, 2))
    assert "Memorize[objective_func]" in h.dtype.names
    assert np.allclose(h["Memorize[objective_func]"], [3 * 64 / 2**i for i in range(0, 19, 2)])
    assert not (s.workdir / "data.npz.tmp").exists()

    # MANUAL mode: a checkpoint at idx 4 holds the pre-step state x_4
    s2 = _ToySolver.make(folder=tmp_path / "b", stop_rate=1, writeback_rate=4)
    s2.fit(x0=np.ones(2) * 16, stop_crit=pxst.MaxIter(100), mode=__import__("pyxu_amd.abc", fromlist=["Mode"]).Mode.MANUAL)
    for _ in s2.steps(5):
        pass
    s2._wb_drain()
    assert np.array_equal(np.load(s2.datafile)["x"], np.ones(2) * 16 / 2**4)


def test_writeback_bad_rates_and_failure_keeps_last_checkpoint(tmp_path, capsys):
    import pyxu_amd.opt.stop as pxst

    with pytest.raises(ValueError):
        _ToySolver.make(folder=tmp_path / "c", stop_rate=3, writeback_rate=4)
    with pytest.raises(ValueError):
        _ToySolver.make(folder=tmp_path / "d", stop_rate=2, verbosity=3)
    s = _ToySolver.make(folder=tmp_path / "e", stop_rate=1, writeback_rate=2)
    s.fit(x0=np.ones(2) * 8, stop_crit=pxst.MaxIter(50), fail_at=5)
    err = capsys.readouterr().err
    assert "Something went wrong" in err
    log = s.logfile.read_text()
    assert "Last valid checkpoint done at iteration=4" in log
    assert np.array_equal(np.load(s.datafile)["x"], np.ones(2) * 8 / 2**4)


def test_atomic_savez_concurrent_writers(tmp_path):
    """Concurrent checkpoint writers (the caller's writeback() and the asynchronous writer thread) each
    write a temporary file of their own and never leave a partial data.npz."""
    import threading

    from pyxu_amd.abc.solver import _atomic_savez

    path = tmp_path / "data.npz"
    errs = []

    def writer(v):
        try:
            for _ in range(20):
                _atomic_savez(path, {"x": np.full(20000, v, dtype=np.float64)})
        except Exception as e:  # pragma: no cover
            errs.append(e)

    ts = [threading.Thread(target=writer, args=(float(i),)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs
    with np.load(path) as f:
        x = f["x"]
    assert x.shape == (20000,) and np.all(x == x[0])
    assert [p.name for p in tmp_path.iterdir()] == ["data.npz"]  # no stray temporary files


def test_distributed_device_path_has_no_torch_kernels():
    """distributed.py moves device data only through the HIP library (pxa_copy2d / pxa_fill): every torch
    copy / fill / concatenation / in-place arithmetic in the module sits on a line marked as the gloo
    host-staging path (or inside the CPU-test fallbacks of _dev_zeros / _dev_copy_rows)."""
    src = open(os.path.join(ROOT, "pyxu_amd", "distributed.py")).read().splitlines()
    pat = re.compile(r"torch\.(zeros|cat|stack|ones|full)\(|\.contiguous\(\)\.|\.copy_\(|\.add_\(|\+= |\] = ")
    fallback = False
    bad = []
    for i, line in enumerate(src, 1):
        if line.startswith("def "):
            fallback = line.startswith("def _dev_zeros") or line.startswith("def _dev_copy_rows")
        if pat.search(line) and not fallback and "gloo host staging" not in line and "gloo CPU tests" not in line:
            bad.append((i, line.strip()))
    assert not bad, bad


def test_pds_lookahead_priming_rule():
    """The look-ahead PDS step reuses its march only for exactly the state arrays it left, unmodified
    (an in-place edit of the state between steps must re-prime)."""
    import torch

    import pyxu_amd.opt.solver as pxs

    s = object.__new__(pxs.PD3O)
    a, b, c, d = (torch.zeros(3) for _ in range(4))
    s._la = None
    assert not s._primed(a, b, c)
    s._la = (s._la_key(a, b, c), d)
    assert s._primed(a, b, c)
    assert not s._primed(a, b, d)  # a replaced z re-primes
    assert not s._primed(a, b)  # a different state layout
    b.add_(1.0)  # the user edits u in place (MANUAL mode): its version counter moves
    assert not s._primed(a, b, c)
    s._la = (s._la_key(a, b, c), d)
    assert s._primed(a, b, c)
    s.reset_lookahead()
    assert not s._primed(a, b, c)
    cv = object.__new__(pxs.CondatVu)
    cv._la = (cv._la_key(a, b), None)
    assert cv._primed(a, b) and not cv._primed(b, a)


def test_directional_lipschitz_chain_rule():
    """The directional operators' Lipschitz constant is the reference's Sum * DiagonalOp * diff chain
    product (diff.py:2171-2173; reduce.py:103-106; base.py:236-243, 330; blocks.py:684-708).  Values
    below were printed by the reference in this container (fp64); the goldens carry the rest
    (test_gpu_directional.py::test_directional_golden)."""
    from pyxu_amd.operator.linop.diff import _Directional, _unit

    L_grad2 = float(np.sqrt(8.0))  # forward-difference Gradient on a 2-D grid
    chain = _Directional._chain_lipschitz
    # DirectionalDerivative((7, 9), order 1, (0.3, -1.2)) -> 3.8805700005813275
    w = _unit(np.array([0.3, -1.2]), np.float64)[None]
    assert abs(chain(w, 1, 2, 2, L_grad2) - 3.8805700005813275) < 1e-12
    # DirectionalDerivative((5, 6), order 1, (0, 1)): weights not allclose to 0 / 1 -> 4.000000000000001
    w = _unit(np.array([0.0, 1.0]), np.float64)[None]
    assert abs(chain(w, 1, 2, 2, L_grad2) - 4.0) < 1e-12
    # DirectionalGradient((5, 6), [(1, 0), (0, 1)]): vstack of two DiagonalOps -> 5.6568542494923815
    w = np.stack([_unit(np.array(d), np.float64) for d in ((1.0, 0.0), (0.0, 1.0))])
    assert abs(chain(w, 2, 2, 2, L_grad2) - 5.6568542494923815) < 1e-12
    # 1-D: the reference's square Sum loses the constant in the composition -> inf
    assert np.isinf(chain(np.ones((1, 1)), 1, 1, 1, 2.0))


def test_flag_wait_raises_when_stream_idle_and_seq_never_published():
    """HostFlagBuffer.wait must not spin forever on a sequence number that is never
    published (faulted or missing kernel, overwritten seq) once the stream has drained."""
    from pyxu_amd import _dev

    flags = np.zeros(4, dtype=np.uint32)
    flags[:] = 6
    _dev.wait_flags(flags, 6, 1e-4, lambda: True)  # already published: returns at once
    busy = iter([False, False, True])
    with pytest.raises(_dev.FlagWaitError):
        _dev.wait_flags(flags, 7, 1e-4, lambda: next(busy))
    # a publication that lands while the stream is still busy is accepted
    calls = {"n": 0}

    def idle():
        calls["n"] += 1
        if calls["n"] == 3:
            flags[:] = 8
        return False

    _dev.wait_flags(flags, 8, 1e-4, idle)
    assert calls["n"] >= 3


def test_stencil_fft_threshold_follows_tile_envelope():
    """the 1280-tap 2-D FFT threshold holds only for tap boxes the LDS-tiled direct kernel takes
    (both extents <= 65, <= 2048 taps); wider 2-D boxes (e.g. 5 x 101) keep 256, as do 3-D kernels."""
    from pyxu_amd.operator.linop.stencil import Stencil

    assert Stencil._default_fft_min_taps((31, 31)) == 1280
    assert Stencil._default_fft_min_taps((65, 19)) == 1280
    assert Stencil._default_fft_min_taps((5, 101)) == 256  # 505 taps: FFT, not the generic direct kernel
    assert Stencil._default_fft_min_taps((45, 46)) == 256  # 2070 taps: beyond the tap table
    assert Stencil._default_fft_min_taps((9, 9, 9)) == 256


def test_profile_hooks_wrap_m_step(monkeypatch):
    """PXA_PROFILE / PXA_DEBUG_SYNC: m_step runs inside a named range and is followed by a device
    check; with neither flag the method is left alone (and a wrapper of an earlier fit is removed)."""
    from pyxu_amd import profile

    calls = []

    class FakeSolver:
        _astate = {"idx": 3}

        def m_step(self):
            calls.append("step")

    monkeypatch.setattr(profile, "range_push", lambda n: calls.append(("push", n)))
    monkeypatch.setattr(profile, "range_pop", lambda: calls.append("pop"))
    monkeypatch.setattr(profile, "_check_device", lambda: calls.append("sync"))
    s = FakeSolver()
    monkeypatch.setenv("PXA_PROFILE", "1")
    monkeypatch.setenv("PXA_DEBUG_SYNC", "1")
    profile.instrument(s)
    profile.instrument(s)  # idempotent
    s.m_step()
    assert calls == [("push", "FakeSolver.m_step[3]"), "step", "sync", "pop"]
    monkeypatch.setenv("PXA_PROFILE", "0")
    monkeypatch.setenv("PXA_DEBUG_SYNC", "0")
    profile.instrument(s)
    calls.clear()
    s.m_step()
    assert calls == ["step"]
    assert profile._roctx().roctxRangePushA(b"x") >= 0 and profile._roctx().roctxRangePop() >= -1  # loads here


def test_lagged_stop_check_eligibility():
    """abc/solver.py _lag_plan: the lagged engine (round 6) applies only to stop_rate 1, BLOCK / MANUAL mode, no
    checkpoints / objective tracking, an OR of MaxIter and exactly one plain RelError on a logged variable, a solver
    that supports it, and iterates small enough to hold ~_LAG + 3 of (host logic only; the GPU tests pin the engine's
    results, tests/test_gpu_solver_lag.py)."""
    import pyxu_amd.distributed as pd

    class _S(pxa.Solver):
        def _lag_supported(self):
            return True

    class _Iterate:  # the size of a float32 iterate (no allocation)
        def __init__(self, n):
            self.n = n

        def numel(self):
            return self.n

        def element_size(self):
            return 4

    def plan(crit, stop_rate=1, mode=pxa.Mode.BLOCK, wb=None, track=False, n=16, supported=True):
        s = _S(show_progress=False, stop_rate=stop_rate, log_var=("x",), _internal=False)
        s._astate.update(stop_crit=crit, mode=mode, wb_rate=wb, track_objective=track)
        s._mstate["x"] = _Iterate(n)
        if not supported:
            s._lag_supported = lambda: False
        return s._lag_plan()

    ok = plan(pxst.MaxIter(10) | pxst.RelError(eps=1e-3))
    assert ok is not None and type(ok[0]) is pxst.RelError and len(ok[1]) == 1
    assert plan(pxst.RelError(eps=1e-3)) is not None
    assert plan(pxst.MaxIter(3) | (pxst.RelError(eps=1e-3) | pxst.MaxIter(5)))[1][1]._n == 5
    assert plan(pxst.MaxIter(10) | pxst.RelError(eps=1e-3), mode=pxa.Mode.MANUAL) is not None
    for bad in (dict(stop_rate=2), dict(mode=pxa.Mode.ASYNC), dict(wb=1), dict(track=True), dict(supported=False)):
        assert plan(pxst.MaxIter(10) | pxst.RelError(eps=1e-3), **bad) is None, bad
    assert plan(pxst.MaxIter(10) & pxst.RelError(eps=1e-3)) is None  # AND: the decision is not RelError's alone
    assert plan(pxst.AbsError(eps=1e-3) | pxst.RelError(eps=1e-3)) is None
    assert plan(pxst.RelError(eps=1e-3) | pxst.RelError(eps=1e-2)) is None
    assert plan(pxst.RelError(eps=1e-3, var="y")) is None  # not a logged variable
    assert plan(pxst.RelError(eps=1e-3, norm=1)) is None
    assert plan(pxst.RelError(eps=1e-3, f=lambda v: v)) is None
    assert plan(pd.ShardedRelError(eps=1e-3)) is None  # its all-reduce per check is a collective: not lagged
    big = int(_S._LAG_MAX_BYTES // 4 // (_S._LAG + 3)) + 1
    assert plan(pxst.RelError(eps=1e-3), n=big) is None  # the held iterates would not fit the budget
