"""Shared case logic of the directional / Gaussian-derivative / Jacobian goldens
(tests/golden/make_goldens.py gen_directional): rebuild a case's directions, its pyxu_amd operator and
its oracle (oracle/pyxu_np.py) apply / adjoint from the recorded constructor kwargs."""
import json

import numpy as np

import oracle as orc


def case(g):
    return str(g["kind"]), json.loads(str(g["kwargs"]))


def dir_arrays(kw, dt):
    """The direction vectors of a case (make_goldens._dir_arrays): constant, or scaled per pixel."""
    sh = tuple(kw["arg_shape"])
    out = []
    for d in kw["dirs"]:
        v = np.array(d, dtype=dt)
        if kw["varying"]:
            scale = np.linspace(0.5, 2.0, int(np.prod(sh))).reshape(sh).astype(dt)
            v = (v.reshape((-1,) + (1,) * len(sh)) * scale[None]).astype(dt)
        out.append(v)
    return out


def _gd(kw):
    return {k: (tuple(v) if isinstance(v, list) else v) for k, v in kw.items() if k in ("sigma", "truncate", "sampling")}


def make_op(mod, kind, kw, dt):
    """The case's operator from `mod` (pyxu_amd.operator)."""
    sh = tuple(kw["arg_shape"])
    gd = _gd(kw)
    if kind == "jacobian":
        d = kw.get("directions")
        return mod.Jacobian(arg_shape=sh, n_channels=kw["n_channels"], directions=tuple(d) if d else None)
    if kind == "gradient_gd":
        return mod.Gradient(arg_shape=sh, diff_method="gd", **gd)
    if kind == "hessian_gd":
        return mod.Hessian(arg_shape=sh, diff_method="gd", **gd)
    if kind == "laplacian_gd":
        return mod.Laplacian(arg_shape=sh, diff_method="gd", **gd)
    if kind == "divergence_gd":
        return mod.Divergence(arg_shape=sh, diff_method="gd", **gd)
    dirs = dir_arrays(kw, dt)
    method = kw.get("diff_method", "gd" if kind == "dirhess" else "fd")
    if kind == "dirderiv":
        d = dirs[0] if len(dirs) == 1 else tuple(dirs)
        return mod.DirectionalDerivative(arg_shape=sh, order=kw["order"], directions=d, diff_method=method, **gd)
    if kind == "dirgrad":
        return mod.DirectionalGradient(arg_shape=sh, directions=dirs, diff_method=method, **gd)
    if kind == "dirlap":
        return mod.DirectionalLaplacian(arg_shape=sh, directions=dirs, weights=kw["weights"], diff_method=method, **gd)
    return mod.DirectionalHessian(arg_shape=sh, directions=dirs, diff_method=method, **gd)


def oracle_fns(kind, kw, dt):
    """(apply, adjoint) of the case restated on the oracle (NumPy, `dt` precision)."""
    sh = tuple(kw["arg_shape"])
    N = int(np.prod(sh))
    gd = _gd(kw)
    if kind == "jacobian":
        d = kw.get("directions")
        comps = [orc.gradient_kernels(sh, a, dtype=dt) for a in (d if d else range(len(sh)))]
        C, K = kw["n_channels"], len(comps)

        def ap(x):
            xs = x.reshape(*x.shape[:-1], C, N)
            return orc.stack_apply(xs, sh, comps).reshape(*x.shape[:-1], C * K * N)

        def ad(z):
            zs = z.reshape(*z.shape[:-1], C, K * N)
            return orc.stack_adjoint(zs, sh, comps).reshape(*z.shape[:-1], C * N)

        return ap, ad
    if kind == "gradient_gd":
        comps = orc.gd_gradient_comps(sh, dt, **gd)
        return (lambda x: orc.stack_apply(x, sh, comps)), (lambda z: orc.stack_adjoint(z, sh, comps))
    if kind == "hessian_gd":
        comps = orc.gd_hessian_comps(sh, dt, **gd)
        return (lambda x: orc.stack_apply(x, sh, comps)), (lambda z: orc.stack_adjoint(z, sh, comps))
    if kind == "laplacian_gd":
        comps = orc.gd_hessian_comps(sh, dt, [[i, i] for i in range(len(sh))], **gd)
        w = np.ones((1, len(sh)), dtype=dt)
        return ((lambda x: orc.contract_apply(w, orc.stack_apply(x, sh, comps), N)),
                (lambda z: orc.stack_adjoint(orc.contract_adjoint(w, z, N, len(sh)), sh, comps)))
    if kind == "divergence_gd":
        comps = orc.gd_gradient_comps(sh, dt, **gd)
        K = len(comps)

        def ap(z):
            out = 0
            for j, (k, c) in enumerate(comps):
                out = out + orc.stencil_apply(z[..., j * N:(j + 1) * N], sh, k, c)
            return out

        return ap, (lambda x: np.concatenate([orc.stencil_adjoint(x, sh, k, c) for k, c in comps], axis=-1))
    dirs = dir_arrays(kw, dt)
    method = kw.get("diff_method", "gd" if kind == "dirhess" else "fd")
    units = [orc.unit_direction(d, dt) for d in dirs]
    if kind == "dirderiv" and kw["order"] == 1:
        comps = orc.gd_gradient_comps(sh, dt, **gd) if method == "gd" else \
            [orc.gradient_kernels(sh, a, dtype=dt) for a in range(len(sh))]
        w = units[0][None]
    else:
        comps = orc.gd_hessian_comps(sh, dt, **gd) if method == "gd" else orc.fd_hessian_comps(sh, dt)
        if kind == "dirgrad":
            comps = orc.gd_gradient_comps(sh, dt, **gd) if method == "gd" else \
                [orc.gradient_kernels(sh, a, dtype=dt) for a in range(len(sh))]
            w = np.stack(units)
        elif kind == "dirderiv":
            w = orc.outer_triu(units[0], units[-1])[None]
        elif kind == "dirlap":
            w = np.concatenate([wt * orc.outer_triu(u, u) for wt, u in zip(kw["weights"], units)], axis=0)[None]
        else:  # dirhess
            w = np.stack([orc.outer_triu(units[i], units[j]) for i in range(len(units)) for j in range(i, len(units))])
    K = len(comps)
    return ((lambda x: orc.contract_apply(w, orc.stack_apply(x, sh, comps), N)),
            (lambda z: orc.stack_adjoint(orc.contract_adjoint(w, z, N, K), sh, comps)))
