"""
The RCCL path of pyxu_amd.distributed, executed on the one GPU of a test box (VERDICT r05 Next #7).

A world-size-1 ``nccl`` process group (RCCL) with ``PXA_DIST_COLLECTIVES=always``: every collective the
sharded path issues -- ShardedRelError's all-reduce of the row statistics, gather_slabs' all-gather,
RowShardedLinOp's adjoint all-reduce inside ADMM / CG -- runs as a real RCCL call on device buffers
instead of short-circuiting at one rank.  A sum over one rank is the identity, so the results must equal
the unsharded ones bit for bit (reference: operator/blocks.py:838-860 has no device
collective at all, its Dask path chunks arrays on the host).
"""
import os

import numpy as np
import pytest

from test_distributed_cpu import spawn

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs an MI355X", allow_module_level=True)


def test_rccl_world1_sharded_paths_match_unsharded():
    old = os.environ.get("PXA_DIST_COLLECTIVES")
    os.environ["PXA_DIST_COLLECTIVES"] = "always"
    try:
        res = spawn("gpu_rccl_world1", world=1, _backend="nccl", B=3, sh=(40, 56), iters=300, eps=1e-2,
                    M=96, N=256, n_iter=10)[0]
    finally:
        if old is None:
            os.environ.pop("PXA_DIST_COLLECTIVES", None)
        else:
            os.environ["PXA_DIST_COLLECTIVES"] = old
    assert res["rccl_libs"], "librccl is not mapped: the nccl backend did not load RCCL"
    # every stop check of the sharded PGD all-reduced its device statistics through RCCL
    pgd_calls = res["pgd_collectives"]
    assert pgd_calls and all(c == ("all_reduce", True) for c in pgd_calls)
    assert res["pgd_it"] == res["pgd_it_ref"] < 300
    np.testing.assert_array_equal(res["pgd_x"], res["pgd_x_ref"])
    assert res["gathered_is_cuda"]
    np.testing.assert_array_equal(res["gathered"].reshape(-1), res["pgd_x"].reshape(-1))
    # RowShardedLinOp.adjoint: local GEMV + RCCL all-reduce == the unsharded dense adjoint, bit for bit
    assert res["adj_collectives"] == [("all_reduce", True)]
    np.testing.assert_array_equal(res["adj_sharded"], res["adj_ref"])
    # ADMM through the sharded normal operator (one RCCL all-reduce per CG step); d p is added after the
    # all-reduce instead of inside the kernel, hence the norm-wise fp32 tolerance
    assert res["admm_collectives"] > 10
    d = np.linalg.norm(res["admm_x"] - res["admm_x_ref"]) / np.linalg.norm(res["admm_x_ref"])
    assert d <= 1e-5, d
