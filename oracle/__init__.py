"""
oracle — CPU restatement of Pyxu's proximal-splitting hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker / the timed CPU
baseline.  The product (``pyxu_amd``) never imports it and never falls back to it.

Parity status: pinned.  ``tests/golden/*.npz`` hold vectors produced by importing the upstream
reference snapshot (``/root/reference/src``, via ``oracle/refshim``) and running its own NumPy
code path; ``tests/test_oracle_golden.py`` checks this restatement against every one of them and
against the reference's own known-answer tests (``src/pyxu_tests/operator/func/test_norm.py``,
``src/pyxu_tests/operator/linop/test_stencil.py`` / ``scipy.ndimage``).
"""
from .pyxu_np import *  # noqa: F401,F403
