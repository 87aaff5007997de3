"""Solvers (mirrors reference ``pyxu.opt.solver``)."""
from pyxu_amd.opt.solver.cg import *  # noqa: F401,F403
from pyxu_amd.opt.solver.pds import *  # noqa: F401,F403
from pyxu_amd.opt.solver.pgd import *  # noqa: F401,F403
