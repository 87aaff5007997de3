"""Abstract base classes (mirrors reference ``pyxu.abc``)."""
from pyxu_amd.abc.operator import *  # noqa: F401,F403
from pyxu_amd.abc.solver import Mode, Solver, StoppingCriterion  # noqa: F401
from pyxu_amd.abc.operator import _core_operators  # noqa: F401
