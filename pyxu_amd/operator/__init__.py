"""Operators (mirrors reference ``pyxu.operator``): the hot-path subset."""
from pyxu_amd.operator.blocks import *  # noqa: F401,F403
from pyxu_amd.operator.func import *  # noqa: F401,F403
from pyxu_amd.operator.interop import *  # noqa: F401,F403
from pyxu_amd.operator.linop import *  # noqa: F401,F403
