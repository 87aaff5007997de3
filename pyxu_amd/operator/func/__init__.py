from pyxu_amd.operator.func.indicator import *  # noqa: F401,F403
from pyxu_amd.operator.func.loss import *  # noqa: F401,F403
from pyxu_amd.operator.func.norm import *  # noqa: F401,F403
from pyxu_amd.operator.linop.base import NullFunc  # noqa: F401
