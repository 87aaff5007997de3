from pyxu_amd.operator.linop.base import *  # noqa: F401,F403
from pyxu_amd.operator.linop.diff import *  # noqa: F401,F403
from pyxu_amd.operator.linop.fft import *  # noqa: F401,F403
from pyxu_amd.operator.linop.filter import *  # noqa: F401,F403
from pyxu_amd.operator.linop.stencil import *  # noqa: F401,F403
from pyxu_amd.operator.linop.pad import *  # noqa: F401,F403
from pyxu_amd.operator.linop.select import *  # noqa: F401,F403
