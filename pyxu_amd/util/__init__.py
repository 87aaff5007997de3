"""Array-module helpers (mirrors reference ``pyxu.util.array_module``, src/pyxu/util/array_module.py)."""
from .array_module import *  # noqa: F401,F403
