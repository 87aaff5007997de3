"""Make the read-only upstream Pyxu snapshot importable (golden generation only; see README.md)."""
import importlib.metadata as _md
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"

if _HERE not in sys.path:
    sys.path.insert(0, _HERE)
if REF_SRC not in sys.path:
    sys.path.insert(0, REF_SRC)

_version = _md.version


def _patched_version(name):
    # pyxu/__init__.py asks for its own distribution version; the snapshot is not pip-installed.
    return "0+reference-snapshot" if name == "pyxu" else _version(name)


_md.version = _patched_version
