from pyxu_amd.operator.interop.source import from_source  # noqa: F401
