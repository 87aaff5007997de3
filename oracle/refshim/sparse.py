"""Placeholder for the absent `sparse` package (never instantiated on the NumPy path)."""


class SparseArray:
    pass
