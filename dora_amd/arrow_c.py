"""Arrow C Data Interface structs (public Arrow ABI) and pyarrow <-> C helpers."""
from __future__ import annotations

import ctypes


class ArrowSchema(ctypes.Structure):
    pass


ArrowSchema._fields_ = [
    ("format", ctypes.c_char_p),
    ("name", ctypes.c_char_p),
    ("metadata", ctypes.c_void_p),
    ("flags", ctypes.c_int64),
    ("n_children", ctypes.c_int64),
    ("children", ctypes.POINTER(ctypes.POINTER(ArrowSchema))),
    ("dictionary", ctypes.POINTER(ArrowSchema)),
    ("release", ctypes.c_void_p),
    ("private_data", ctypes.c_void_p),
]


class ArrowArray(ctypes.Structure):
    pass


ArrowArray._fields_ = [
    ("length", ctypes.c_int64),
    ("null_count", ctypes.c_int64),
    ("offset", ctypes.c_int64),
    ("n_buffers", ctypes.c_int64),
    ("n_children", ctypes.c_int64),
    ("buffers", ctypes.POINTER(ctypes.c_void_p)),
    ("children", ctypes.POINTER(ctypes.POINTER(ArrowArray))),
    ("dictionary", ctypes.POINTER(ArrowArray)),
    ("release", ctypes.c_void_p),
    ("private_data", ctypes.c_void_p),
]

_REL_S = ctypes.CFUNCTYPE(None, ctypes.POINTER(ArrowSchema))
_REL_A = ctypes.CFUNCTYPE(None, ctypes.POINTER(ArrowArray))


def release_schema(s: ArrowSchema):
    if s.release:
        _REL_S(s.release)(ctypes.byref(s))


def release_array(a: ArrowArray):
    if a.release:
        _REL_A(a.release)(ctypes.byref(a))


class CArray:
    """An exported (array, schema) pair in C structs; releases both on close()."""

    def __init__(self):
        self.array = ArrowArray()
        self.schema = ArrowSchema()

    @classmethod
    def from_pyarrow(cls, arr) -> "CArray":
        c = cls()
        arr._export_to_c(ctypes.addressof(c.array), ctypes.addressof(c.schema))
        return c

    def to_pyarrow(self):
        """Move both structs into a pyarrow.Array (host buffers only)."""
        import pyarrow as pa
        return pa.Array._import_from_c(ctypes.addressof(self.array), ctypes.addressof(self.schema))

    def close(self):
        release_array(self.array)
        release_schema(self.schema)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
