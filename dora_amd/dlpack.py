"""DLPack export of device-resident Arrow arrays.

pyarrow 25 cannot import ROCm device arrays, so Python nodes reach received HBM samples through
DLPack instead: `torch.from_dlpack(device_array)` (or any DLPack consumer) gets a zero-copy
`kDLROCM` tensor over the values buffer of a fixed-width array.  The tensor keeps the
DeviceArray — and therefore the input's drop token — alive until it is freed.
"""
from __future__ import annotations

import ctypes

kDLROCM = 10
_DL_INT, _DL_UINT, _DL_FLOAT, _DL_BOOL = 0, 1, 2, 6

# Arrow C format -> (DLPack type code, bits)
_DTYPES = {"c": (_DL_INT, 8), "C": (_DL_UINT, 8), "s": (_DL_INT, 16), "S": (_DL_UINT, 16),
           "i": (_DL_INT, 32), "I": (_DL_UINT, 32), "l": (_DL_INT, 64), "L": (_DL_UINT, 64),
           "e": (_DL_FLOAT, 16), "f": (_DL_FLOAT, 32), "g": (_DL_FLOAT, 64)}


class DLDevice(ctypes.Structure):
    _fields_ = [("device_type", ctypes.c_int32), ("device_id", ctypes.c_int32)]


class DLDataType(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint8), ("bits", ctypes.c_uint8), ("lanes", ctypes.c_uint16)]


class DLTensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("device", DLDevice), ("ndim", ctypes.c_int32),
                ("dtype", DLDataType), ("shape", ctypes.POINTER(ctypes.c_int64)),
                ("strides", ctypes.POINTER(ctypes.c_int64)), ("byte_offset", ctypes.c_uint64)]


class DLManagedTensor(ctypes.Structure):
    pass


_DELETER = ctypes.CFUNCTYPE(None, ctypes.POINTER(DLManagedTensor))
DLManagedTensor._fields_ = [("dl_tensor", DLTensor), ("manager_ctx", ctypes.c_void_p),
                            ("deleter", _DELETER)]

_live = {}  # id(managed) -> (managed, shape, owner): keeps the exported memory alive


@_DELETER
def _delete(p):
    _live.pop(ctypes.addressof(p.contents), None)


_CAPSULE_DESTRUCTOR = ctypes.CFUNCTYPE(None, ctypes.py_object)
_PyCapsule_New = ctypes.pythonapi.PyCapsule_New
_PyCapsule_New.restype = ctypes.py_object
_PyCapsule_New.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]


def to_dlpack_capsule(ptr: int, length: int, fmt: str, device_id: int, owner):
    """A 'dltensor' PyCapsule over `length` elements of Arrow format `fmt` at device `ptr`."""
    if fmt not in _DTYPES:
        raise TypeError(f"DLPack export supports fixed-width numeric arrays, not {fmt!r}")
    code, bits = _DTYPES[fmt]
    shape = (ctypes.c_int64 * 1)(length)
    m = DLManagedTensor()
    m.dl_tensor.data = ptr
    m.dl_tensor.device = DLDevice(kDLROCM, device_id)
    m.dl_tensor.ndim = 1
    m.dl_tensor.dtype = DLDataType(code, bits, 1)
    m.dl_tensor.shape = shape
    m.dl_tensor.strides = None
    m.dl_tensor.byte_offset = 0
    m.manager_ctx = None
    m.deleter = _delete
    _live[ctypes.addressof(m)] = (m, shape, owner)
    # the consumer renames the capsule to "used_dltensor" and calls the deleter itself
    return _PyCapsule_New(ctypes.addressof(m), b"dltensor", None)


def values_view(device_array):
    """(pointer, length, format) of the values buffer of a fixed-width DeviceArray."""
    import pyarrow as pa
    t = device_array.type
    if pa.types.is_dictionary(t) or not (pa.types.is_integer(t) or pa.types.is_floating(t)):
        raise TypeError(f"DLPack export needs a fixed-width numeric array, got {t}")
    fmt = {pa.int8(): "c", pa.uint8(): "C", pa.int16(): "s", pa.uint16(): "S",
           pa.int32(): "i", pa.uint32(): "I", pa.int64(): "l", pa.uint64(): "L",
           pa.float16(): "e", pa.float32(): "f", pa.float64(): "g"}[t]
    a = device_array.array
    width = _DTYPES[fmt][1] // 8
    if a.n_buffers < 2 or not a.buffers[1]:
        ptr = 0
    else:
        ptr = a.buffers[1] + a.offset * width
    return ptr, a.length, fmt
