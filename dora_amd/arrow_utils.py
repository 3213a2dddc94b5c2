"""`dora_node_api::arrow_utils` on the device (apis/rust/node/src/node/arrow_utils.rs:4-71).

    required_data_size(array) -> int
    copy_array_into_sample(target, array, stream=None) -> ArrowTypeInfo

`array` is a `DeviceArray` (buffers in HBM: the pack is one HIP kernel) or a host
`pyarrow.Array` (the pack is a DMA of each buffer into the device sample).  `target` is any
object with `.ptr` and `.size` addressing device memory (a `DeviceBuffer`, a `DataSample`).
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_size_t, c_uint8, c_uint64, c_void_p

from ._lib import ARROW_DEVICE_CPU, ARROW_DEVICE_ROCM, call, load
from .arrow_c import CArray, release_schema
from .device import DeviceArray
from .type_info import ArrowTypeInfo, decode


class Plan:
    """A planned pack: segment table + ArrowTypeInfo, borrowed array kept alive."""

    def __init__(self, handle: int, keep):
        self.handle = handle
        self._keep = keep
        self._lib = load()

    @classmethod
    def of(cls, array, compact: bool = False) -> "Plan":
        """Reference layout (`copy_array_into_sample`), or with `compact=True` the compacting
        plan (slices reduced to their own bytes, offset 0 everywhere)."""
        h = c_void_p()
        fn = "dora_gpu_plan_compact" if compact else "dora_gpu_plan"
        if isinstance(array, DeviceArray):
            s = array.export_schema()
            try:
                call(fn, byref(array.array), byref(s), ARROW_DEVICE_ROCM, byref(h))
            finally:
                release_schema(s)
            return cls(h.value, array)
        c = CArray.from_pyarrow(array)
        try:
            call(fn, byref(c.array), byref(c.schema), ARROW_DEVICE_CPU, byref(h))
        except Exception:
            c.close()
            raise
        return cls(h.value, c)

    @classmethod
    def of_bytes(cls, ptr: int, n: int, on_device: bool) -> "Plan":
        h = c_void_p()
        call("dora_gpu_plan_bytes", ptr, n, ARROW_DEVICE_ROCM if on_device else ARROW_DEVICE_CPU,
             byref(h))
        return cls(h.value, None)

    @property
    def size(self) -> int:
        return self._lib.dora_gpu_plan_size(self.handle)

    def segments(self):
        out = []
        for i in range(self._lib.dora_gpu_plan_num_segments(self.handle)):
            src, off, n = c_void_p(), c_uint64(), c_uint64()
            call("dora_gpu_plan_segment", self.handle, i, byref(src), byref(off), byref(n))
            out.append((src.value, off.value, n.value))
        return out

    def type_info_bytes(self) -> bytes:
        n = c_size_t()
        call("dora_gpu_plan_type_info", self.handle, None, 0, byref(n))
        buf = (c_uint8 * max(n.value, 1))()
        call("dora_gpu_plan_type_info", self.handle, buf, n.value, byref(n))
        return bytes(buf[:n.value])

    def type_info(self) -> ArrowTypeInfo:
        return decode(self.type_info_bytes())

    def pack(self, dst_ptr: int, dst_len: int, stream=None):
        call("dora_gpu_pack", self.handle, dst_ptr, dst_len, stream.handle if stream else None)

    def close(self):
        if self.handle:
            self._lib.dora_gpu_plan_free(self.handle)
            self.handle = None
        if isinstance(self._keep, CArray):
            self._keep.close()
        self._keep = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def required_data_size(array) -> int:
    """arrow_utils.rs:4-8"""
    with Plan.of(array) as p:
        return p.size


def copy_array_into_sample(target, array, stream=None) -> ArrowTypeInfo:
    """arrow_utils.rs:23-26: pack `array` into the device sample `target`; returns the type
    info.  Asynchronous on `stream`; the source must stay alive until the stream is synced
    (this call syncs when no stream is given)."""
    with Plan.of(array) as p:
        p.pack(target.ptr, target.size, stream)
        info = p.type_info()
        if stream is None:
            call("dora_gpu_stream_sync", None)
        else:
            stream.sync()
    return info


def sample_to_device_array(sample_ptr: int, sample_len: int, type_info: ArrowTypeInfo,
                           keepalive=None) -> DeviceArray:
    """`RawData::into_arrow_array` (event_stream/event.rs:35-54): zero-copy view of a device
    sample as a device Arrow array."""
    import pyarrow as pa

    from .arrow_c import ArrowArray, ArrowSchema
    raw = type_info.raw
    buf = (c_uint8 * max(len(raw), 1)).from_buffer_copy(raw or b"\0")
    a, s = ArrowArray(), ArrowSchema()
    call("dora_gpu_sample_import", sample_ptr, sample_len, buf, len(raw), byref(a), byref(s))
    t = pa.DataType._import_from_c(ctypes.addressof(s))
    return DeviceArray(a, t, keepalive)
