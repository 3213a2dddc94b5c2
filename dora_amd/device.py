"""HBM plumbing over the C ABI: streams, events, device buffers, device-resident Arrow arrays."""
from __future__ import annotations

import ctypes
from ctypes import byref, c_float, c_int, c_uint64, c_void_p

from . import _lib
from ._lib import call
from .arrow_c import ArrowArray, ArrowSchema, CArray, release_array, release_schema


def device_count() -> int:
    n = c_int(0)
    call("dora_gpu_device_count", byref(n))
    return n.value


def set_device(ordinal: int):
    call("dora_gpu_set_device", ordinal)


class Stream:
    def __init__(self):
        h = c_void_p()
        call("dora_gpu_stream_create", byref(h))
        self.handle = h.value

    def sync(self):
        call("dora_gpu_stream_sync", self.handle)

    def close(self):
        if self.handle:
            call("dora_gpu_stream_destroy", self.handle)
            self.handle = None


class Event:
    def __init__(self):
        h = c_void_p()
        call("dora_gpu_event_create", byref(h))
        self.handle = h.value

    def record(self, stream: Stream | None = None):
        call("dora_gpu_event_record", self.handle, stream.handle if stream else None)

    def sync(self):
        call("dora_gpu_event_sync", self.handle)

    def elapsed_ms(self, later: "Event") -> float:
        ms = c_float()
        call("dora_gpu_event_elapsed_ms", self.handle, later.handle, byref(ms))
        return ms.value

    def close(self):
        if self.handle:
            call("dora_gpu_event_destroy", self.handle)
            self.handle = None


class DeviceBuffer:
    """A plain hipMalloc allocation."""

    def __init__(self, nbytes: int):
        p = c_void_p()
        call("dora_gpu_malloc", byref(p), nbytes)
        self.ptr, self.size = p.value, nbytes

    @classmethod
    def from_bytes(cls, data: bytes, stream: Stream | None = None) -> "DeviceBuffer":
        b = cls(len(data))
        if data:
            src = ctypes.create_string_buffer(bytes(data), len(data))
            call("dora_gpu_memcpy_async", b.ptr, src, len(data), stream.handle if stream else None)
            call("dora_gpu_stream_sync", stream.handle if stream else None)
        return b

    def to_bytes(self, n: int | None = None, offset: int = 0, stream: Stream | None = None) -> bytes:
        n = self.size - offset if n is None else n
        out = ctypes.create_string_buffer(max(n, 1))
        if n:
            call("dora_gpu_memcpy_async", out, self.ptr + offset, n,
                 stream.handle if stream else None)
            call("dora_gpu_stream_sync", stream.handle if stream else None)
        return out.raw[:n]

    def fill(self, value: int, stream: Stream | None = None):
        call("dora_gpu_memset_async", self.ptr, value, self.size, stream.handle if stream else None)

    def free(self):
        if self.ptr:
            call("dora_gpu_free", self.ptr)
            self.ptr = None

    close = free


def csum64(ptr: int, n: int, stream: Stream | None = None) -> int:
    out = c_uint64()
    call("dora_gpu_csum64_sync", ptr, n, stream.handle if stream else None, byref(out))
    return out.value


def aql_dispatch_counts(device: int = 0) -> dict:
    """Raw AQL packets this process dispatched on `device`, per pack kernel."""
    lib = _lib.load()
    c = (c_uint64 * 16)()
    n = ctypes.c_size_t()
    call("dora_gpu_aql_dispatch_counts", device, c, 16, byref(n))
    return {lib.dora_gpu_aql_kernel_name(k).decode(): c[k] for k in range(n.value)}


def set_keep_awake(period_us: float = 25.0) -> None:
    """While this process sends device samples, keep the GPU's command processor from idling:
    an empty AQL packet whenever nothing was dispatched for `period_us` (0: off;
    dora_gpu_set_keep_awake).  Process-wide."""
    call("dora_gpu_set_keep_awake", float(period_us))


def aql_cp_signalled(device: int = 0) -> int:
    """Packs whose fill the command processor signalled (aql.cpp aql_cp_candidate)."""
    a = c_uint64()
    call("dora_gpu_aql_cp_signalled", device, byref(a))
    return a.value


def aql_batch_stats(device: int = 0) -> dict:
    """Batch packs dispatched, the sends they carried, sends that waited for a queue."""
    a, b, c = c_uint64(), c_uint64(), c_uint64()
    call("dora_gpu_aql_batch_stats", device, byref(a), byref(b), byref(c))
    return {"batches": a.value, "batched_msgs": b.value, "backlogged": c.value}


def aql_hold(device: int, hold: bool):
    """Test tool: hold batchable AQL sends in the backlog / release them as batch packs."""
    call("dora_gpu_test_aql_hold", device, int(hold))


def fill_splitmix(ptr: int, n: int, seed: int, stream: Stream | None = None):
    call("dora_gpu_fill_splitmix", ptr, n, seed, stream.handle if stream else None)


class DeviceArray:
    """An Arrow array whose buffers live in HBM (device ArrowArray + ArrowSchema, owned)."""

    def __init__(self, array: ArrowArray, arrow_type, keepalive=None):
        self.array, self.type = array, arrow_type
        self._keepalive = keepalive
        self._schema = None  # exported once, lent to every send (borrowed by the C ABI)

    @classmethod
    def from_pyarrow(cls, arr) -> "DeviceArray":
        with CArray.from_pyarrow(arr) as host:
            dev = ArrowArray()
            call("dora_gpu_array_upload", byref(host.array), byref(host.schema), byref(dev))
        return cls(dev, arr.type)

    def export_schema(self) -> ArrowSchema:
        """A freshly exported ArrowSchema of this array's type (the caller owns it)."""
        s = ArrowSchema()
        self.type._export_to_c(ctypes.addressof(s))
        return s

    def borrowed_schema(self) -> ArrowSchema:
        """This array's ArrowSchema, exported once and kept until close(): for calls that only
        borrow it (dora_node_send_output, plans).  A nested type's export costs ~4 us, more
        than the rest of a Python send."""
        if self._schema is None:
            self._schema = self.export_schema()
        return self._schema

    def send_addrs(self):
        """(ArrowArray address, borrowed ArrowSchema address) for the native send path."""
        addrs = self.__dict__.get("_addrs")
        if addrs is None:
            addrs = self._addrs = (ctypes.addressof(self.array),
                                   ctypes.addressof(self.borrowed_schema()))
        return addrs

    def to_pyarrow(self):
        """Download to host memory and import into pyarrow (F12: pyarrow cannot import ROCm)."""
        import pyarrow as pa
        host = ArrowArray()
        s = self.export_schema()
        try:
            call("dora_gpu_array_download", byref(self.array), byref(s), byref(host))
        except Exception:
            release_schema(s)
            raise
        return pa.Array._import_from_c(ctypes.addressof(host), ctypes.addressof(s))

    @property
    def length(self) -> int:
        return self.array.length

    # DLPack (kDLROCM): zero-copy hand-off of fixed-width device samples to torch & co.
    def __dlpack__(self, stream=None, **kwargs):
        from .dlpack import to_dlpack_capsule, values_view
        ptr, n, fmt = values_view(self)
        return to_dlpack_capsule(ptr, n, fmt, self.device_id, self)

    def __dlpack_device__(self):
        from .dlpack import kDLROCM
        return (kDLROCM, self.device_id)

    @property
    def device_id(self) -> int:
        return getattr(self, "_device_id", 0)

    def close(self):
        release_array(self.array)
        if self._schema is not None:
            release_schema(self._schema)
            self._schema = None
        self.__dict__.pop("_addrs", None)
        self._keepalive = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


__all__ = ["Stream", "Event", "DeviceBuffer", "DeviceArray", "device_count", "set_device",
           "csum64", "fill_splitmix", "_lib"]
