"""`ArrowTypeInfo` / `BufferOffset` (libraries/message/src/metadata.rs:51-59,140-143) decoded
from the C ABI wire format (include/dora_gpu.h, dora_gpu_plan_type_info)."""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional

FLAG_DICTIONARY_ORDERED = 1
FLAG_NULLABLE = 2
FLAG_MAP_KEYS_SORTED = 4


@dataclass
class SchemaNode:
    format: str
    name: str
    flags: int
    metadata: Optional[bytes]
    children: List["SchemaNode"]
    dictionary: Optional["SchemaNode"]

    def signature(self) -> str:
        """Canonical type signature (same definition as the C++ `schema_sig`)."""
        if self.dictionary is not None:
            ordered = ",ordered" if self.flags & FLAG_DICTIONARY_ORDERED else ""
            return f"dict<{self.format},{self.dictionary.signature()}{ordered}>"
        out = self.format
        if self.format == "+m" and self.flags & FLAG_MAP_KEYS_SORTED:
            out += "s"
        if self.children:
            parts = [f"{c.name}:{'?' if c.flags & FLAG_NULLABLE else '!'}{c.signature()}"
                     for c in self.children]
            out += "[" + ",".join(parts) + "]"
        return out


@dataclass
class BufferOffset:
    offset: int
    len: int


@dataclass
class ArrowTypeInfo:
    data_type: str                     # canonical signature of the DataType
    len: int
    null_count: int
    validity: Optional[bytes]
    offset: int
    buffer_offsets: List[BufferOffset] = field(default_factory=list)
    child_data: List["ArrowTypeInfo"] = field(default_factory=list)
    schema: Optional[SchemaNode] = None
    raw: bytes = b""                   # the serialized form this was decoded from
    # tag 2 (node sends of device arrays): the bitmap is sample[off, off + len) of the slot's
    # validity tail; dora_event_type_info hands receivers the inline form (validity bytes)
    validity_in_sample: Optional[tuple] = None

    @staticmethod
    def byte_array(data_len: int) -> "ArrowTypeInfo":   # metadata.rs:74-87
        return ArrowTypeInfo("C", data_len, 0, None, 0, [BufferOffset(0, data_len)], [],
                             SchemaNode("C", "", 0, None, [], None))

    def to_json(self):
        return {
            "data_type": self.data_type, "len": self.len, "null_count": self.null_count,
            "validity": None if self.validity is None else self.validity.hex(),
            "offset": self.offset,
            "buffer_offsets": [[b.offset, b.len] for b in self.buffer_offsets],
            "child_data": [c.to_json() for c in self.child_data],
        }

    def arrow_type(self):
        """The DataType as a pyarrow.DataType."""
        import ctypes

        import pyarrow as pa

        from . import _lib
        from .arrow_c import ArrowSchema
        s = ArrowSchema()
        buf = (ctypes.c_uint8 * len(self.raw)).from_buffer_copy(self.raw)
        _lib.call("dora_gpu_type_info_schema", buf, len(self.raw), ctypes.byref(s))
        return pa.DataType._import_from_c(ctypes.addressof(s))


class _Reader:
    def __init__(self, b: bytes):
        self.b, self.i = b, 0

    def take(self, n):
        if self.i + n > len(self.b):
            raise ValueError("truncated type info")
        v = self.b[self.i:self.i + n]
        self.i += n
        return v

    def u8(self):
        return self.take(1)[0]

    def u32(self):
        return struct.unpack("<I", self.take(4))[0]

    def u64(self):
        return struct.unpack("<Q", self.take(8))[0]

    def i64(self):
        return struct.unpack("<q", self.take(8))[0]

    def s(self):
        return self.take(self.u32())


def _schema(r: _Reader) -> SchemaNode:
    fmt = r.s().decode()
    name = r.s().decode()
    flags = r.i64()
    meta = r.s() if r.u8() else None
    children = [_schema(r) for _ in range(r.u32())]
    dictionary = _schema(r) if r.u8() else None
    return SchemaNode(fmt, name, flags, meta, children, dictionary)


def _type_info(r: _Reader, raw_all: bytes) -> ArrowTypeInfo:
    start = r.i
    schema = _schema(_Reader(r.s()))
    n = r.u64()
    null_count = r.u64()
    tag = r.u8()
    validity, in_sample = None, None
    if tag == 1:
        validity = r.take(r.u64())
    elif tag == 2:
        in_sample = (r.u64(), r.u64())
    elif tag != 0:
        raise ValueError(f"unknown validity tag {tag}")
    offset = r.u64()
    bufs = [BufferOffset(r.u64(), r.u64()) for _ in range(r.u32())]
    children = [_type_info(r, raw_all) for _ in range(r.u32())]
    return ArrowTypeInfo(schema.signature(), n, null_count, validity, offset, bufs, children,
                         schema, raw_all[start:r.i], in_sample)


def decode(raw: bytes) -> ArrowTypeInfo:
    r = _Reader(bytes(raw))
    ti = _type_info(r, bytes(raw))
    if r.i != len(raw):
        raise ValueError("trailing bytes after type info")
    return ti
