"""TEST INFRASTRUCTURE ONLY — part of the CPU oracle, never shipped or measured.

Reads an Arrow array through the Arrow C Data Interface exactly the way arrow-rs 53.2.0's FFI
import does (`ArrayData::from_pyarrow_bound` -> `arrow::ffi::from_ffi`), which is how a pyarrow
array reaches `copy_array_into_sample` in the reference Python node
(`apis/python/node/src/lib.rs:157-185`).  Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s cpu_baseline leg may import this module.

Restated third-party rules (arrow-rs 53.2.0 is pinned by `Cargo.lock:319-517`, not vendored):
  * buffer lengths: `ImportedArrowArray::buffer_len` (arrow/src/ffi.rs) — `(len+offset+1)*w` for
    offsets buffers, last offset value for Utf8/Binary data buffers, `ceil((len+offset)*bits/8)`
    otherwise;
  * nulls: the validity buffer is kept only when its null count is non-zero
    (`ArrayDataBuilder::build_unchecked`'s `.filter(|b| b.null_count() != 0)`).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional


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

_RELEASE_SCHEMA = ctypes.CFUNCTYPE(None, ctypes.POINTER(ArrowSchema))
_RELEASE_ARRAY = ctypes.CFUNCTYPE(None, ctypes.POINTER(ArrowArray))

FLAG_DICTIONARY_ORDERED = 1
FLAG_NULLABLE = 2
FLAG_MAP_KEYS_SORTED = 4


class Exported:
    """Owns a C-exported pyarrow array (schema + array) and releases it on close."""

    def __init__(self, arr):
        self.schema = ArrowSchema()
        self.array = ArrowArray()
        arr._export_to_c(ctypes.addressof(self.array), ctypes.addressof(self.schema))
        self._arr = arr

    def close(self):
        if self.array.release:
            _RELEASE_ARRAY(self.array.release)(ctypes.byref(self.array))
        if self.schema.release:
            _RELEASE_SCHEMA(self.schema.release)(ctypes.byref(self.schema))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# ----------------------------------------------------------------------------------------------
# Layout table: arrow-data 53.2.0 `layout()` restated.  Each entry is the list of non-null
# buffer specs: ("fixed", byte_width, alignment) | ("bitmap",) | ("var",).  Alignments are those
# of the Rust 1.76 toolchain the reference pins (`rust-toolchain.toml:2`): i128/u128 align 8.
# ----------------------------------------------------------------------------------------------
_PRIM = {
    "c": (1, 1), "C": (1, 1), "s": (2, 2), "S": (2, 2), "e": (2, 2),
    "i": (4, 4), "I": (4, 4), "f": (4, 4),
    "l": (8, 8), "L": (8, 8), "g": (8, 8),
}


def _fixed(w, a):
    return ("fixed", w, a)


def layout(fmt: str):
    """Return (buffer specs, can_contain_null_mask) for an Arrow C format string."""
    if fmt == "n":
        return [], False
    if fmt == "b":
        return [("bitmap",)], True
    if fmt in _PRIM:
        return [_fixed(*_PRIM[fmt])], True
    if fmt in ("tdD", "tts", "ttm", "tiM"):
        return [_fixed(4, 4)], True
    if fmt in ("tdm", "ttu", "ttn") or fmt.startswith("ts") or fmt.startswith("tD"):
        return [_fixed(8, 8)], True
    if fmt == "tiD":
        return [_fixed(8, 4)], True
    if fmt == "tin":
        return [_fixed(16, 8)], True
    if fmt.startswith("d:"):
        parts = fmt[2:].split(",")
        bw = int(parts[2]) if len(parts) > 2 else 128
        if bw not in (128, 256):
            raise NotImplementedError(f"decimal bit width {bw}")
        return [_fixed(bw // 8, 8)], True
    if fmt.startswith("w:"):
        return [_fixed(int(fmt[2:]), 1)], True
    if fmt in ("z", "u"):
        return [_fixed(4, 4), ("var",)], True
    if fmt in ("Z", "U"):
        return [_fixed(8, 8), ("var",)], True
    if fmt in ("+l", "+m"):
        return [_fixed(4, 4)], True
    if fmt == "+L":
        return [_fixed(8, 8)], True
    if fmt.startswith("+w:") or fmt == "+s":
        return [], True
    if fmt == "+r":
        return [], False
    raise NotImplementedError(f"format {fmt!r} is outside the parity set")


@dataclass
class Node:
    """One ArrayData node as arrow-rs sees it after FFI import."""
    fmt: str
    sig: str
    length: int
    offset: int
    null_count: int
    validity: Optional[bytes]
    buffers: List[bytes]           # ArrayData::buffers(): excludes the null buffer
    specs: list
    children: List["Node"] = field(default_factory=list)


def _bits_for(spec):
    if spec[0] == "bitmap":
        return 1
    return spec[1] * 8


def _count_nulls(validity: bytes, offset: int, length: int) -> int:
    n = 0
    for i in range(offset, offset + length):
        if not (validity[i >> 3] >> (i & 7)) & 1:
            n += 1
    return n


def schema_sig(s: ArrowSchema) -> str:
    """Canonical data-type signature (shared definition with include/dora_gpu.h)."""
    fmt = s.format.decode()
    if s.dictionary:
        ordered = ",ordered" if (s.flags & FLAG_DICTIONARY_ORDERED) else ""
        return f"dict<{fmt},{schema_sig(s.dictionary.contents)}{ordered}>"
    out = fmt
    if fmt == "+m" and (s.flags & FLAG_MAP_KEYS_SORTED):
        out += "s"
    if s.n_children:
        parts = []
        for i in range(s.n_children):
            c = s.children[i].contents
            name = c.name.decode() if c.name else ""
            nul = "?" if (c.flags & FLAG_NULLABLE) else "!"
            parts.append(f"{name}:{nul}{schema_sig(c)}")
        out += "[" + ",".join(parts) + "]"
    return out


def read_node(a: ArrowArray, s: ArrowSchema) -> Node:
    fmt = s.format.decode()
    is_dict = bool(s.dictionary)
    specs, can_null = layout(fmt)   # dictionary: layout(key) == layout(index format)
    length, offset = a.length, a.offset
    total = length + offset
    bufs = [a.buffers[i] for i in range(a.n_buffers)]
    begin = 1 if can_null else 0
    data_bufs = []
    lens = []
    for k, spec in enumerate(specs):
        idx = begin + k
        ptr = bufs[idx] if idx < len(bufs) else None
        if spec[0] == "var":
            if length == 0:
                blen = 0
            else:
                owidth = specs[0][1]
                ctype = ctypes.c_int32 if owidth == 4 else ctypes.c_int64
                last = (lens[0] // owidth) - 1
                blen = int(ctypes.cast(bufs[begin], ctypes.POINTER(ctype))[last])
        elif k == 0 and fmt in ("z", "u", "Z", "U", "+l", "+L", "+m") and not is_dict:
            blen = (total + 1) * spec[1]
        else:
            bits = _bits_for(spec)
            blen = (total * bits + 7) // 8
        lens.append(blen)
        if ptr:
            data_bufs.append(ctypes.string_at(ptr, blen))
        elif blen == 0:
            data_bufs.append(b"")
        else:
            raise ValueError(f"null buffer {idx} with length {blen}")
    validity = None
    null_count = 0
    if can_null and bufs and bufs[0]:
        vlen = (total + 7) // 8
        vbytes = ctypes.string_at(bufs[0], vlen)
        nc = a.null_count if a.null_count >= 0 else _count_nulls(vbytes, offset, length)
        if nc != 0:
            validity, null_count = vbytes, nc
    children = []
    if is_dict:
        children.append(read_node(a.dictionary.contents, s.dictionary.contents))
    else:
        for i in range(a.n_children):
            children.append(read_node(a.children[i].contents, s.children[i].contents))
    return Node(fmt=fmt, sig=schema_sig(s), length=length, offset=offset, null_count=null_count,
                validity=validity, buffers=data_bufs, specs=specs, children=children)


def import_array(arr) -> Node:
    """pyarrow.Array -> Node tree (what `ArrayData::from_pyarrow_bound` would hold)."""
    with Exported(arr) as ex:
        return read_node(ex.array, ex.schema)
