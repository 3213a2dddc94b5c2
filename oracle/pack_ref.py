"""TEST INFRASTRUCTURE ONLY — CPU restatement (oracle) of the reference packing path.

Follows, statement for statement:
  * `required_data_size` / `required_data_size_inner`      apis/rust/node/src/node/arrow_utils.rs:4-21
  * `copy_array_into_sample` / `_inner`                   apis/rust/node/src/node/arrow_utils.rs:23-71
  * `RawData::into_arrow_array` / `buffer_into_arrow_array` apis/rust/node/src/event_stream/event.rs:35-91
  * `ArrowTypeInfo` / `BufferOffset` / `byte_array`      libraries/message/src/metadata.rs:51-87,140-143
  * `allocate_data_sample` (< 4096 B: zeroed Vec)         apis/rust/node/src/node/mod.rs:40,303-319

Parity is pinned by the reference's own known-answer tests (apis/python/operator/src/lib.rs:227-295,
libraries/arrow-convert/src/from_impls.rs:188-195) — see tests/golden/.  Never imported by the
product package `dora_amd`; only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
cpu_baseline leg use it, as the checker.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

from .arrow_ffi import Node, import_array

ZERO_COPY_THRESHOLD = 4096  # apis/rust/node/src/node/mod.rs:40


@dataclass
class BufferOffset:                      # libraries/message/src/metadata.rs:140-143
    offset: int
    len: int


@dataclass
class ArrowTypeInfo:                     # libraries/message/src/metadata.rs:51-59
    data_type: str                       # canonical signature, see oracle.arrow_ffi.schema_sig
    len: int
    null_count: int
    validity: Optional[bytes]
    offset: int
    buffer_offsets: List[BufferOffset] = field(default_factory=list)
    child_data: List["ArrowTypeInfo"] = field(default_factory=list)

    @staticmethod
    def byte_array(data_len: int) -> "ArrowTypeInfo":   # metadata.rs:74-87
        return ArrowTypeInfo("C", data_len, 0, None, 0, [BufferOffset(0, data_len)], [])

    def to_json(self):
        return {
            "data_type": self.data_type, "len": self.len, "null_count": self.null_count,
            "validity": None if self.validity is None else self.validity.hex(),
            "offset": self.offset,
            "buffer_offsets": [[b.offset, b.len] for b in self.buffer_offsets],
            "child_data": [c.to_json() for c in self.child_data],
        }

    @staticmethod
    def from_json(d) -> "ArrowTypeInfo":
        return ArrowTypeInfo(
            d["data_type"], d["len"], d["null_count"],
            None if d["validity"] is None else bytes.fromhex(d["validity"]),
            d["offset"], [BufferOffset(o, n) for o, n in d["buffer_offsets"]],
            [ArrowTypeInfo.from_json(c) for c in d["child_data"]])


def _as_node(array) -> Node:
    return array if isinstance(array, Node) else import_array(array)


def _pad(next_offset: int, spec) -> int:
    # arrow_utils.rs:13-15 / :44-46 — only BufferSpec::FixedWidth pads
    if spec[0] == "fixed":
        a = spec[2]
        return (next_offset + a - 1) // a * a
    return next_offset


def required_data_size(array) -> int:
    """arrow_utils.rs:4-8"""
    node = _as_node(array)
    return _required_inner(node, 0)


def _required_inner(node: Node, next_offset: int) -> int:
    """arrow_utils.rs:9-21: buffers zip layout, then children, DFS pre-order."""
    for buf, spec in zip(node.buffers, node.specs):
        next_offset = _pad(next_offset, spec)
        next_offset += len(buf)
    for child in node.children:
        next_offset = _required_inner(child, next_offset)
    return next_offset


def copy_array_into_sample(target: bytearray, array) -> ArrowTypeInfo:
    """arrow_utils.rs:23-26.  Writes into `target` in place; padding bytes are NOT written."""
    node = _as_node(array)
    info, _ = _copy_inner(target, 0, node)
    return info


def _copy_inner(target: bytearray, next_offset: int, node: Node):
    """arrow_utils.rs:28-71"""
    buffer_offsets = []
    for buf, spec in zip(node.buffers, node.specs):
        n = len(buf)
        # arrow_utils.rs:37-42: the size check precedes the padding step
        if len(target) - next_offset < n:
            raise AssertionError(
                f"target buffer too small (total_len: {len(target)}, offset: {next_offset}, "
                f"required_len: {n})")
        next_offset = _pad(next_offset, spec)
        if next_offset + n > len(target):
            raise IndexError("range end index out of range for slice")  # Rust slice panic
        target[next_offset:next_offset + n] = buf
        buffer_offsets.append(BufferOffset(next_offset, n))
        next_offset += n
    child_data = []
    for child in node.children:
        ci, next_offset = _copy_inner(target, next_offset, child)
        child_data.append(ci)
    info = ArrowTypeInfo(
        data_type=node.sig, len=node.length, null_count=node.null_count,
        validity=node.validity, offset=node.offset,
        buffer_offsets=buffer_offsets, child_data=child_data)
    return info, next_offset


def pack(array):
    """The sender's `send_output` (node/mod.rs:198-215) minus transport: size, zeroed sample,
    pack.  Returns (sample bytes, ArrowTypeInfo)."""
    node = _as_node(array)
    size = required_data_size(node)
    sample = bytearray(size)      # a fresh zeroed AVec / fresh shm region
    info = copy_array_into_sample(sample, node)
    return bytes(sample), info


@dataclass
class Unpacked:
    """Receiver-side ArrayData as `buffer_into_arrow_array` builds it (event.rs:61-91)."""
    data_type: str
    len: int
    offset: int
    validity: Optional[bytes]
    buffers: List[bytes]
    children: List["Unpacked"]


def into_arrow_array(raw: bytes, info: ArrowTypeInfo) -> Unpacked:
    """event.rs:35-54 + 61-91.  An empty raw buffer yields `ArrayData::new_empty(data_type)`."""
    if len(raw) == 0:
        return Unpacked(info.data_type, 0, 0, None, [], [])
    return _unpack(raw, info)


def _unpack(raw: bytes, info: ArrowTypeInfo) -> Unpacked:
    bufs = []
    for b in info.buffer_offsets:
        if b.offset + b.len > len(raw):          # Buffer::slice_with_length asserts
            raise IndexError("the offset of the new Buffer cannot exceed the existing length")
        bufs.append(raw[b.offset:b.offset + b.len])
    children = [_unpack(raw, c) for c in info.child_data]
    return Unpacked(info.data_type, info.len, info.offset, info.validity, bufs, children)


def node_regions(node: Node):
    """DFS concatenation of (validity, buffers) of the sender-side array, for checksums."""
    out = []
    if node.validity is not None:
        out.append(node.validity)
    out.extend(node.buffers)
    for c in node.children:
        out.extend(node_regions(c))
    return out


def sample_regions(sample: bytes, info: ArrowTypeInfo):
    """The parity view of a sample: validity bytes + every [offset, offset+len) region, DFS."""
    out = []
    if info.validity is not None:
        out.append(info.validity)
    for b in info.buffer_offsets:
        out.append(sample[b.offset:b.offset + b.len])
    for c in info.child_data:
        out.extend(sample_regions(sample, c))
    return out
