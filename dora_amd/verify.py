"""Device-side checksums of received samples (size-independent parity at full sizes).

`regions_csum(sample_ptr, type_info)` folds csum64 of every parity region of a sample in DFS
order — validity bytes of the node (from the type info) then each [offset, offset+len) buffer
region — with combine(acc, c) = fmix64(acc + c * GOLDEN).  The definitions match
oracle/checksum_ref.py; this module computes them on the GPU for the product path.
"""
from __future__ import annotations

from .device import DeviceBuffer, Stream, csum64
from .type_info import ArrowTypeInfo

MASK = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15


def fmix64(z: int) -> int:
    z &= MASK
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
    return z ^ (z >> 31)


def combine(acc: int, c: int) -> int:
    return fmix64((acc + c * GOLDEN) & MASK)


def regions_csum(sample_ptr: int, ti: ArrowTypeInfo, stream: Stream | None = None) -> int:
    acc = 0

    def walk(t: ArrowTypeInfo):
        nonlocal acc
        if t.validity is not None:
            b = DeviceBuffer.from_bytes(t.validity, stream)
            try:
                acc = combine(acc, csum64(b.ptr, len(t.validity), stream))
            finally:
                b.free()
        for bo in t.buffer_offsets:
            acc = combine(acc, csum64(sample_ptr + bo.offset, bo.len, stream))
        for c in t.child_data:
            walk(c)
    walk(ti)
    return acc


def to_i64(u: int) -> int:
    """Unsigned 64-bit -> signed (metadata integers are i64)."""
    return u - (1 << 64) if u >= (1 << 63) else u


def to_u64(i: int) -> int:
    return i & MASK
