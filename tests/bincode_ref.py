"""TEST INFRASTRUCTURE ONLY — a second, independent statement of the reference's inter-daemon wire
format, in Python, from pyarrow types rather than Arrow C format strings (the product codec,
dora_amd/csrc/bincode.cpp, works from this library's schema trees).

`bincode::serialize(&Timestamped<InterDaemonEvent>)` (binaries/daemon/src/inter_daemon.rs:66) with
bincode 1.3.3: little-endian fixed-width integers, u64 lengths, u32 enum variant indices, u8 bool /
Option tags, structs as their fields in declaration order:
  Timestamped { inner, timestamp }                     libraries/message/src/common.rs:128-131
  InterDaemonEvent::Output / ::InputsClosed            libraries/message/src/daemon_to_daemon.rs:9-21
  Metadata, ArrowTypeInfo, BufferOffset, Parameter     libraries/message/src/metadata.rs:9-15,51-59,133-143
Third-party layouts (not in /root/reference; restated from their published sources, so the bytes
below are parity-unpinned): uuid 1.11 (16 raw bytes behind a u64 length), uhlc 0.5.2 Timestamp
{time: NTP64 u64, id: u128}, arrow-schema 53.2.0 DataType (variant order below) and Field
{name, data_type, nullable, dict_id, dict_is_ordered, metadata}.
"""
import struct

import pyarrow as pa


def u8(v):
    return struct.pack("<B", v)


def u16(v):
    return struct.pack("<H", v)


def u32(v):
    return struct.pack("<I", v)


def u64(v):
    return struct.pack("<Q", v)


def i32(v):
    return struct.pack("<i", v)


def i64(v):
    return struct.pack("<q", v)


def string(s):
    b = s.encode() if isinstance(s, str) else bytes(s)
    return u64(len(b)) + b


def option(v, enc):
    return u8(0) if v is None else u8(1) + enc(v)


# arrow-schema 53.2.0 DataType, in declaration order
VARIANTS = ["Null", "Boolean", "Int8", "Int16", "Int32", "Int64", "UInt8", "UInt16", "UInt32",
            "UInt64", "Float16", "Float32", "Float64", "Timestamp", "Date32", "Date64", "Time32",
            "Time64", "Duration", "Interval", "Binary", "FixedSizeBinary", "LargeBinary",
            "BinaryView", "Utf8", "LargeUtf8", "Utf8View", "List", "ListView", "FixedSizeList",
            "LargeList", "LargeListView", "Struct", "Union", "Dictionary", "Decimal128",
            "Decimal256", "Map", "RunEndEncoded"]
V = {n: i for i, n in enumerate(VARIANTS)}
UNIT = {"s": 0, "ms": 1, "us": 2, "ns": 3}
SIMPLE = [(pa.types.is_null, "Null"), (pa.types.is_boolean, "Boolean"),
          (pa.types.is_int8, "Int8"), (pa.types.is_int16, "Int16"), (pa.types.is_int32, "Int32"),
          (pa.types.is_int64, "Int64"), (pa.types.is_uint8, "UInt8"),
          (pa.types.is_uint16, "UInt16"), (pa.types.is_uint32, "UInt32"),
          (pa.types.is_uint64, "UInt64"), (pa.types.is_float16, "Float16"),
          (pa.types.is_float32, "Float32"), (pa.types.is_float64, "Float64"),
          (pa.types.is_date32, "Date32"), (pa.types.is_date64, "Date64"),
          (pa.types.is_large_binary, "LargeBinary"), (pa.types.is_large_string, "LargeUtf8")]


def datatype(t: pa.DataType) -> bytes:
    if pa.types.is_dictionary(t):
        return u32(V["Dictionary"]) + datatype(t.index_type) + datatype(t.value_type)
    for pred, name in SIMPLE:
        if pred(t):
            return u32(V[name])
    if pa.types.is_fixed_size_binary(t) and not pa.types.is_decimal(t):
        return u32(V["FixedSizeBinary"]) + i32(t.byte_width)
    if pa.types.is_binary(t):
        return u32(V["Binary"])
    if pa.types.is_string(t):
        return u32(V["Utf8"])
    if pa.types.is_timestamp(t):
        return u32(V["Timestamp"]) + u32(UNIT[t.unit]) + option(t.tz, string)
    if pa.types.is_time32(t):
        return u32(V["Time32"]) + u32(UNIT[t.unit])
    if pa.types.is_time64(t):
        return u32(V["Time64"]) + u32(UNIT[t.unit])
    if pa.types.is_duration(t):
        return u32(V["Duration"]) + u32(UNIT[t.unit])
    if pa.types.is_interval(t):  # pyarrow's only interval type: MonthDayNano (IntervalUnit 2)
        return u32(V["Interval"]) + u32(2)
    if pa.types.is_decimal128(t):
        return u32(V["Decimal128"]) + u8(t.precision) + struct.pack("<b", t.scale)
    if pa.types.is_decimal256(t):
        return u32(V["Decimal256"]) + u8(t.precision) + struct.pack("<b", t.scale)
    if pa.types.is_map(t):
        entries = pa.field("entries", pa.struct([t.key_field, t.item_field]), nullable=False)
        return u32(V["Map"]) + field(entries) + u8(1 if t.keys_sorted else 0)
    if pa.types.is_fixed_size_list(t):
        return u32(V["FixedSizeList"]) + field(t.value_field) + i32(t.list_size)
    if pa.types.is_large_list(t):
        return u32(V["LargeList"]) + field(t.value_field)
    if pa.types.is_list(t):
        return u32(V["List"]) + field(t.value_field)
    if pa.types.is_struct(t):
        return u32(V["Struct"]) + u64(t.num_fields) + b"".join(
            field(t.field(k)) for k in range(t.num_fields))
    if pa.types.is_run_end_encoded(t):
        return (u32(V["RunEndEncoded"]) + field(pa.field("run_ends", t.run_end_type, False)) +
                field(pa.field("values", t.value_type, True)))
    raise ValueError(f"no statement for {t}")


def field(f: pa.Field) -> bytes:
    ordered = pa.types.is_dictionary(f.type) and f.type.ordered
    meta = f.metadata or {}
    return (string(f.name) + datatype(f.type) + u8(1 if f.nullable else 0) + i64(0) +
            u8(1 if ordered else 0) + u64(len(meta)) +
            b"".join(string(k) + string(v) for k, v in meta.items()))


def child_types(t: pa.DataType):
    """The data types of an array's ArrayData children (ArrowTypeInfo.child_data)."""
    if pa.types.is_dictionary(t):
        return [t.value_type]
    if pa.types.is_map(t):
        return [pa.struct([t.key_field, t.item_field])]
    if pa.types.is_list(t) or pa.types.is_large_list(t) or pa.types.is_fixed_size_list(t):
        return [t.value_type]
    if pa.types.is_struct(t):
        return [t.field(k).type for k in range(t.num_fields)]
    if pa.types.is_run_end_encoded(t):
        return [t.run_end_type, t.value_type]
    return []


def type_info(t: pa.DataType, ti: dict) -> bytes:
    """ArrowTypeInfo from the array's type and this library's type info (oracle JSON form)."""
    kids = child_types(t)
    assert len(kids) == len(ti["child_data"]), (t, ti)
    v = ti["validity"]
    return (datatype(t) + u64(ti["len"]) + u64(ti["null_count"]) +
            option(None if v is None else bytes.fromhex(v), string) + u64(ti["offset"]) +
            u64(len(ti["buffer_offsets"])) +
            b"".join(u64(o) + u64(n) for o, n in ti["buffer_offsets"]) +
            u64(len(kids)) + b"".join(type_info(k, c) for k, c in zip(kids, ti["child_data"])))


def parameters(meta: dict) -> bytes:
    """BTreeMap<String, Parameter>: keys in byte order; Bool 0, Integer 1, String 2."""
    out = [u64(len(meta))]
    for k in sorted(meta, key=lambda s: s.encode()):
        v = meta[k]
        if isinstance(v, bool):
            out.append(string(k) + u32(0) + u8(int(v)))
        elif isinstance(v, int):
            out.append(string(k) + u32(1) + i64(v))
        else:
            out.append(string(k) + u32(2) + string(str(v)))
    return b"".join(out)


def ntp64(ns: int) -> int:
    """uhlc NTP64 of a UNIX-epoch time: seconds << 32 | the fraction of a second (rounded up,
    so that converting back truncates to the same nanosecond)."""
    s, sub = divmod(ns, 10**9)
    return (s << 32) + -(-(sub << 32) // 10**9)


def timestamp(ns: int, hlc_id: bytes) -> bytes:
    assert len(hlc_id) == 16
    return u64(ntp64(ns)) + hlc_id


def output_event(df_uuid: bytes, node: str, output: str, version: int, meta_ns: int,
                 hlc_id: bytes, ti: bytes, params: bytes, data, event_ns: int) -> bytes:
    return (u32(0) + string(df_uuid) + string(node) + string(output) + u16(version) +
            timestamp(meta_ns, hlc_id) + ti + params + option(data, string) +
            timestamp(event_ns, hlc_id))


def inputs_closed_event(df_uuid: bytes, inputs, event_ns: int, hlc_id: bytes) -> bytes:
    pairs = sorted(set(inputs), key=lambda p: (p[0].encode(), p[1].encode()))
    return (u32(1) + string(df_uuid) + u64(len(pairs)) +
            b"".join(string(r) + string(i) for r, i in pairs) + timestamp(event_ns, hlc_id))
