"""The inter-daemon wire: frames carry bincode of Timestamped<InterDaemonEvent>, as the
reference's daemons exchange them (binaries/daemon/src/inter_daemon.rs:66, :156;
libraries/message/src/daemon_to_daemon.rs:9-21).  The product codec (csrc/bincode.cpp, through its
test hooks) against a second statement of the format written from pyarrow types
(tests/bincode_ref.py), decode(encode(x)) == x for every type of the parity set, one event spelled
out byte by byte, and the malformed frames a reader must refuse.  No fixture in the reference holds
these bytes and no Rust toolchain is here to make one: the serde layouts of uuid / uhlc /
arrow-schema are restated from their published sources (parity-unpinned)."""
import ctypes
import json
from decimal import Decimal

import numpy as np
import pyarrow as pa
import pytest

from dora_amd import _lib
from dora_amd.arrow_utils import Plan
from dora_amd.node import encode_parameters_py
from tests import bincode_ref as ref

HLC = bytes(range(1, 17))
DF = "0191f0e4-3c7a-7b2e-9d41-5a6b7c8d9e0f"
DF_BYTES = bytes.fromhex(DF.replace("-", ""))
META_NS = 1_700_000_000_123_456_789
EVENT_NS = 1_700_000_000_223_456_789


def _call(fn, *args):
    lib = _lib.load_testing()
    n = ctypes.c_size_t()
    getattr(lib, fn)(*args, None, 0, ctypes.byref(n))
    buf = ctypes.create_string_buffer(max(1, n.value))
    rc = getattr(lib, fn)(*args, buf, n.value, ctypes.byref(n))
    assert rc == 0, _lib.load().dora_gpu_last_error()
    return buf.raw[:n.value]


def encode_output(ti: bytes, params: bytes, data, df=DF, node="src", output="data"):
    return _call("dora_gpu_test_ide_output", df.encode(), node.encode(), output.encode(), ti,
                 len(ti), params, len(params), META_NS, EVENT_NS, HLC, data or b"",
                 len(data or b""), data is not None)


def encode_closed(pairs, df=DF):
    rs = (ctypes.c_char_p * max(1, len(pairs)))(*[r.encode() for r, _ in pairs])
    ins = (ctypes.c_char_p * max(1, len(pairs)))(*[i.encode() for _, i in pairs])
    return _call("dora_gpu_test_ide_inputs_closed", df.encode(), rs, ins, len(pairs), EVENT_NS,
                 HLC)


def decode(frame: bytes) -> dict:
    lib = _lib.load_testing()
    n = ctypes.c_size_t()
    buf = ctypes.create_string_buffer(1 << 20)
    rc = lib.dora_gpu_test_ide_decode(frame, len(frame), buf, len(buf), ctypes.byref(n))
    if rc != 0:
        raise ValueError(_lib.load().dora_gpu_last_error().decode())
    return json.loads(buf.value.decode())


def _arrays():
    from dora_amd.workloads import point_cloud
    rng = np.random.default_rng(7)
    meta_struct = pa.StructArray.from_arrays(
        [pa.array([1, 2, 3], pa.int64()), pa.array(["x", None, "z"])],
        fields=[pa.field("x", pa.int64(), nullable=False, metadata={"unit": "m", "a": "1"}),
                pa.field("label", pa.string())])
    return {
        "uint8": pa.array(rng.integers(0, 256, 1000, dtype=np.uint8)),
        "int32_nulls": pa.array([1, None, 3, None, 5], pa.int32()),
        "float16": pa.array(np.array([1.0, 2.5], np.float16)),
        "bool": pa.array([True, False, None, True]),
        "null": pa.nulls(3),
        "utf8": pa.array(["a", "bc", None, "def"]),
        "large_binary": pa.array([b"x", b"yz", b""], pa.large_binary()),
        "fixed_size_binary": pa.array([b"abcd", b"efgh"], pa.binary(4)),
        "timestamp_tz": pa.array([1, 2], pa.timestamp("us", tz="UTC")),
        "timestamp_naive": pa.array([1, 2], pa.timestamp("ns")),
        "date32": pa.array([1, 2], pa.date32()),
        "date64": pa.array([86400000], pa.date64()),
        "time32": pa.array([1, 2], pa.time32("ms")),
        "time64": pa.array([1, 2], pa.time64("ns")),
        "duration": pa.array([5], pa.duration("s")),
        "interval": pa.array([pa.MonthDayNano([1, 2, 3])], pa.month_day_nano_interval()),
        "decimal128": pa.array([Decimal("1.23"), None], pa.decimal128(10, 2)),
        "decimal256": pa.array([Decimal("-4.5")], pa.decimal256(40, 1)),
        "list_struct_cloud": point_cloud(n_points=200, n_lists=4),
        "fixed_size_list": pa.array([[1.0, 2.0], [3.0, 4.0]], pa.list_(pa.float32(), 2)),
        "large_list": pa.array([[1], [2, 3]], pa.large_list(pa.int16())),
        "dictionary": pa.array(["a", "b", "a", None]).dictionary_encode(),
        "map": pa.array([[("k", 1)], [("j", 2), ("x", 3)]], pa.map_(pa.string(), pa.int32())),
        "run_end_encoded": pa.RunEndEncodedArray.from_arrays(pa.array([2, 5], pa.int32()),
                                                             pa.array([1.0, 2.0])),
        "field_metadata": meta_struct,
        "sliced": pa.array(list(range(40)), pa.int64()).slice(3, 20),
    }


ARRAYS = _arrays()


@pytest.mark.parametrize("name", sorted(ARRAYS))
def test_output_event_matches_the_second_statement_and_round_trips(name):
    arr = ARRAYS[name]
    with Plan.of(arr) as p:
        ti = p.type_info_bytes()
        ti_json = p.type_info().to_json()
    meta = {"seq": 7, "ok": True, "tag": f"m-{name}", "neg": -3}
    params = encode_parameters_py(meta)
    data = bytes(range(256)) * 3
    frame = encode_output(ti, params, data)
    want = ref.output_event(DF_BYTES, "src", "data", 0, META_NS, HLC,
                            ref.type_info(arr.type, ti_json), ref.parameters(meta), data,
                            EVENT_NS)
    assert frame == want
    d = decode(frame)
    assert d["kind"] == 0 and d["node_id"] == "src" and d["output_id"] == "data"
    assert d["dataflow_uuid"] == DF_BYTES.hex()
    assert d["meta_ns"] == META_NS and d["event_ns"] == EVENT_NS
    assert bytes.fromhex(d["type_info"]) == ti  # this library's own form comes back exactly
    assert bytes.fromhex(d["parameters"]) == params
    assert d["has_data"] and bytes.fromhex(d["data"]) == data


def test_output_without_data_and_without_parameters():
    with Plan.of(pa.array([], pa.uint8())) as p:
        ti = p.type_info_bytes()
    frame = encode_output(ti, b"", None)
    d = decode(frame)
    assert not d["has_data"] and d["data"] == "" and d["parameters"] == ""
    # data: None is one tag byte before the trailing Timestamped timestamp (24 bytes)
    assert frame[-25] == 0


def test_one_event_byte_by_byte():
    """A 4-byte UInt8 message (ArrowTypeInfo::byte_array, metadata.rs:74-87) spelled out."""
    with Plan.of(pa.array([9, 8, 7, 6], pa.uint8())) as p:
        ti = p.type_info_bytes()
    frame = encode_output(ti, encode_parameters_py({"k": 1}), b"\x09\x08\x07\x06",
                          df=DF, node="n", output="o")
    ntp = (1_700_000_000 << 32) + 530242872   # 0.123456789 s in 2^-32 s, rounded up
    ntp_e = (1_700_000_000 << 32) + 959739601
    want = b"".join([
        bytes.fromhex("00000000"),                                  # InterDaemonEvent::Output
        bytes.fromhex("1000000000000000") + DF_BYTES,               # dataflow_id: Uuid
        bytes.fromhex("0100000000000000") + b"n",                   # node_id
        bytes.fromhex("0100000000000000") + b"o",                   # output_id
        bytes.fromhex("0000"),                                      # metadata_version
        ntp.to_bytes(8, "little") + HLC,                            # timestamp: NTP64, ID
        bytes.fromhex("06000000"),                                  # DataType::UInt8
        (4).to_bytes(8, "little"),                                  # len
        (0).to_bytes(8, "little"),                                  # null_count
        b"\x00",                                                    # validity: None
        (0).to_bytes(8, "little"),                                  # offset
        (1).to_bytes(8, "little") + (0).to_bytes(8, "little") + (4).to_bytes(8, "little"),
        (0).to_bytes(8, "little"),                                  # child_data: []
        (1).to_bytes(8, "little") + (1).to_bytes(8, "little") + b"k" +  # parameters {"k":
        bytes.fromhex("01000000") + (1).to_bytes(8, "little"),      #   Parameter::Integer(1)}
        b"\x01" + (4).to_bytes(8, "little") + b"\x09\x08\x07\x06",  # data: Some(AVec)
        ntp_e.to_bytes(8, "little") + HLC,                          # Timestamped::timestamp
    ])
    assert frame == want


def test_inputs_closed_event():
    pairs = [("dst1", "data"), ("dst0", "side"), ("dst0", "data"), ("dst1", "data")]
    frame = encode_closed(pairs)
    assert frame == ref.inputs_closed_event(DF_BYTES, pairs, EVENT_NS, HLC)
    d = decode(frame)
    assert d["kind"] == 1 and d["event_ns"] == EVENT_NS
    assert d["inputs"] == [["dst0", "data"], ["dst0", "side"], ["dst1", "data"]]  # BTreeSet order


def test_dataflow_names_map_to_one_uuid():
    """A UUID's text is its bytes; any other dataflow name hashes to a version-8 UUID, the same on
    every daemon, so two daemons of one dataflow agree and different names do not."""
    with Plan.of(pa.array([1], pa.uint8())) as p:
        ti = p.type_info_bytes()
    a = decode(encode_output(ti, b"", None, df="df-test"))["dataflow_uuid"]
    b = decode(encode_output(ti, b"", None, df="df-test"))["dataflow_uuid"]
    c = decode(encode_output(ti, b"", None, df="df-other"))["dataflow_uuid"]
    assert a == b != c
    u = bytes.fromhex(a)
    assert u[6] >> 4 == 8 and u[8] >> 6 == 2
    assert decode(encode_output(ti, b"", None, df=DF.upper()))["dataflow_uuid"] == DF_BYTES.hex()


@pytest.mark.parametrize("ns", [0, 1, 999_999_999, 1_000_000_000, 1_500_000_000,
                                1_700_000_000_123_456_789, 1_953_125,
                                ((1 << 32) - 1) * 10**9 + 999_999_999])  # NTP64's last second
def test_ntp64_round_trip_is_exact(ns):
    with Plan.of(pa.array([1], pa.uint8())) as p:
        ti = p.type_info_bytes()
    frame = _call("dora_gpu_test_ide_output", DF.encode(), b"s", b"o", ti, len(ti), b"", 0, ns,
                  ns, HLC, b"", 0, 0)
    assert decode(frame)["meta_ns"] == ns
    assert int.from_bytes(frame[-24:-16], "little") == ref.ntp64(ns)
    if ns == 1_500_000_000:
        assert ref.ntp64(ns) == (1 << 32) + (1 << 31)


def test_malformed_frames_are_refused():
    with Plan.of(pa.array([1, 2], pa.int32())) as p:
        ti = p.type_info_bytes()
    frame = encode_output(ti, encode_parameters_py({"a": "b"}), b"xy")
    for cut in (0, 3, 20, len(frame) // 2, len(frame) - 1):
        with pytest.raises(ValueError):
            decode(frame[:cut])
    with pytest.raises(ValueError, match="trailing"):
        decode(frame + b"\x00")
    with pytest.raises(ValueError, match="variant"):
        decode(b"\x02\x00\x00\x00" + frame[4:])
    bad_type = bytearray(frame)
    at = 4 + 8 + 16 + 8 + 3 + 8 + 4 + 2 + 24          # the type info's DataType variant
    bad_type[at:at + 4] = (33).to_bytes(4, "little")  # Union: outside the parity set
    with pytest.raises(ValueError, match="parity set|variant"):
        decode(bytes(bad_type))


def test_validity_left_in_the_sample_is_refused():
    """The forwarder folds a device sample's validity tail back inline before encoding
    (interdaemon.cpp Forwarder::stage); a type info still pointing into the sample cannot be
    expressed as the reference's Option<Vec<u8>>."""
    with Plan.of(pa.array([1, None], pa.int32())) as p:
        ti = bytearray(p.type_info_bytes())
    # the validity tag follows the u32 schema length, the schema, len and null_count
    sl = int.from_bytes(ti[:4], "little")
    tag_at = 4 + sl + 16
    assert ti[tag_at] == 1
    lib = _lib.load_testing()
    n = ctypes.c_size_t()
    ti2 = bytes(ti[:tag_at]) + b"\x02" + (0).to_bytes(8, "little") + (1).to_bytes(8, "little") + \
        bytes(ti[tag_at + 1 + 8 + 1:])
    rc = lib.dora_gpu_test_ide_output(DF.encode(), b"s", b"o", ti2, len(ti2), b"", 0, 0, 0, HLC,
                                      b"", 0, 0, None, 0, ctypes.byref(n))
    assert rc != 0 and b"validity" in _lib.load().dora_gpu_last_error()
