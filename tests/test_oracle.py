"""Pin the CPU oracle against the reference's known-answer tests (hand-written layouts)."""
import json
import os

import pytest

from oracle.checksum_ref import combine, csum64, regions_csum, splitmix_bytes
from oracle.pack_ref import (ArrowTypeInfo, into_arrow_array, node_regions, pack,
                             required_data_size, sample_regions)
from oracle.arrow_ffi import import_array
from tests.golden import recipes

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
KATS = json.load(open(os.path.join(GOLDEN, "kats.json")))
CASES = json.load(open(os.path.join(GOLDEN, "cases.json")))


@pytest.mark.parametrize("kat", KATS, ids=[k["recipe"] for k in KATS])
def test_oracle_matches_reference_kat(kat):
    arr = recipes.build(kat["recipe"])
    sample, info = pack(arr)
    assert sample.hex() == kat["sample"]
    assert info.to_json() == kat["type_info"]
    assert required_data_size(arr) == len(sample)


@pytest.mark.parametrize("kat", KATS, ids=[k["recipe"] for k in KATS])
def test_oracle_roundtrip_like_assert_roundtrip(kat):
    """apis/python/operator/src/lib.rs:227-240: pack then into_arrow_array gives the same
    ArrayData (buffers, validity, offset, children)."""
    arr = recipes.build(kat["recipe"])
    node = import_array(arr)
    sample, info = pack(node)
    un = into_arrow_array(sample, info)
    if len(sample) == 0:
        assert un.len == 0  # ArrayData::new_empty (event.rs:65-67)
        return

    def same(n, u):
        assert n.sig == u.data_type and n.length == u.len and n.offset == u.offset
        assert n.validity == u.validity
        assert n.buffers == u.buffers
        assert len(n.children) == len(u.children)
        for a, b in zip(n.children, u.children):
            same(a, b)
    same(node, un)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_regression_cases(case):
    arr = recipes.build(case["recipe"])
    sample, info = pack(arr)
    assert len(sample) == case["sample_len"]
    assert csum64(sample) == case["sample_csum64"]
    if "sample" in case:
        assert sample.hex() == case["sample"]
    if case["type_info"] is not None:
        assert info.to_json() == case["type_info"]
        assert ArrowTypeInfo.from_json(case["type_info"]).to_json() == case["type_info"]


def test_c3_required_size_matches_survey():
    from dora_amd.workloads import point_cloud
    # 13,000,068 B for 1M points in 16 lists
    assert required_data_size(point_cloud()) == 13_000_068


def test_padding_not_written_into_recycled_sample():
    """arrow_utils.rs:48: only [off, off+len) is written; stale padding stays."""
    from oracle.pack_ref import copy_array_into_sample
    arr = recipes.build("kat4")
    target = bytearray(b"\xee" * 20)
    info = copy_array_into_sample(target, arr)
    assert target[1:4] == b"\xee\xee\xee"
    assert info.child_data[1].buffer_offsets[0].offset == 4


def test_too_small_target_asserts():
    from oracle.pack_ref import copy_array_into_sample
    with pytest.raises(AssertionError, match="target buffer too small"):
        copy_array_into_sample(bytearray(3), recipes.build("kat1"))


def test_checksum_properties():
    a = splitmix_bytes(1000, 0xD05A + 1000)
    assert len(a) == 1000
    assert csum64(a) != csum64(a[:-1] + bytes([a[-1] ^ 1]))
    assert csum64(b"") != csum64(b"\0")
    assert csum64(a[:8] + a[8:]) == csum64(a)
    assert regions_csum([a, b"x"]) == combine(combine(0, csum64(a)), csum64(b"x"))
    # position sensitivity: swapping two words changes the checksum
    b = a[8:16] + a[:8] + a[16:]
    assert csum64(a) != csum64(b)


def test_sample_regions_cover_sender_regions():
    arr = recipes.build("struct_nulls_sliced")
    node = import_array(arr)
    sample, info = pack(node)
    assert regions_csum(sample_regions(sample, info)) == regions_csum(node_regions(node))
