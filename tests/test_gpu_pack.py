"""GPU parity of the pack kernel (through the C ABI) against the CPU oracle.

* every KAT / regression fixture: device array -> HIP pack -> sample bytes == oracle sample,
  ArrowTypeInfo == oracle, and the reference's `assert_roundtrip`
  (apis/python/operator/src/lib.rs:227-240) on the device: import the sample zero-copy,
  download, compare with the original pyarrow array;
* alignment sweep: every (src mod 16, dst mod 16, length) class of the funnel-shift paths;
* full sizes (BASELINE.json configs) through size-independent properties: csum64 of the sample
  regions == csum64 of the source regions computed independently, payload generator parity.
"""
import ctypes
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def dev():
    from dora_amd import device
    assert device.device_count() >= 1
    device.set_device(0)
    s = device.Stream()
    yield s
    s.close()


def _pack_on_device(arr, stream, poison=None):
    from dora_amd.arrow_utils import Plan
    from dora_amd.device import DeviceArray, DeviceBuffer
    da = DeviceArray.from_pyarrow(arr)
    plan = Plan.of(da)
    n = plan.size
    buf = DeviceBuffer(max(n, 1))
    if poison is not None:
        buf.fill(poison, stream)
    plan.pack(buf.ptr, buf.size, stream)
    stream.sync()
    return da, plan, buf, n


def _all_cases():
    from tests.golden import recipes
    return recipes.KATS + recipes.CASES


@pytest.mark.parametrize("name", _all_cases())
def test_pack_matches_oracle(dev, name):
    from oracle.pack_ref import pack
    from tests.golden import recipes
    arr = recipes.build(name)
    want, info = pack(arr)
    da, plan, buf, n = _pack_on_device(arr, dev, poison=0)
    try:
        assert n == len(want)
        assert plan.type_info().to_json() == info.to_json()
        got = buf.to_bytes(n)
        assert got == want
    finally:
        plan.close(); buf.free(); da.close()


@pytest.mark.parametrize("name", _all_cases())
def test_device_assert_roundtrip(dev, name):
    """assert_roundtrip on the device: pack -> into_arrow_array (zero copy) -> equal array."""
    from dora_amd.arrow_utils import sample_to_device_array
    from tests.golden import recipes
    arr = recipes.build(name)
    da, plan, buf, n = _pack_on_device(arr, dev, poison=0xAB)
    try:
        ti = plan.type_info()
        back = sample_to_device_array(buf.ptr, n, ti)
        try:
            host = back.to_pyarrow()
        finally:
            back.close()
        if n == 0:
            assert len(host) == 0 and host.type == arr.type  # ArrayData::new_empty
        else:
            assert host.type == arr.type
            assert host.equals(arr), (host, arr)
    finally:
        plan.close(); buf.free(); da.close()


def test_stale_padding_is_not_written(dev):
    """Padding bytes stay as they were (recycled shm regions, arrow_utils.rs:48)."""
    from tests.golden import recipes
    da, plan, buf, n = _pack_on_device(recipes.build("kat4"), dev, poison=0xEE)
    try:
        got = buf.to_bytes(n)
        assert got[1:4] == b"\xee\xee\xee"
        assert got[0] == 0x0C
    finally:
        plan.close(); buf.free(); da.close()


def test_too_small_target_is_an_error(dev):
    from dora_amd import _lib
    from tests.golden import recipes
    da, plan, buf, n = _pack_on_device(recipes.build("kat2"), dev)
    try:
        with pytest.raises(_lib.DoraGpuError, match="too small"):
            plan.pack(buf.ptr, n - 1, dev)
    finally:
        plan.close(); buf.free(); da.close()


@pytest.mark.parametrize("src_mis", list(range(16)))
def test_alignment_sweep(dev, src_mis):
    """Byte-array segments at every src/dst misalignment and ragged lengths."""
    from dora_amd import device
    from dora_amd.arrow_utils import Plan
    from oracle.checksum_ref import splitmix_bytes
    rng = np.random.default_rng(src_mis)
    data = splitmix_bytes(70000, 0xD05A + src_mis)
    src = device.DeviceBuffer.from_bytes(b"\0" * (16 + src_mis) + data + b"\0" * 16, dev)
    dst = device.DeviceBuffer(80000)
    try:
        for dst_off in range(16):
            for length in [0, 1, 15, 16, 17, 31, 33, 255, 4096 + 5, 16384 + 7,
                           int(rng.integers(1, 65000))]:
                dst.fill(0x5A, dev)
                with Plan.of_bytes(src.ptr + 16 + src_mis, length, on_device=True) as p:
                    p.pack(dst.ptr + dst_off, length, dev)
                dev.sync()
                got = dst.to_bytes(length + 32)
                assert got[:dst_off] == b"\x5a" * dst_off
                assert got[dst_off:dst_off + length] == data[:length], (dst_off, length)
                assert got[dst_off + length:] == b"\x5a" * (32 - dst_off)
    finally:
        src.free(); dst.free()


@pytest.mark.parametrize("size", [4096, 40960, 409600, 4096000, 40960000])
def test_payload_fill_and_checksum_full_sizes(dev, size):
    """C2 payloads: device splitmix == oracle bytes (checked via csum64 both sides)."""
    from dora_amd import device
    from oracle.checksum_ref import csum64, splitmix_bytes
    want = splitmix_bytes(size, 0xD05A + size)
    b = device.DeviceBuffer(size)
    try:
        device.fill_splitmix(b.ptr, size, 0xD05A + size, dev)
        dev.sync()
        assert device.csum64(b.ptr, size, dev) == csum64(want)
        if size <= 409600:
            assert b.to_bytes() == want
    finally:
        b.free()


@pytest.mark.parametrize("off", [0, 1, 3, 8, 13])
def test_device_checksum_unaligned(dev, off):
    from dora_amd import device
    from oracle.checksum_ref import csum64
    data = bytes(np.random.default_rng(off).integers(0, 256, 10007, dtype=np.uint8))
    b = device.DeviceBuffer.from_bytes(data, dev)
    try:
        for n in [0, 1, 7, 8, 9, 1000, 10007 - off]:
            assert device.csum64(b.ptr + off, n, dev) == csum64(data[off:off + n]), n
    finally:
        b.free()


def test_c3_point_cloud_full_size(dev):
    """C3: 1M-point List<Struct<x,y,z,intensity>>: 13,000,068 B sample, checksum parity of every
    region against the oracle (size-independent), type info identical."""
    from dora_amd import device
    from dora_amd.workloads import point_cloud
    from oracle.arrow_ffi import import_array
    from oracle.checksum_ref import csum64
    from oracle.pack_ref import copy_array_into_sample, required_data_size
    arr = point_cloud()
    node = import_array(arr)
    size = required_data_size(node)
    assert size == 13_000_068
    ref = bytearray(size)
    info = copy_array_into_sample(ref, node)
    da, plan, buf, n = _pack_on_device(arr, dev, poison=0)
    try:
        assert n == size
        assert plan.type_info().to_json() == info.to_json()
        assert device.csum64(buf.ptr, n, dev) == csum64(bytes(ref))
    finally:
        plan.close(); buf.free(); da.close()


def test_golden_cases_checksums(dev):
    """Replay cases.json (oracle-generated, committed) on the device."""
    from dora_amd import device
    from tests.golden import recipes
    cases = json.load(open(os.path.join(GOLDEN, "cases.json")))
    for c in cases:
        da, plan, buf, n = _pack_on_device(recipes.build(c["recipe"]), dev, poison=0)
        try:
            assert n == c["sample_len"]
            assert device.csum64(buf.ptr, n, dev) == c["sample_csum64"], c["name"]
        finally:
            plan.close(); buf.free(); da.close()


@pytest.mark.parametrize("dtype", ["uint8", "int32", "float32", "float64"])
def test_dlpack_export_to_torch(dev, dtype):
    """§8f-1: a device sample reaches torch zero-copy through DLPack (kDLROCM)."""
    import pyarrow as pa
    import torch
    from dora_amd.device import DeviceArray
    vals = np.arange(1000, dtype=dtype) * 3
    arr = pa.array(vals).slice(10, 900)
    with DeviceArray.from_pyarrow(arr) as da:
        t = torch.from_dlpack(da)
        assert t.device.type == "cuda" and t.shape == (900,)
        assert np.array_equal(t.cpu().numpy(), vals[10:910])
        del t


def _compact_cases():
    import pyarrow as pa
    from tests.golden import recipes
    out = [pa.array(range(100), pa.int32()).slice(17, 40),
           pa.array([True, False, True] * 40).slice(5, 77),
           pa.array(["a", "bb", None, "dddd"] * 20).slice(9, 31),
           pa.array([[1, 2], [], None, [3, 4, 5]] * 10, pa.list_(pa.int64())).slice(3, 21),
           pa.array([{"a": i, "b": str(i)} if i % 7 else None for i in range(60)]).slice(11, 33)]
    out += [recipes.build(n) for n in recipes.KATS + recipes.CASES
            if n not in ("run_end_encoded", "kat11")]
    return out


@pytest.mark.parametrize("arr", _compact_cases())
def test_compact_pack_roundtrip(dev, arr):
    """Compacting plans (new capability): bit-shifted bitmaps, rebased offsets and sliced
    children on the GPU give a sample that imports (unchanged receiver) to an equal array."""
    from dora_amd.arrow_utils import Plan, sample_to_device_array
    from dora_amd.device import DeviceArray, DeviceBuffer
    da = DeviceArray.from_pyarrow(arr)
    plan = Plan.of(da, compact=True)
    buf = DeviceBuffer(max(plan.size, 1))
    try:
        buf.fill(0xCD, dev)
        plan.pack(buf.ptr, buf.size, dev)
        dev.sync()
        ti = plan.type_info()
        back = sample_to_device_array(buf.ptr, plan.size, ti)
        try:
            host = back.to_pyarrow()
        finally:
            back.close()
        assert host.type == arr.type
        if plan.size == 0:
            assert len(host) == 0  # empty sample -> ArrayData::new_empty (event.rs:65-67)
        else:
            assert host.equals(arr), (host, arr)
            assert host.offset == 0
    finally:
        plan.close(); buf.free(); da.close()


def _regions(info):
    out = [(b.offset, b.len) for b in info.buffer_offsets]
    for c in info.child_data:
        out += _regions(c)
    return out


@pytest.mark.parametrize("name", _all_cases())
@pytest.mark.parametrize("slack", [0, 48])
def test_stitched_edges_keep_regions_and_padding(dev, name, slack):
    """Boundary units written whole (pack_device.h: a segment's unaligned head/tail unit is
    gathered from every segment holding a byte of it and stored at full width when it lies in
    the writable destination): every region equals the oracle's, and every byte outside the
    regions — padding between buffers and the slack past the sample — keeps the poison."""
    from oracle.pack_ref import pack
    from tests.golden import recipes
    from dora_amd.arrow_utils import Plan
    from dora_amd.device import DeviceArray, DeviceBuffer
    arr = recipes.build(name)
    want, info = pack(arr)
    da = DeviceArray.from_pyarrow(arr)
    plan = Plan.of(da)
    n = plan.size
    buf = DeviceBuffer(n + slack + 1)
    try:
        buf.fill(0xC7, dev)
        plan.pack(buf.ptr, n + slack, dev)
        dev.sync()
        got = buf.to_bytes(n + slack + 1)
        covered = bytearray(n + slack + 1)
        for off, ln in _regions(info):
            assert got[off:off + ln] == want[off:off + ln], (name, off, ln)
            covered[off:off + ln] = b"\x01" * ln
        stale = [i for i in range(n + slack + 1) if not covered[i] and got[i] != 0xC7]
        assert not stale, (name, stale[:16])
    finally:
        plan.close(); buf.free(); da.close()
