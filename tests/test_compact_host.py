"""Compacting plans on the CPU (planning only; packing needs the GPU): a slice's compact type
info equals the reference-layout type info of the same values materialised without an offset
(pyarrow.concat_arrays copies a slice into fresh buffers), i.e. offset 0 everywhere and only the
slice's bytes."""
import pyarrow as pa
import pytest

from dora_amd.arrow_utils import Plan
from tests.golden import recipes


def _fresh(arr):
    return pa.concat_arrays([arr])


def _mask_validity(ti, n_bits=None):
    """Drop bits beyond len in validity bitmaps (not part of the logical array)."""
    j = ti.to_json() if hasattr(ti, "to_json") else ti
    def walk(t):
        if t["validity"] is not None:
            b = bytearray(bytes.fromhex(t["validity"]))
            n = t["len"]
            if n % 8:
                b[-1] &= (1 << (n % 8)) - 1
            t["validity"] = bytes(b).hex()
        for c in t["child_data"]:
            walk(c)
    walk(j)
    return j


SLICED = [
    pa.array(range(100), pa.int32()).slice(17, 40),
    pa.array([True, False, True] * 40).slice(5, 77),
    pa.array(["a", "bb", None, "dddd"] * 20).slice(9, 31),
    pa.array([b"xy", b"", b"zzz"] * 30, pa.large_binary()).slice(4, 50),
    pa.array([[1, 2], [], None, [3, 4, 5]] * 10, pa.list_(pa.int64())).slice(3, 21),
    pa.array([{"a": i, "b": str(i)} if i % 7 else None for i in range(60)]).slice(11, 33),
    pa.FixedSizeListArray.from_arrays(pa.array(range(90), pa.int16()), 3).slice(4, 20),
    pa.array([1.5, None, 2.5] * 30).slice(1, 60),
]


@pytest.mark.parametrize("arr", SLICED, ids=[str(a.type) for a in SLICED])
def test_compact_type_info_equals_fresh_copy(arr):
    with Plan.of(arr, compact=True) as p:
        got = _mask_validity(p.type_info())
        size = p.size
    with Plan.of(_fresh(arr)) as p:
        want = _mask_validity(p.type_info())
        want_size = p.size
    assert got == want
    assert size == want_size


@pytest.mark.parametrize("name", [n for n in recipes.KATS + recipes.CASES
                                  if n not in ("run_end_encoded", "kat11")])
def test_compact_never_larger_than_reference(name):
    arr = recipes.build(name)
    with Plan.of(arr, compact=True) as c, Plan.of(arr) as r:
        assert c.size <= r.size
        ti = c.type_info()

    def offsets_zero(t):
        assert t.offset == 0
        for ch in t.child_data:
            offsets_zero(ch)
    offsets_zero(ti)


def test_compact_rejects_run_end_encoded():
    from dora_amd import _lib
    with pytest.raises(_lib.UnsupportedType):
        Plan.of(recipes.build("run_end_encoded"), compact=True)
