"""Deterministic pyarrow array recipes shared by the golden fixtures and the parity tests."""
from __future__ import annotations

import numpy as np
import pyarrow as pa

from dora_amd.workloads import point_cloud


def _rng(name):
    return np.random.default_rng(sum(map(ord, name)) * 7919)


def kat(name):
    if name == "kat1":
        return pa.array([1, -2, 3, 4], pa.int8())
    if name == "kat2":
        return pa.array([1, -2, 3, 4], pa.int64())
    if name == "kat3":
        return pa.array([1.0, -2.0, 3.0, 4.0], pa.float64())
    if name == "kat4":
        b = pa.array([False, False, True, True])
        c = pa.array([42, 28, 19, 31], pa.int32())
        return pa.StructArray.from_arrays(
            [b, c], fields=[pa.field("b", pa.bool_(), False), pa.field("c", pa.int32(), False)])
    if name == "kat5":
        return pa.ListArray.from_arrays(
            pa.array([0, 3, 6, 8], pa.int32()), pa.array(range(8), pa.int32()),
            type=pa.list_(pa.field("item", pa.int32(), False)))
    if name == "kat6":
        return pa.array([42], pa.uint8())
    if name == "kat7":
        return pa.array([1, 2, 3, 4, 5])
    if name == "kat8":
        return pa.array([1, None, 3], pa.int32())
    if name == "kat9":
        return pa.array(["ab", "c", None], pa.string())
    if name == "kat10":
        return pa.array([1, 2, 3, 4, 5, 6], pa.int16()).slice(2, 3)
    if name == "kat11":
        return pa.array([], pa.int32())
    raise KeyError(name)


def _ints(rng, n, null_p=0.0, dtype=pa.int32()):
    vals = rng.integers(-1000, 1000, n)
    mask = rng.random(n) < null_p if null_p else None
    return pa.array(vals, type=dtype, mask=mask)


def case(name):
    rng = _rng(name)
    if name == "u8_ragged_4099":
        return pa.array(rng.integers(0, 256, 4099, dtype=np.uint8))
    if name == "i32_nulls_1000":
        return _ints(rng, 1000, 0.3)
    if name == "bool_sliced":
        return pa.array(rng.random(300) < 0.5).slice(13, 201)
    if name == "f64_sliced_nulls":
        vals = rng.standard_normal(500)
        return pa.array(vals, mask=rng.random(500) < 0.1).slice(7, 333)
    if name == "utf8_nulls":
        words = ["".join(chr(97 + x) for x in rng.integers(0, 26, rng.integers(0, 9)))
                 for _ in range(200)]
        return pa.array(words, mask=rng.random(200) < 0.2)
    if name == "large_utf8":
        return pa.array(["alpha", "", "gamma", None, "epsilon"] * 7, pa.large_string())
    if name == "binary_sliced":
        return pa.array([bytes(rng.integers(0, 256, k, dtype=np.uint8)) for k in range(40)],
                        pa.binary()).slice(5, 20)
    if name == "fixed_size_binary":
        return pa.array([bytes([i] * 5) for i in range(17)], pa.binary(5))
    if name == "decimal128":
        import decimal
        return pa.array([decimal.Decimal(f"{i}.{i % 100:02d}") for i in range(23)],
                        pa.decimal128(10, 2))
    if name == "timestamp_date_time":
        ts = pa.array(rng.integers(0, 2 ** 40, 31), pa.timestamp("us", tz="UTC"))
        d = pa.array(rng.integers(0, 20000, 31).astype(np.int32), pa.date32())
        t = pa.array(rng.integers(0, 86400, 31).astype(np.int32), pa.time32("s"))
        return pa.StructArray.from_arrays([ts, d, t], names=["ts", "d", "t"])
    if name == "float16":
        return pa.array(rng.standard_normal(77).astype(np.float16))
    if name == "duration_interval":
        du = pa.array(rng.integers(0, 10 ** 9, 9), pa.duration("ns"))
        iv = pa.array([pa.MonthDayNano([i, i + 1, i * 1000]) for i in range(9)],
                      pa.month_day_nano_interval())
        return pa.StructArray.from_arrays([du, iv], names=["du", "iv"])
    if name == "list_i64_nulls":
        offs = np.cumsum([0] + list(rng.integers(0, 6, 50)))
        vals = pa.array(rng.integers(0, 100, int(offs[-1])), pa.int64())
        mask = pa.array(rng.random(50) < 0.2)
        return pa.ListArray.from_arrays(pa.array(offs, pa.int32()), vals, mask=mask)
    if name == "large_list_sliced":
        offs = np.cumsum([0] + list(rng.integers(0, 4, 40)))
        vals = pa.array(rng.standard_normal(int(offs[-1])).astype(np.float32))
        return pa.LargeListArray.from_arrays(pa.array(offs, pa.int64()), vals).slice(3, 30)
    if name == "fixed_size_list":
        vals = pa.array(rng.integers(0, 9, 3 * 25).astype(np.int16))
        return pa.FixedSizeListArray.from_arrays(vals, 3)
    if name == "struct_nulls_sliced":
        a = _ints(rng, 90, 0.1)
        b = pa.array(rng.random(90) < 0.5)
        c = pa.array(["x" * int(k) for k in rng.integers(0, 5, 90)])
        s = pa.StructArray.from_arrays([a, b, c], names=["a", "b", "c"],
                                       mask=pa.array(rng.random(90) < 0.15))
        return s.slice(11, 60)
    if name == "dictionary":
        idx = pa.array(rng.integers(0, 4, 50).astype(np.int16))
        return pa.DictionaryArray.from_arrays(idx, pa.array(["red", "green", "blue", "cyan"]))
    if name == "map":
        return pa.array([[("a", 1), ("b", 2)], [], None, [("c", 3)]],
                        pa.map_(pa.string(), pa.int32()))
    if name == "null_array":
        return pa.nulls(12)
    if name == "run_end_encoded":
        return pa.RunEndEncodedArray.from_arrays(pa.array([3, 5, 9], pa.int32()),
                                                 pa.array([1.5, None, 2.5]))
    if name == "deep_nesting":
        inner = pa.array([[{"p": 1, "q": "x"}], [], [{"p": None, "q": "yy"}, None]] * 5,
                         pa.list_(pa.struct([("p", pa.int8()), ("q", pa.string())])))
        offs = pa.array([0, 2, 2, 7, 15], pa.int32())
        return pa.ListArray.from_arrays(offs, inner)
    if name == "point_cloud_small":
        return point_cloud(n_points=37, n_lists=4, seed=7)
    if name == "point_cloud_medium":
        return point_cloud(n_points=20000, n_lists=16, seed=11)
    raise KeyError(name)


KATS = [f"kat{i}" for i in range(1, 12)]
CASES = ["u8_ragged_4099", "i32_nulls_1000", "bool_sliced", "f64_sliced_nulls", "utf8_nulls",
         "large_utf8", "binary_sliced", "fixed_size_binary", "decimal128",
         "timestamp_date_time", "float16", "duration_interval", "list_i64_nulls",
         "large_list_sliced", "fixed_size_list", "struct_nulls_sliced", "dictionary", "map",
         "null_array", "run_end_encoded", "deep_nesting", "point_cloud_small",
         "point_cloud_medium"]


def build(name):
    return kat(name) if name.startswith("kat") else case(name)
