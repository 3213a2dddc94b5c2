"""Writes tests/golden/*.json.

Two kinds of fixtures:

* `kats.json` — the reference's own known-answer tests with their expected sample layout written
  out BY HAND from the layout rules (not computed by the oracle), so the oracle can be checked
  against them:
    KAT-1..5  apis/python/operator/src/lib.rs:244-292  (`serialize_deserialize_arrow`)
    KAT-6     libraries/arrow-convert/src/from_impls.rs:188-195 (u8 42 roundtrip)
    KAT-7     examples/pyarrow-test/dataflow.yml:1-16 + node-hub/pyarrow-assert/pyarrow_assert/main.py:55
  The reference tests pin logical roundtrip equality; the byte offsets below follow the
  arrow-data 53.2.0 layout rules restated in SURVEY.md §8c.
* `cases.json` — oracle-generated regression vectors (seeded random nested arrays, sliced arrays,
  nulls, strings, dictionaries, C3-shaped point clouds) that the GPU parity tests replay on a
  box; each entry stores the array recipe, the expected ArrowTypeInfo and the sample bytes.

Run: python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import pyarrow as pa  # noqa: E402

from tests.golden import recipes  # noqa: E402


def le(fmt, vals):
    return b"".join(struct.pack("<" + fmt, v) for v in vals)


def ti(dt, n, bufs, children=(), null_count=0, validity=None, offset=0):
    return {"data_type": dt, "len": n, "null_count": null_count, "validity": validity,
            "offset": offset, "buffer_offsets": [list(b) for b in bufs],
            "child_data": list(children)}


KATS = [
    {"name": "KAT-1 Int8 [1,-2,3,4]", "recipe": "kat1",
     "sample": le("b", [1, -2, 3, 4]).hex(),
     "type_info": ti("c", 4, [(0, 4)])},
    {"name": "KAT-2 Int64 [1,-2,3,4]", "recipe": "kat2",
     "sample": le("q", [1, -2, 3, 4]).hex(),
     "type_info": ti("l", 4, [(0, 32)])},
    {"name": "KAT-3 Float64 [1,-2,3,4]", "recipe": "kat3",
     "sample": le("d", [1.0, -2.0, 3.0, 4.0]).hex(),
     "type_info": ti("g", 4, [(0, 32)])},
    {"name": "KAT-4 Struct{b: Boolean, c: Int32}", "recipe": "kat4",
     # b bitmap 0b1100 @0 (BitMap: no alignment), 3 pad bytes, c @4 (align 4)
     "sample": (b"\x0c" + b"\0" * 3 + le("i", [42, 28, 19, 31])).hex(),
     "type_info": ti("+s[b:!b,c:!i]", 4, [], children=[
         ti("b", 4, [(0, 1)]), ti("i", 4, [(4, 16)])])},
    {"name": "KAT-5 List<Int32> [[0,1,2],[3,4,5],[6,7]]", "recipe": "kat5",
     "sample": (le("i", [0, 3, 6, 8]) + le("i", range(8))).hex(),
     "type_info": ti("+l[item:!i]", 3, [(0, 16)], children=[ti("i", 8, [(16, 32)])])},
    {"name": "KAT-6 UInt8 [42]", "recipe": "kat6",
     "sample": "2a", "type_info": ti("C", 1, [(0, 1)])},
    {"name": "KAT-7 pyarrow [1,2,3,4,5]", "recipe": "kat7",
     "sample": le("q", [1, 2, 3, 4, 5]).hex(), "type_info": ti("l", 5, [(0, 40)])},
    {"name": "KAT-8 Int32 with a null [1,None,3] (hand-derived)", "recipe": "kat8",
     "sample": le("i", [1, 0, 3]).hex(),
     "type_info": ti("i", 3, [(0, 12)], null_count=1, validity="05")},
    {"name": "KAT-9 Utf8 ['ab','c',None] (hand-derived)", "recipe": "kat9",
     "sample": (le("i", [0, 2, 3, 3]) + b"abc").hex(),
     "type_info": ti("u", 3, [(0, 16), (16, 3)], null_count=1, validity="03")},
    {"name": "KAT-10 Int16 [1..6] sliced [2:5] (offset passes through, whole prefix copied)",
     "recipe": "kat10",
     # arrow-rs FFI import: buffer len = (len+offset)*2 = 10 bytes; offset 2 kept in type info
     "sample": le("h", [1, 2, 3, 4, 5]).hex(),
     "type_info": ti("s", 3, [(0, 10)], offset=2)},
    {"name": "KAT-11 empty Int32 [] -> empty sample", "recipe": "kat11",
     "sample": "", "type_info": ti("i", 0, [(0, 0)])},
]


def main():
    from oracle.pack_ref import pack  # the oracle is only used for cases.json
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(KATS, f, indent=1)
    cases = []
    from oracle.checksum_ref import csum64
    for name in recipes.CASES:
        arr = recipes.build(name)
        sample, info = pack(arr)
        entry = {"name": name, "recipe": name, "sample_len": len(sample),
                 "sample_csum64": csum64(sample), "type_info": info.to_json()}
        if len(sample) <= 8192:
            entry["sample"] = sample.hex()
        if len(sample) > 8192:   # keep big fixtures small: checksums only
            entry["type_info_csum64"] = csum64(json.dumps(info.to_json()).encode())
            entry["type_info"] = None
        cases.append(entry)
    with open(os.path.join(HERE, "cases.json"), "w") as f:
        json.dump(cases, f, indent=0)
    print(f"wrote {len(KATS)} KATs and {len(cases)} cases")


if __name__ == "__main__":
    main()
