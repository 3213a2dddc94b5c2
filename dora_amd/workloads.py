"""Synthetic, seeded workloads of BASELINE.json's configs (inputs only — no checking logic).

* C1/C2: UInt8 payloads, splitmix64 bytes with seed 0xD05A + size.
* C3:    List<Struct<x,y,z: f32, intensity: u8>> point clouds: L lists with
         seeded multinomial lengths summing to n_points, one null list, struct validity
         Bernoulli(0.99), x/y/z uniform in [-100, 100), intensity uniform u8.
"""
from __future__ import annotations

import numpy as np

BENCH_SIZES = [4096, 16384, 40960, 65536, 409600, 1 << 20, 4096000, 4 << 20, 16 << 20,
               40960000]
REFERENCE_LADDER = [0, 8, 64, 512, 2048, 4096, 4 * 4096, 10 * 4096, 100 * 4096, 1000 * 4096]
C3_POINTS = 1_000_000
C3_LISTS = 16


def payload_seed(size: int) -> int:
    return 0xD05A + size


def splitmix_bytes(n: int, seed: int) -> bytes:
    g = np.uint64(0x9E3779B97F4A7C15)
    nw = (n + 7) // 8
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + np.arange(1, nw + 1, dtype=np.uint64) * g
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").tobytes()[:n]


def point_cloud(n_points: int = C3_POINTS, n_lists: int = C3_LISTS, seed: int = 3):
    import pyarrow as pa
    rng = np.random.default_rng(seed)
    lens = rng.multinomial(n_points, np.full(n_lists, 1.0 / n_lists))
    offsets = np.zeros(n_lists + 1, dtype=np.int32)
    np.cumsum(lens, out=offsets[1:])
    xyz = rng.uniform(-100.0, 100.0, size=(3, n_points)).astype(np.float32)
    inten = rng.integers(0, 256, n_points, dtype=np.uint8)
    valid = rng.random(n_points) < 0.99
    pts = pa.StructArray.from_arrays(
        [pa.array(xyz[0]), pa.array(xyz[1]), pa.array(xyz[2]), pa.array(inten)],
        names=["x", "y", "z", "intensity"], mask=pa.array(~valid))
    list_mask = np.zeros(n_lists, dtype=bool)
    list_mask[n_lists // 2] = True
    return pa.ListArray.from_arrays(pa.array(offsets), pts, mask=pa.array(list_mask))
